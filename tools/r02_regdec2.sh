#!/bin/bash
# Min-based register O0 decoder: rANS parity, then -3 A/B against the LDS
# decoder, then the -5 item.
set -euo pipefail
OUT=gpurun_out/regdec2
mkdir -p $OUT
export TMPDIR=/tmp
B3="--no-cpu --no-level5 --no-crc --no-dropin"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_rans_gpu.py tests/test_dropin_gpu.py > $OUT/tests.log 2>&1
timeout -k 10 300 python3 bench.py $B3 --steps 8 --warmup 2 > $OUT/b_default.json 2> $OUT/b_default.log
FQZ5_NO_REGDEC=1 timeout -k 10 300 python3 bench.py $B3 --steps 8 --warmup 2 > $OUT/b_noreg.json 2> $OUT/b_noreg.log
timeout -k 10 600 python3 bench.py --no-cpu --no-crc --no-dropin --level 5 --kind novaseq --gb 4 \
    --steps 5 --warmup 2 > $OUT/b5.json 2> $OUT/b5.log
echo done
