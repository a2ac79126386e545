#!/bin/bash
# Register O0 decoder + XCD-grouped hedged copies: parity (rANS tests, the
# section/block tests), then -3 bench A/B (default, FQZ5_NO_REGDEC,
# FQZ5_NO_XCD_GROUP), then FETCH_SIZE passes of the decode with and without
# the XCD grouping.
set -euo pipefail
OUT=gpurun_out/regdec
mkdir -p $OUT
export TMPDIR=/tmp
B3="--no-cpu --no-level5 --no-crc --no-dropin"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_rans_gpu.py tests/test_trial_parity_gpu.py tests/test_sections_gpu.py \
    tests/test_tok3_gpu.py > $OUT/tests.log 2>&1
timeout -k 10 300 env FQZ5_STEP_TRACE=1 python3 -u tools/names_timing.py 3 > $OUT/t3.log 2>&1
timeout -k 10 300 python3 bench.py $B3 --steps 5 --warmup 2 > $OUT/b_default.json 2> $OUT/b_default.log
FQZ5_NO_REGDEC=1 timeout -k 10 300 python3 bench.py $B3 --steps 5 --warmup 2 > $OUT/b_noreg.json 2> $OUT/b_noreg.log
FQZ5_NO_XCD_GROUP=1 timeout -k 10 300 python3 bench.py $B3 --steps 5 --warmup 2 > $OUT/b_noxcd.json 2> $OUT/b_noxcd.log
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fx -o f -- \
    python3 bench.py $B3 --steps 1 --warmup 0 > $OUT/fx.log 2>&1
export FQZ5_NO_XCD_GROUP=1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fn -o f -- \
    python3 bench.py $B3 --steps 1 --warmup 0 > $OUT/fn.log 2>&1
echo done
