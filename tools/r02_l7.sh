#!/bin/bash
# The bounded trial (encode_run_bounded) against encode_run, then configs[3]
# shape at the -7 preset's 500 MB blocks on one GPU.
set -uo pipefail
OUT=gpurun_out/l7
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_sections_gpu.py -k bounded > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python3 -u bench.py --no-cpu --no-level5 --no-crc --no-dropin --level 7 --kind ont \
    --gb 1.5 --steps 1 --warmup 0 > $OUT/b7.json 2> $OUT/b7.log
echo "rc=$?"; tail -5 $OUT/b7.log; head -c 1500 $OUT/b7.json
