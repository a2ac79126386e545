#!/bin/bash
# refinement session reused by the commit: the bounded tests (with the
# widened intervals that leave every decision open), then the -7 step
set -uo pipefail
OUT=gpurun_out/r03/merge
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 400 --timeout-method thread -m gpu \
    tests/test_sections_gpu.py -k bounded > $OUT/tests.log 2>&1
rc=$?; grep -E "intervals decided|passed|failed|Error" $OUT/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --no-cpu --no-level5 --no-crc --no-dropin \
    --level 7 --kind ont --gb 1.5 --steps 1 --warmup 0 > $OUT/b7.json 2> $OUT/b7.log
echo "l7 rc=$?"; grep "bench\]\|sections\]\|Error" $OUT/b7.log
