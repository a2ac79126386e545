#!/bin/bash
# -7 ONT step with the interval trial (which decisions stay open, the
# exact refinement), then the bounded-path GPU tests
set -uo pipefail
OUT=gpurun_out/r03/why
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --no-cpu --no-level5 --no-crc --no-dropin \
    --level 7 --kind ont --gb 1.5 --steps 1 --warmup 0 > $OUT/b7.json 2> $OUT/b7.log
rc=$?; echo "rc=$rc"; grep "bench\]\|sections\]\|Error" $OUT/b7.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_sections_gpu.py -k bounded > $OUT/tests.log 2>&1
echo "tests rc=$?"; tail -2 $OUT/tests.log
