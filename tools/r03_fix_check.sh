#!/bin/bash
# the file-path and fqz tests after the serial-path bound fix, then the -7 step
set -uo pipefail
OUT=gpurun_out/r03/fix
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_fqz5file_gpu.py tests/test_fqz_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --no-cpu --no-level5 --no-crc --no-dropin \
    --level 7 --kind ont --gb 1.5 --steps 1 --warmup 0 > $OUT/b7.json 2> $OUT/b7.log
echo "l7 rc=$?"; grep "bench\]\|sections\]\|Error" $OUT/b7.log
