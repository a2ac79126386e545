#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02c
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
    tests/test_lzp_gpu.py tests/test_sections_gpu.py tests/test_trial_parity_gpu.py > gpurun_out/r02c/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -8 gpurun_out/r02c/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
FQZ5_STEP_TRACE=1 timeout -k 10 300 python -u tools/step_timing.py 3 > gpurun_out/r02c/st3.log 2>&1 || exit $?
FQZ5_STEP_TRACE=1 timeout -k 10 300 python -u tools/step_timing.py 5 > gpurun_out/r02c/st5.log 2>&1 || exit $?
tail -12 gpurun_out/r02c/st3.log; tail -12 gpurun_out/r02c/st5.log
