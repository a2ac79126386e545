#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02j
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_rans_gpu.py tests/test_sections_gpu.py tests/test_dropin_gpu.py > gpurun_out/r02j/t.log 2>&1 || { tail -30 gpurun_out/r02j/t.log; exit 1; }
tail -2 gpurun_out/r02j/t.log
timeout -k 10 300 python -u tools/step_timing.py 3 > gpurun_out/r02j/st3.log 2>&1 || exit $?
tail -3 gpurun_out/r02j/st3.log
timeout -k 10 300 python -u tools/step_timing.py 5 > gpurun_out/r02j/st5.log 2>&1 || exit $?
tail -3 gpurun_out/r02j/st5.log
