#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02f
timeout -k 10 300 python -u tools/step_timing.py 3 > gpurun_out/r02f/a.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/step_timing.py 3 prof > gpurun_out/r02f/b.log 2>&1 || exit $?
tail -3 gpurun_out/r02f/a.log; tail -3 gpurun_out/r02f/b.log
