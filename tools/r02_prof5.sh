#!/bin/bash
# kernel-time breakdown of the -5 and -3 bench steps (step_timing.py, 3 reps)
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02d
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02d/k5 -o kt -- \
    python3 tools/step_timing.py 5 > gpurun_out/r02d/k5.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02d/k3 -o kt -- \
    python3 tools/step_timing.py 3 > gpurun_out/r02d/k3.log 2>&1 || exit $?
find gpurun_out/r02d -name "*kernel_stats.csv" | head
