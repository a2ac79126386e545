#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02n
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02n/prof -o run -- python3 tools/names_timing.py 3 > gpurun_out/r02n/p3.log 2>&1 || { tail -30 gpurun_out/r02n/p3.log; exit 1; }
f=$(find gpurun_out/r02n/prof -name "*kernel_stats.csv" | head -1)
head -25 "$f" | cut -d, -f1-8
