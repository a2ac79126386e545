#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02n
timeout -k 10 300 python -u tools/dec_jobs_probe.py 5 > gpurun_out/r02n/j5.log 2>&1 || { tail gpurun_out/r02n/j5.log; exit 1; }
cat gpurun_out/r02n/j5.log
