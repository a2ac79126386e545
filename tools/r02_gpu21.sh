#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02w
timeout -k 10 300 python -u tools/dec_jobs_probe.py 3 > gpurun_out/r02w/j3.log 2>&1 || { tail gpurun_out/r02w/j3.log; exit 1; }
head -3 gpurun_out/r02w/j3.log; tail -12 gpurun_out/r02w/j3.log
