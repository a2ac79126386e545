#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02n
timeout -k 10 300 python -u tools/names_timing.py 3 > gpurun_out/r02n/t3.log 2>&1 || { tail -40 gpurun_out/r02n/t3.log; exit 1; }
grep -v "^$" gpurun_out/r02n/t3.log | tail -40
