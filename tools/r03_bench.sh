#!/bin/bash
# The driver's default bench command (N=1), output under gpurun_out/r03/bench
set -uo pipefail
OUT=gpurun_out/r03/bench
mkdir -p $OUT
timeout -k 10 1100 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.log
echo "rc=$?"
