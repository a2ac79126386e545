#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02b
timeout -k 10 1000 python -u bench.py > gpurun_out/r02b/bench.json 2> gpurun_out/r02b/bench.log || { tail -40 gpurun_out/r02b/bench.log; exit 1; }
tail -c 3000 gpurun_out/r02b/bench.json
