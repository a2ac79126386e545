#!/bin/bash
# microbenchmarks of chain-step pieces + the -3 bench item with per-step times
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02e
timeout -k 10 60 ./tools/probe/ub2 > gpurun_out/r02e/ub2.log 2>&1 || exit $?
cat gpurun_out/r02e/ub2.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-level5 --no-crc --no-dropin --no-cpu > gpurun_out/r02e/b3.json 2> gpurun_out/r02e/b3.log || exit $?
grep "step:" gpurun_out/r02e/b3.log | head -30
cut -c1-900 gpurun_out/r02e/b3.json
