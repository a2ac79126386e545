#!/bin/bash
# round-2 first GPU pass: the GPU suite, then the driver's bench command
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02a
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r02a/tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 900 python -u bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r02a/bench.json 2> gpurun_out/r02a/bench.err
echo "bench rc=$?"
tail -c 3000 gpurun_out/r02a/bench.json
