#!/bin/bash
# round-2 first GPU pass: the GPU suite, then the bench
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02a
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r02a/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/r02a/tests.log
# 0 = passed, 1 = a test failed: anything else (timeout, abort, fault) ends the call
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -u bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r02a/bench.json 2> gpurun_out/r02a/bench.err
rc=$?
echo "bench rc=$rc"
tail -c 4000 gpurun_out/r02a/bench.json
exit $rc
