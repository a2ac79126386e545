#!/bin/bash
# round-2 GPU pass 2: LZP / sections / trial-parity tests, then the bench
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02b
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
    tests/test_lzp_gpu.py tests/test_sections_gpu.py tests/test_trial_parity_gpu.py > gpurun_out/r02b/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -15 gpurun_out/r02b/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -u bench.py --gpus 1 --steps 5 --warmup 2 --no-dropin --no-crc > gpurun_out/r02b/bench.json 2> gpurun_out/r02b/bench.err
rc=$?
echo "bench rc=$rc"
tail -c 2500 gpurun_out/r02b/bench.json
exit $rc
