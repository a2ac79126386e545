#!/bin/bash
# sequence-model decoder: GPU tests, then timing (tools/seq_timing.py)
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_seq_gpu.py > gpurun_out/r03/seq_t.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/seq_timing.py 8 > gpurun_out/r03/seq_timing.log 2>&1
