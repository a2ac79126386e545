#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02t
timeout -k 10 900 python -u -m pytest -v -x --timeout 600 --timeout-method thread -m gpu tests/test_trial_parity_gpu.py tests/test_tok3_gpu.py tests/test_lzp_gpu.py > gpurun_out/r02t/p.log 2>&1 || { tail -80 gpurun_out/r02t/p.log; exit 1; }
tail -15 gpurun_out/r02t/p.log
