#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02z
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rans_gpu.py tests/test_dropin_gpu.py tests/test_fqz_gpu.py > gpurun_out/r02z/t.log 2>&1 || { tail -30 gpurun_out/r02z/t.log; exit 1; }
tail -2 gpurun_out/r02z/t.log
