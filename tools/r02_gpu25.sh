#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02t
timeout -k 10 700 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_dropin_gpu.py > gpurun_out/r02t/d.log 2>&1 || { tail -60 gpurun_out/r02t/d.log; exit 1; }
tail -12 gpurun_out/r02t/d.log
