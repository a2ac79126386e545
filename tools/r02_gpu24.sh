#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02t
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_tok3_gpu.py > gpurun_out/r02t/t.log 2>&1 || { tail -60 gpurun_out/r02t/t.log; exit 1; }
tail -3 gpurun_out/r02t/t.log
