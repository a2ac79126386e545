#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02f
timeout -k 10 800 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_fqz5file_gpu.py > gpurun_out/r02f/t.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/r02f/t.log | head -60; tail -30 gpurun_out/r02f/t.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r02f/t.log | tail -20; tail -2 gpurun_out/r02f/t.log
