#!/bin/bash
# FASTA path and the file/drop-in suites on the GPU box
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fasta
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_fqz5file_gpu.py tests/test_dropin_gpu.py tests/test_capi.py > gpurun_out/fasta/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/fasta/tests.log | tail -15
exit $rc
