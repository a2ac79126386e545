#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02n
timeout -k 10 900 python -u -m pytest -q -x --timeout 400 --timeout-method thread -m gpu tests/test_tok3_gpu.py tests/test_trial_parity_gpu.py tests/test_fqz5file_gpu.py tests/test_dropin_gpu.py > gpurun_out/r02n/t.log 2>&1 || { tail -40 gpurun_out/r02n/t.log; exit 1; }
tail -2 gpurun_out/r02n/t.log
timeout -k 10 300 python -u tools/names_timing.py 3 > gpurun_out/r02n/t3.log 2>&1 || { tail -40 gpurun_out/r02n/t3.log; exit 1; }
grep -E "names encode|encode_run|sections_try: [0-9]|rANS candidates" gpurun_out/r02n/t3.log | tail -4
