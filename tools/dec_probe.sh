#!/bin/bash
# fqz decoder: GPU tests, then the probe build's cycle split (inside the run
# loop / per miss / between runs) on ONT and HiFi strategies.
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fqz_gpu.py > gpurun_out/fqz_t.log 2>&1 || exit 1
FQZ5_DEBUG=1 FQZ5_LIB_VARIANT=tools/vbuild/libfqz5_probe.so timeout -k 10 300 python -u tools/fqz_dec_bench.py 4 ${1:-novaseq,ont,hifi} ${2:-0,1,2,3} > gpurun_out/probe2.log 2>&1
