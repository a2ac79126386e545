#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02l
FQZ5_LIB_VARIANT=$PWD/tools/probe/libfqz5_cprobe.so timeout -k 10 200 python -u tools/enc_probe_run.py 2>&1 | tee gpurun_out/r02l/enc_probe.log
