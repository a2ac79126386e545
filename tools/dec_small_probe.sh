#!/bin/bash
# k_fqz_dec_small: plain-build ns per symbol (tools/fqz_dec_bench.py), then
# the stamped build's cycle split (tools/dec_small_probe_run.py).  Outputs
# under gpurun_out/dec_small_probe.
set -euo pipefail
OUT=gpurun_out/dec_small_probe
mkdir -p $OUT
FQZ5_DEBUG=1 timeout -k 10 300 python3 -u tools/fqz_dec_bench.py 4 novaseq,illumina8 0,1,2 > $OUT/plain.txt 2>&1
FQZ5_LIB_VARIANT=tools/vbuild/libfqz5_sprobe.so timeout -k 10 300 python3 -u tools/dec_small_probe_run.py 4 > $OUT/probe.txt 2>&1
echo done
