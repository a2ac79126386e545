#!/bin/bash
# A/B of two probe builds of the fqz decoder on the same box:
#   tools/r03_ab_probe.sh <variantA.so> <variantB.so> [kinds] [strats]
set -o pipefail
for v in "$1" "$2" "$1" "$2"; do
  echo "== $v" >> gpurun_out/ab.log
  FQZ5_DEBUG=1 FQZ5_LIB_VARIANT=$v timeout -k 10 200 python -u tools/fqz_dec_bench.py 4 ${3:-novaseq,hifi} ${4:-1} >> gpurun_out/ab.log 2>&1 || exit 1
done
