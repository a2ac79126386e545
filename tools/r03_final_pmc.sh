#!/bin/bash
# HBM traffic of the -5 Illumina step (hedged k_fqz_dec): FETCH_SIZE and
# WRITE_SIZE passes of their own
set -uo pipefail
OUT=gpurun_out/r03/final
mkdir -p $OUT
export TMPDIR=/tmp
B5I="--no-cpu --no-crc --no-dropin --no-level5 --level 5 --kind illumina --gb 1"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/l5i/fetch -o fetch -- \
    python3 bench.py $B5I --steps 1 --warmup 0 > $OUT/fetch5i.log 2>&1
echo "fetch rc=$?"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/l5i/write -o write -- \
    python3 bench.py $B5I --steps 1 --warmup 0 > $OUT/write5i.log 2>&1
echo "write rc=$?"
python3 tools/pmc_summary.py $OUT/l5i $OUT/pmc_l5i.json > /dev/null; echo "summary rc=$?"
