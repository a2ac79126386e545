#!/bin/bash
# configs[4] shape (PacBio HiFi, -9 preset: full trial, 1 GB block size) at a
# reduced size on one GPU, one step (the fqz / sequence-model decode chains
# bound it)
set -uo pipefail
OUT=gpurun_out/r03/l9
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u bench.py --no-cpu --no-level5 --no-crc --no-dropin --level 9 --kind hifi \
    --gb 0.15 --steps 1 --warmup 0 > $OUT/b9.json 2> $OUT/b9.log
echo "rc=$?"; tail -5 $OUT/b9.log; head -c 1500 $OUT/b9.json
