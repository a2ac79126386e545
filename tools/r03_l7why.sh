#!/bin/bash
# -7 ONT step: which trial decision the size intervals leave open
set -uo pipefail
OUT=gpurun_out/r03/why
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --no-cpu --no-level5 --no-crc --no-dropin \
    --level 7 --kind ont --gb 1.5 --steps 1 --warmup 0 > $OUT/b7.json 2> $OUT/b7.log
echo "rc=$?"; grep "bench\]\|sections\]" $OUT/b7.log
