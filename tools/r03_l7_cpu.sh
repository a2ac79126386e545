#!/bin/bash
# configs[3] shape (ONT, -7 preset: 500 MB blocks) on one GPU with the
# reference CLI (-7 -t16) on the same text as cpu_baseline
set -uo pipefail
OUT=gpurun_out/r03/l7
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1100 python3 -u bench.py --no-level5 --no-crc --no-dropin --level 7 --kind ont \
    --gb 1.5 --steps 1 --warmup 0 > $OUT/b7.json 2> $OUT/b7.log
echo "rc=$?"; tail -5 $OUT/b7.log; head -c 3000 $OUT/b7.json
