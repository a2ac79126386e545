#!/bin/bash
# -5 decode regression hunt: default vs FQZ5_NO_XCD_GROUP vs FQZ5_NO_REGDEC.
set -euo pipefail
OUT=gpurun_out/l5ab
mkdir -p $OUT
export TMPDIR=/tmp
B5="--no-cpu --no-crc --no-dropin --level 5 --kind novaseq --gb 4 --steps 4 --warmup 1"
timeout -k 10 400 python3 bench.py $B5 > $OUT/def.json 2> $OUT/def.log
FQZ5_NO_XCD_GROUP=1 timeout -k 10 400 python3 bench.py $B5 > $OUT/noxcd.json 2> $OUT/noxcd.log
FQZ5_NO_REGDEC=1 timeout -k 10 400 python3 bench.py $B5 > $OUT/noreg.json 2> $OUT/noreg.log
echo done
