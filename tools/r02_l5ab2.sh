#!/bin/bash
# -5 decode regression hunt 2: default vs 24 hardware queues vs the kernel
# without the register-decoder instantiations (code size).
set -euo pipefail
OUT=gpurun_out/l5ab2
mkdir -p $OUT
export TMPDIR=/tmp
B5="--no-cpu --no-crc --no-dropin --level 5 --kind novaseq --gb 4 --steps 4 --warmup 1"
FQZ5_HW_QUEUES=24 timeout -k 10 400 python3 bench.py $B5 > $OUT/q24.json 2> $OUT/q24.log
FQZ5_LIB_VARIANT=$PWD/tools/variants/libfqz5_noregk.so timeout -k 10 400 python3 bench.py $B5 > $OUT/noregk.json 2> $OUT/noregk.log
timeout -k 10 400 python3 bench.py $B5 > $OUT/def.json 2> $OUT/def.log
echo done
