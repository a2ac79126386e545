#!/bin/bash
# -5 Illumina encode with the fqz hot-model threshold at its default and
# lower (FQZ5_HOT_MIN); outputs under gpurun_out/hotmin.
set -euo pipefail
OUT=gpurun_out/hotmin
mkdir -p $OUT
B5I="--no-cpu --no-crc --no-dropin --no-level5 --level 5 --kind illumina --steps 3 --warmup 1"
for h in default 4096 1024; do
  if [ $h = default ]; then
    FQZ5_STEP_TRACE=1 timeout -k 10 300 python3 bench.py $B5I > $OUT/b5i_$h.json 2> $OUT/b5i_$h.log
  else
    FQZ5_HOT_MIN=$h FQZ5_STEP_TRACE=1 timeout -k 10 300 python3 bench.py $B5I > $OUT/b5i_$h.json 2> $OUT/b5i_$h.log
  fi
done
echo done
