#!/bin/bash
# -5 decode: this tree's library against the same library with the decode
# kernel file of the round-2 profile commit (0ac8a94), both without the XCD
# layout (the old kernel has no padding-job exit), alternating, same box.
set -uo pipefail
OUT=gpurun_out/ab5f
mkdir -p $OUT
export TMPDIR=/tmp
B5="--no-cpu --no-crc --no-dropin --level 5 --kind novaseq --gb 4 --steps 4 --warmup 1"
for v in cur gap cur gap; do
  if [ $v = gap ]; then export FQZ5_BENCH_GAP_S=0.5; else unset FQZ5_BENCH_GAP_S; fi
  timeout -k 10 300 python3 bench.py $B5 > $OUT/b5$v.json 2> $OUT/b5$v.log || { echo "b5 $v failed"; tail -5 $OUT/b5$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b5$v.json'));print('$v',d['value'],d['enc_ms_per_step'],d['dec_ms_per_step'],d['roofline']['dec_avg_ms'])"
done
