#!/bin/bash
# -7 ONT encode with the step trace (where the 70 s go), -9 HiFi with the
# reference CLI beside it, then the N = 2 bench path rehearsed on one GPU
# (two ranks sharing the device, gloo exchange)
set -uo pipefail
OUT=gpurun_out/r03/ev
mkdir -p $OUT
export TMPDIR=/tmp
FQZ5_STEP_TRACE=1 timeout -k 10 400 python3 -u bench.py --no-cpu --no-level5 --no-crc --no-dropin \
    --level 7 --kind ont --gb 1.5 --steps 1 --warmup 0 > $OUT/b7t.json 2> $OUT/b7t.log
rc=$?; echo "l7 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --no-level5 --no-crc --no-dropin --level 9 --kind hifi \
    --gb 0.15 --steps 1 --warmup 0 > $OUT/b9.json 2> $OUT/b9.log
rc=$?; echo "l9 rc=$rc"; [ $rc -eq 0 ] || exit $rc
FQZ5_BENCH_SHARE_GPU=1 timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 \
    --no-level5 --no-cpu --no-dropin --no-crc > $OUT/n2.json 2> $OUT/n2.log
rc=$?; echo "n2 rc=$rc"; tail -3 $OUT/n2.log; cat $OUT/n2.json | head -c 1500
