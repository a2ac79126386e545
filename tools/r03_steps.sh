#!/bin/bash
# one step each: -7 ONT (500 MB blocks), -5 on configs[1]'s Illumina data
# (FQZ1 decode), -9 HiFi
set -uo pipefail
OUT=gpurun_out/r03/steps
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --no-cpu --no-level5 --no-crc --no-dropin \
    --level 7 --kind ont --gb 1.5 --steps 1 --warmup 0 > $OUT/b7.json 2> $OUT/b7.log
rc=$?; echo "l7 rc=$rc"; grep "bench\]" $OUT/b7.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu --no-level5 --no-crc --no-dropin \
    --level 5 --kind illumina --gb 1 --steps 1 --warmup 0 > $OUT/b5i.json 2> $OUT/b5i.log
rc=$?; echo "l5i rc=$rc"; grep "bench\]" $OUT/b5i.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu --no-level5 --no-crc --no-dropin \
    --level 9 --kind hifi --gb 0.15 --steps 1 --warmup 0 > $OUT/b9.json 2> $OUT/b9.log
echo "l9 rc=$?"; grep "bench\]" $OUT/b9.log
