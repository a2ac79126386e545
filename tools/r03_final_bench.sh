#!/bin/bash
# the driver's bench command on the final tree, then the -5 Illumina
# (FQZ1, hedged decode) kernel statistics and HBM traffic passes
set -uo pipefail
OUT=gpurun_out/r03/final
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 800 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.log
rc=$?; echo "bench rc=$rc"; grep "bench\]" $OUT/bench.log | tail -4; [ $rc -eq 0 ] || exit $rc
B5I="--no-cpu --no-crc --no-dropin --no-level5 --level 5 --kind illumina --gb 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt5i -o kt -- \
    python3 bench.py $B5I --steps 1 --warmup 0 > $OUT/kt5i.log 2>&1
echo "kt5i rc=$?"
