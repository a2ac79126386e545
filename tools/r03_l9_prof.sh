#!/bin/bash
# kernel-trace summary of the -9 HiFi single-block step (round 3)
set -uo pipefail
OUT=gpurun_out/r03/l9p
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
    python3 -u bench.py --no-cpu --no-level5 --no-crc --no-dropin --level 9 --kind hifi \
    --gb 0.05 --steps 1 --warmup 0 > $OUT/b9.json 2> $OUT/b9.log
rc=$?; echo "rc=$rc"; grep "\[bench\]" $OUT/b9.log | tail -3
f=$(find $OUT/kt -name "*kernel_stats.csv" | head -1); echo "$f"; head -12 "$f" | cut -c1-200
exit $rc
