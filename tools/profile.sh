#!/bin/bash
# Round profile on the GPU box: the bench line, the rocprofv3 kernel-trace
# summary of the same command, and the HBM traffic PMC passes (FETCH_SIZE
# and WRITE_SIZE cannot share a pass on gfx950; MI355X_MICROARCH.md).
# Usage: tools/profile.sh <tag>   (outputs under gpurun_out/prof_<tag>)
set -euo pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
    python3 bench.py --no-cpu > $OUT/kt.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- \
    python3 bench.py --no-cpu --steps 1 --warmup 0 > $OUT/fetch.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- \
    python3 bench.py --no-cpu --steps 1 --warmup 0 > $OUT/write.log 2>&1
echo done
