#!/bin/bash
# kernel statistics of the -7 ONT step (500 MB blocks, 1.5 GB): where the
# try chunks' time goes
set -uo pipefail
OUT=gpurun_out/r03/l7p
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o l7 -- \
    python3 -u $GRAFT_REPO_ROOT/bench.py --no-cpu --no-level5 --no-crc --no-dropin \
    --level 7 --kind ont --gb 1.5 --steps 1 --warmup 0 > $GRAFT_REPO_ROOT/$OUT/b7.json 2> $GRAFT_REPO_ROOT/$OUT/b7.log
echo "rc=$?"; find $GRAFT_REPO_ROOT/$OUT/prof -name "*stats*" | head
