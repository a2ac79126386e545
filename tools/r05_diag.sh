#!/bin/bash
# Round-5 diagnostics on the GPU box: the -5 NovaSeq encode step's phases
# (FQZ5_STEP_TRACE: try / commit / per-family timings on stderr), then the
# rocprofv3 kernel-trace summaries of the three bench items (tools/profile.sh
# phase a without its bench run).  Outputs under gpurun_out/diag_<tag>.
# $PHASES picks the parts (default all): trace5 trace3 trace5i kt3 kt5 kt5i.
set -euo pipefail
TAG=${1:-r05}
PHASES=${PHASES:-"trace5 trace3 trace5i kt3 kt5 kt5i"}
OUT=gpurun_out/diag_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B3="--no-cpu --no-level5 --no-crc --no-dropin"
B5="--no-cpu --no-crc --no-dropin --level 5 --kind novaseq --gb 4"
B5I="--no-cpu --no-crc --no-dropin --no-level5 --level 5 --kind illumina"
has() { [[ " $PHASES " == *" $1 "* ]]; }
if has trace5; then
    FQZ5_STEP_TRACE=1 FQZ5_FQZ_SEGSTATS=1 timeout -k 10 300 python3 bench.py $B5 --steps 2 --warmup 1 \
        > $OUT/trace5.json 2> $OUT/trace5.log
fi
if has trace3; then
    FQZ5_STEP_TRACE=1 timeout -k 10 300 python3 bench.py $B3 --steps 3 --warmup 1 \
        > $OUT/trace3.json 2> $OUT/trace3.log
fi
if has trace5i; then
    FQZ5_STEP_TRACE=1 timeout -k 10 300 python3 bench.py $B5I --steps 2 --warmup 1 \
        > $OUT/trace5i.json 2> $OUT/trace5i.log
fi
if has kt3; then
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt3 -o kt -- \
        python3 bench.py $B3 --steps 5 --warmup 1 > $OUT/kt3.log 2>&1
fi
if has kt5; then
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt5 -o kt -- \
        python3 bench.py $B5 --steps 5 --warmup 1 > $OUT/kt5.log 2>&1
fi
if has kt5i; then
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt5i -o kt -- \
        python3 bench.py $B5I --steps 2 --warmup 1 > $OUT/kt5i.log 2>&1
fi
echo done
