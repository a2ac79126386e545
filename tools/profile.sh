#!/bin/bash
# Round profile on the GPU box: the driver's bench command, the rocprofv3
# kernel-trace summaries of the same workloads (configs[1] -3, configs[2]
# -5, and -5 on configs[1]'s Illumina, where FQZ1 codes the qualities), and
# the HBM traffic PMC passes of each (FETCH_SIZE and WRITE_SIZE each in a
# pass of its own; MI355X_MICROARCH.md HBM section).
# Usage: tools/profile.sh <tag> [a|b|all]   (outputs under gpurun_out/prof_<tag>;
# phase a = bench + kernel traces, b = PMC passes, so each fits one gpurun call)
set -euo pipefail
TAG=${1:-r02}
PHASE=${2:-all}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B3="--no-cpu --no-level5 --no-crc --no-dropin"
B5="--no-cpu --no-crc --no-dropin --level 5 --kind novaseq --gb 4"
B5I="--no-cpu --no-crc --no-dropin --no-level5 --level 5 --kind illumina"
if [ "$PHASE" != b ]; then
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt3 -o kt -- \
    python3 bench.py $B3 --steps 5 --warmup 1 > $OUT/kt3.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt5 -o kt -- \
    python3 bench.py $B5 --steps 5 --warmup 1 > $OUT/kt5.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt5i -o kt -- \
    python3 bench.py $B5I --steps 2 --warmup 1 > $OUT/kt5i.log 2>&1
fi
[ "$PHASE" = a ] && { echo done; exit 0; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- \
    python3 bench.py $B3 --steps 1 --warmup 0 > $OUT/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- \
    python3 bench.py $B3 --steps 1 --warmup 0 > $OUT/write.log 2>&1
python3 tools/pmc_summary.py $OUT $OUT/pmc.json > /dev/null
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/l5/fetch -o fetch -- \
    python3 bench.py $B5 --steps 1 --warmup 0 > $OUT/fetch5.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/l5/write -o write -- \
    python3 bench.py $B5 --steps 1 --warmup 0 > $OUT/write5.log 2>&1
python3 tools/pmc_summary.py $OUT/l5 $OUT/pmc_l5.json > /dev/null
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/l5i/fetch -o fetch -- \
    python3 bench.py $B5I --steps 1 --warmup 0 > $OUT/fetch5i.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/l5i/write -o write -- \
    python3 bench.py $B5I --steps 1 --warmup 0 > $OUT/write5i.log 2>&1
python3 tools/pmc_summary.py $OUT/l5i $OUT/pmc_l5i.json "the fqz quality chains decode on host cores by the default placement (fqz5_set_host_decode(2))" > /dev/null
echo done
