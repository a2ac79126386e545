#!/bin/bash
# Where the drop-in CLI's time goes (-3 -t16 on the 1 GB bench FASTQ):
# wall times, the library's step trace, and a kernel trace of the decode.
set -euo pipefail
OUT=gpurun_out/dropin
mkdir -p $OUT
export TMPDIR=/tmp
CPU=oracle/_ref/fqzcomp5
GPU=oracle/_ref/fqzcomp5_gpu
python3 -c "import sys; sys.path.insert(0, '.'); import bench; from fqzcomp5_amd import synth; synth.write_fastq(bench.make_reads(1.0, 1, 'illumina'), '/tmp/w.fastq')"
head -c 100000 /tmp/w.fastq | head -n 400 > /tmp/tiny.fastq
t() { local a=$(date +%s%N); "$@"; local b=$(date +%s%N); echo "$(( (b - a) / 1000000 )) ms: $*" >> $OUT/times.txt; }
t timeout -k 10 120 $CPU -3 -t16 /tmp/w.fastq /tmp/c.fqz5
t timeout -k 10 120 $CPU -d -t16 /tmp/c.fqz5 /tmp/c.fq
t timeout -k 10 60 $GPU -3 -t1 /tmp/tiny.fastq /tmp/tiny.fqz5
t timeout -k 10 60 $GPU -d -t1 /tmp/tiny.fqz5 /tmp/tiny.out
t timeout -k 10 120 $GPU -3 -t16 /tmp/w.fastq /tmp/g.fqz5
t timeout -k 10 120 $GPU -d -t16 /tmp/c.fqz5 /tmp/g.fq
FQZ5_STEP_TRACE=1 t timeout -k 10 120 $GPU -d -t16 /tmp/c.fqz5 /tmp/g.fq 2> $OUT/dec_trace.txt
FQZ5_STEP_TRACE=1 t timeout -k 10 120 $GPU -3 -t16 /tmp/w.fastq /tmp/g.fqz5 2> $OUT/enc_trace.txt
t timeout -k 10 200 $GPU -d -t1 /tmp/c.fqz5 /tmp/g.fq
cmp /tmp/c.fq /tmp/w.fastq && cmp /tmp/g.fq /tmp/w.fastq && cmp /tmp/c.fqz5 /tmp/g.fqz5 && echo same >> $OUT/times.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktd -o kt -- \
    $GPU -d -t16 /tmp/c.fqz5 /tmp/g.fq > $OUT/ktd.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kte -o kt -- \
    $GPU -3 -t16 /tmp/w.fastq /tmp/g.fqz5 > $OUT/kte.log 2>&1
echo done
