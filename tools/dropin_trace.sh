#!/bin/bash
# The drop-in CLI (oracle/_ref/fqzcomp5_gpu: the reference CLI relinked on
# libfqz5_mi355x.so) against the CLI as shipped on the bench's 1 GB -3 file,
# with the library's per-call trace (FQZ5_CALL_TRACE=1: thread, call, size,
# ms since load at entry / upload / run / exit) for VERDICT r05 item 2.
# usage: tools/dropin_trace.sh OUTDIR [level]
set -euo pipefail
OUT=${1:-gpurun_out/dropin}
LV=${2:-3}
mkdir -p $OUT
export TMPDIR=/tmp
CPU=oracle/_ref/fqzcomp5
GPU=oracle/_ref/fqzcomp5_gpu
[ -f /tmp/w.fastq ] || python3 -c "import sys; sys.path.insert(0, '.'); import bench; from fqzcomp5_amd import synth; synth.write_fastq(bench.make_reads(1.0, 1, 'illumina'), '/tmp/w.fastq')"
t() { local a=$(date +%s%N); "$@"; local b=$(date +%s%N); echo "$(( (b - a) / 1000000 )) ms: $*" >> $OUT/times.txt; }
t timeout -k 10 120 $CPU -$LV -t16 /tmp/w.fastq /tmp/c.fqz5
t timeout -k 10 120 $CPU -d -t16 /tmp/c.fqz5 /tmp/c.fq
t timeout -k 10 120 $GPU -$LV -t16 /tmp/w.fastq /tmp/g.fqz5
t timeout -k 10 120 $GPU -d -t16 /tmp/c.fqz5 /tmp/g.fq
FQZ5_CALL_TRACE=1 FQZ5_STEP_TRACE=1 t timeout -k 10 120 $GPU -$LV -t16 /tmp/w.fastq /tmp/g.fqz5 2> $OUT/enc_calls.txt
FQZ5_CALL_TRACE=1 t timeout -k 10 120 $GPU -d -t16 /tmp/c.fqz5 /tmp/g.fq 2> $OUT/dec_calls.txt
cmp /tmp/c.fq /tmp/w.fastq && cmp /tmp/g.fq /tmp/w.fastq && cmp /tmp/c.fqz5 /tmp/g.fqz5 && echo same >> $OUT/times.txt
cat $OUT/times.txt
