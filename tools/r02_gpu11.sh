#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02k
F=tests/golden/fastq/regression_srr1238539.fastq
echo start
timeout -k 5 60 oracle/_ref/fqzcomp5_gpu -1 -t1 $F /tmp/a.fqz5; echo "enc rc=$?"
timeout -k 5 60 oracle/_ref/fqzcomp5_gpu -d -t1 /tmp/a.fqz5 /tmp/a.fq; echo "dec rc=$?"
cmp /tmp/a.fq $F && echo same
GPU_MAX_HW_QUEUES=4 timeout -k 5 60 oracle/_ref/fqzcomp5_gpu -1 -t1 $F /tmp/b.fqz5; echo "enc4 rc=$?"
