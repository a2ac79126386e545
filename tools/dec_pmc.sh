#!/bin/bash
# PMC counters of the fqz decoder (k_fqz_dec) on one NovaSeq block, strat 0:
# instructions by type and wave cycles split into issue / issue-stall /
# waitcnt (MI355X_MICROARCH.md, SQ block), one rocprofv3 pass per group.
set -u
export TMPDIR=/tmp
out=gpurun_out/pmc_dec
mkdir -p $out
kind=${1:-novaseq}; strat=${2:-0}
timeout -k 10 120 python -u tools/fqz_dec_once.py $kind $strat 27000 > $out/once.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM -d $out/p1 -o p1 -- python3 tools/fqz_dec_once.py $kind $strat 27000 > $out/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_INSTS_VALU_TRANS_F64 SQ_BUSY_CYCLES -d $out/p2 -o p2 -- python3 tools/fqz_dec_once.py $kind $strat 27000 > $out/p2.log 2>&1 || true
find $out -name "*counter_collection*" | head
