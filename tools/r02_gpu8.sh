#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02h
FQZ5_STEP_TRACE=1 timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --no-crc --no-dropin --no-cpu > gpurun_out/r02h/b.json 2> gpurun_out/r02h/b.log || exit $?
grep "step:" gpurun_out/r02h/b.log
grep -B12 "step:" gpurun_out/r02h/b.log | tail -26
