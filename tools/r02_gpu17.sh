#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02y
FQZ5_STEP_TRACE=1 timeout -k 10 500 python -u bench.py --level 5 --kind novaseq --gb 4 --steps 4 --warmup 1 --no-crc --no-dropin --no-cpu > gpurun_out/r02y/b.json 2> gpurun_out/r02y/b.log || exit $?
grep -B22 "step:" gpurun_out/r02y/b.log | tail -23
