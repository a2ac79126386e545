#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02g
FQZ5_STEP_TRACE=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-level5 --no-crc --no-dropin --no-cpu > gpurun_out/r02g/b.json 2> gpurun_out/r02g/b.log || exit $?
tail -32 gpurun_out/r02g/b.log
