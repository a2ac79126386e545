#!/bin/bash
# Full GPU suite, then the -3 step trace and a short -3 bench.
set -euo pipefail
OUT=gpurun_out/check
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests \
    > $OUT/tests.log 2>&1
tail -2 $OUT/tests.log
timeout -k 10 300 env FQZ5_STEP_TRACE=1 python3 -u tools/names_timing.py 3 > $OUT/t3.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --no-level5 --no-crc --no-dropin --steps 10 --warmup 3 \
    > $OUT/b3.json 2> $OUT/b3.log
echo done
