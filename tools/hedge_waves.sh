#!/bin/bash
# -5 decode launch time against the number of hedged waves in the launch
# ($FQZ5_HEDGE_WAVES caps hedge_plan's CU budget).  Output: gpurun_out/hw/
set -euo pipefail
mkdir -p gpurun_out/hw
for w in 48 96 160 256; do
  FQZ5_HEDGE_WAVES=$w FQZ5_STEP_TRACE=1 timeout -k 10 300 python3 tools/step_timing.py 5 > gpurun_out/hw/w$w.log 2>&1
done
echo ok
