#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02s
for v in hi normal; do
  if [ $v = normal ]; then export FQZ5_AUX_NORMAL_PRIO=1; fi
  FQZ5_STEP_TRACE=1 timeout -k 10 400 python -u bench.py --level 5 --kind novaseq --gb 4 --steps 5 --warmup 2 --no-crc --no-dropin --no-cpu > gpurun_out/r02s/b_$v.json 2> gpurun_out/r02s/b_$v.log || exit $?
  echo "== $v"; grep "step:" gpurun_out/r02s/b_$v.log; grep "helpers waited" gpurun_out/r02s/b_$v.log | tail -5
done
