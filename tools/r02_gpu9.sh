#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02i
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_rans_gpu.py tests/test_sections_gpu.py > gpurun_out/r02i/t.log 2>&1 || { tail -30 gpurun_out/r02i/t.log; exit 1; }
tail -2 gpurun_out/r02i/t.log
FQZ5_STEP_TRACE=1 timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --no-crc --no-dropin --no-cpu > gpurun_out/r02i/b.json 2> gpurun_out/r02i/b.log || exit $?
grep "step:" gpurun_out/r02i/b.log
grep -B12 "step:" gpurun_out/r02i/b.log | tail -13
python - <<'P'
import json; d=json.load(open("gpurun_out/r02i/b.json"))
print(d["value"], d["enc_MBps"], d["dec_MBps"], d["roofline"]["enc_avg_ms"], d["level5"]["value"], d["level5"]["enc_MBps"], d["level5"]["roofline"]["enc_avg_ms"])
P
