#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02x
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_rans_gpu.py tests/test_sections_gpu.py tests/test_dropin_gpu.py tests/test_trial_parity_gpu.py > gpurun_out/r02x/t.log 2>&1 || { tail -30 gpurun_out/r02x/t.log; exit 1; }
tail -2 gpurun_out/r02x/t.log
timeout -k 10 500 python -u bench.py --steps 8 --warmup 2 --no-crc --no-dropin --no-cpu > gpurun_out/r02x/b.json 2> gpurun_out/r02x/b.log || exit $?
grep "step:" gpurun_out/r02x/b.log
python - <<'P'
import json; d=json.load(open("gpurun_out/r02x/b.json"))
print(d["value"], d["enc_MBps"], d["dec_MBps"], d["roofline"]["dec_avg_ms"], d["level5"]["value"], d["level5"]["enc_MBps"], d["level5"]["dec_MBps"])
P
