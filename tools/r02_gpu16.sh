#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02p
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_rans_gpu.py tests/test_sections_gpu.py tests/test_dropin_gpu.py > gpurun_out/r02p/t.log 2>&1 || { tail -30 gpurun_out/r02p/t.log; exit 1; }
tail -2 gpurun_out/r02p/t.log
timeout -k 10 300 python -u tools/dec_jobs_probe.py 5 > gpurun_out/r02p/j5.log 2>&1 || { tail gpurun_out/r02p/j5.log; exit 1; }
head -4 gpurun_out/r02p/j5.log; tail -3 gpurun_out/r02p/j5.log
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --no-crc --no-dropin --no-cpu > gpurun_out/r02p/b.json 2> gpurun_out/r02p/b.log || exit $?
grep "step:" gpurun_out/r02p/b.log
python - <<'P'
import json; d=json.load(open("gpurun_out/r02p/b.json"))
print(d["value"], d["enc_MBps"], d["dec_MBps"], d["roofline"]["dec_avg_ms"], d["level5"]["value"], d["level5"]["dec_MBps"], d["level5"]["roofline"]["dec_avg_ms"])
P
