#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02u
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_rans_gpu.py tests/test_sections_gpu.py > gpurun_out/r02u/t.log 2>&1 || { tail -30 gpurun_out/r02u/t.log; exit 1; }
tail -2 gpurun_out/r02u/t.log
FQZ5_LIB_VARIANT=$PWD/tools/probe/libfqz5_cprobe.so timeout -k 10 200 python -u tools/enc_probe_run.py > gpurun_out/r02u/enc_probe.log 2>&1 || exit $?
cat gpurun_out/r02u/enc_probe.log
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --no-crc --no-dropin --no-cpu > gpurun_out/r02u/b.json 2> gpurun_out/r02u/b.log || exit $?
grep "step:" gpurun_out/r02u/b.log
python - <<'P'
import json; d=json.load(open("gpurun_out/r02u/b.json"))
print(d["value"], d["enc_MBps"], d["dec_MBps"], d["roofline"]["enc_avg_ms"], d["level5"]["value"], d["level5"]["enc_MBps"], d["level5"]["roofline"]["enc_avg_ms"])
P
