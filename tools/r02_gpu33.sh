#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02n
timeout -k 10 300 python -u tools/names_timing.py 3 > gpurun_out/r02n/t3.log 2>&1 || { tail -40 gpurun_out/r02n/t3.log; exit 1; }
grep -E "names|encode_run|sections_try: [0-9]|rANS candidates|decode_sections|roundtrip" gpurun_out/r02n/t3.log | tail -8
timeout -k 10 500 python -u tools/names_timing.py 5 4.0 > gpurun_out/r02n/t5.log 2>&1 || { tail -40 gpurun_out/r02n/t5.log; exit 1; }
grep -E "names|encode_run|sections_try: [0-9]|rANS candidates|decode_sections|roundtrip" gpurun_out/r02n/t5.log | tail -8
