#!/bin/bash
# interval trial + hedged fqz decode: the upper bound asserted on every fqz /
# sequence-model encode (goldens, trial parity), the bounded run against
# encode_run with and without intervals, the streaming file path at -7/-9
set -uo pipefail
OUT=gpurun_out/r03/bounds
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q -s --timeout 400 --timeout-method thread -m gpu \
    tests/test_fqz_gpu.py tests/test_seq_gpu.py tests/test_sections_gpu.py \
    tests/test_trial_parity_gpu.py tests/test_stream_gpu.py > $OUT/tests.log 2>&1
rc=$?; grep -E "intervals decided|passed|failed|Error" $OUT/tests.log | tail -8; exit $rc
