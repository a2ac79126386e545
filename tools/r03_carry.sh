#!/bin/bash
# parallel carry normalisation: fqz / sequence-model goldens, the bounded
# -7/-9 run, the trial parity at -7/-9, then the -7 ONT step time
set -uo pipefail
OUT=gpurun_out/r03/carry
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_fqz_gpu.py tests/test_seq_gpu.py tests/test_sections_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --no-cpu --no-level5 --no-crc --no-dropin \
    --level 7 --kind ont --gb 1.5 --steps 1 --warmup 0 > $OUT/b7.json 2> $OUT/b7.log
echo "rc=$?"; grep "bench\]" $OUT/b7.log
