#!/bin/bash
# GPU tests of the trial paths, then -5 NovaSeq / Illumina bench items with
# the step trace (outputs under gpurun_out/tlzp).
set -euo pipefail
OUT=gpurun_out/tlzp
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_sections_gpu.py tests/test_trial_parity_gpu.py tests/test_fqz5file_gpu.py > $OUT/tests.txt 2>&1
FQZ5_STEP_TRACE=1 timeout -k 10 300 python3 bench.py --no-cpu --no-crc --no-dropin --level 5 --kind novaseq --gb 4 --steps 3 --warmup 1 > $OUT/b5.json 2> $OUT/b5.log
timeout -k 10 300 python3 bench.py --no-cpu --no-crc --no-dropin --no-level5 --level 5 --kind illumina --steps 3 --warmup 1 > $OUT/b5i.json 2> $OUT/b5i.log
echo done
