#!/bin/bash
# Round-6 check of the sequence-model context pass: its GPU parity tests,
# the HBM traffic passes (FETCH_SIZE, WRITE_SIZE) and a kernel trace of the
# -5 NovaSeq item, where the trial tries the sequence models.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/sq1; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_seq_gpu.py tests/test_trial_parity_gpu.py tests/test_sections_gpu.py tests/test_stream_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B5="--no-cpu --no-crc --no-dropin --level 5 --kind novaseq --gb 4"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/l5/fetch -o fetch -- python3 bench.py $B5 --steps 1 --warmup 0 > $O/fetch5.log 2>&1 || { tail $O/fetch5.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/l5/write -o write -- python3 bench.py $B5 --steps 1 --warmup 0 > $O/write5.log 2>&1 || { tail $O/write5.log; exit 1; }
python3 tools/pmc_summary.py $O/l5 $O/pmc_l5.json > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt5 -o kt -- python3 bench.py $B5 --steps 5 --warmup 1 > $O/kt5.log 2>&1 || { tail $O/kt5.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/pmc_l5.json'))['kernels']
for k,v in d.items():
    if 'seq' in k or 'ev_fill' in k: print(k, v)
"
tail -1 $O/kt5.log | cut -c1-600
echo ALLDONE
