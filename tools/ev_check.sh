set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/ev1; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_fqz_gpu.py tests/test_fqz_small_gpu.py tests/test_trial_parity_gpu.py tests/test_sections_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B5I="--no-cpu --no-crc --no-dropin --no-level5 --level 5 --kind illumina"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/l5i/fetch -o fetch -- python3 bench.py $B5I --steps 1 --warmup 0 > $O/fetch5i.log 2>&1 || { tail $O/fetch5i.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/l5i/write -o write -- python3 bench.py $B5I --steps 1 --warmup 0 > $O/write5i.log 2>&1 || { tail $O/write5i.log; exit 1; }
python3 tools/pmc_summary.py $O/l5i $O/pmc_l5i.json "the fqz quality chains decode on host cores by the default placement (fqz5_set_host_decode(2))" > /dev/null
python3 -c "
import json; d=json.load(open('$O/pmc_l5i.json'))['kernels']
for k,v in d.items():
    if 'ev_fill' in k or 'model_pass' in k: print(k, v)
"
echo ALLDONE
