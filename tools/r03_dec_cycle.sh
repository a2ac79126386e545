set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fqz_gpu.py > gpurun_out/fqz_t.log 2>&1 || exit 1
FQZ5_DEBUG=1 timeout -k 10 300 python -u tools/fqz_dec_bench.py 4 novaseq,ont,hifi > gpurun_out/dec_v3.log 2>&1 || exit 1
rm -rf gpurun_out/r03/pmc_dec
bash tools/r03_dec_pmc.sh novaseq 1
