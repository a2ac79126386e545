set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/hc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rans_gpu.py tests/test_fqz_gpu.py tests/test_sections_gpu.py > gpurun_out/hc/tests.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --no-level5 > gpurun_out/hc/b3.json 2> gpurun_out/hc/b3.log
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/hc/write -o write -- python3 bench.py --no-cpu --no-level5 --steps 1 --warmup 0 > gpurun_out/hc/write.log 2>&1
echo ok
