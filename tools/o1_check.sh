set -euo pipefail
mkdir -p gpurun_out/o1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rans_gpu.py tests/test_sections_gpu.py > gpurun_out/o1/tests.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --level 5 --kind novaseq --gb 4 --steps 2 --warmup 1 > gpurun_out/o1/a.json 2> gpurun_out/o1/a.log
timeout -k 10 300 python3 bench.py --no-cpu --no-level5 --steps 2 --warmup 1 > gpurun_out/o1/b.json 2> gpurun_out/o1/b.log
echo ok
