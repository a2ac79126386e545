set -euo pipefail
mkdir -p gpurun_out/l5p
timeout -k 10 300 python3 bench.py --no-cpu --level 5 --kind novaseq --gb 4 --steps 2 --warmup 1 > gpurun_out/l5p/a.json 2> gpurun_out/l5p/a.log
FQZ5_NO_HEDGE=1 timeout -k 10 300 python3 bench.py --no-cpu --level 5 --kind novaseq --gb 4 --steps 2 --warmup 1 > gpurun_out/l5p/b.json 2> gpurun_out/l5p/b.log
timeout -k 10 300 python3 bench.py --no-cpu --level 5 --kind novaseq --gb 1 --steps 2 --warmup 1 > gpurun_out/l5p/c.json 2> gpurun_out/l5p/c.log
echo ok
