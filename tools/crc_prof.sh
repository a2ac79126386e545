set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/crc
timeout -k 10 200 python3 tools/crc_timing.py 4 > gpurun_out/crc/t.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/crc/kt -o kt -- python3 tools/crc_timing.py 4 > gpurun_out/crc/kt.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/crc/fetch -o fetch -- python3 tools/crc_timing.py 1 > gpurun_out/crc/fetch.log 2>&1
echo ok
