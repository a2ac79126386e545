set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/rp
mkdir -p $OUT
B5I="--no-cpu --no-crc --no-dropin --no-level5 --level 5 --kind illumina"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_fqz_gpu.py tests/test_seq_gpu.py tests/test_trial_parity_gpu.py > $OUT/tests.txt 2>&1
timeout -k 10 300 python3 bench.py $B5I --steps 3 --warmup 1 > $OUT/b5i.json 2> $OUT/b5i.log
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/l5i/fetch -o fetch -- python3 bench.py $B5I --steps 1 --warmup 0 > $OUT/fetch5i.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/l5i/write -o write -- python3 bench.py $B5I --steps 1 --warmup 0 > $OUT/write5i.log 2>&1
python3 tools/pmc_summary.py $OUT/l5i $OUT/pmc_l5i.json "the fqz quality chains decode on host cores by the default placement (fqz5_set_host_decode(2))" > /dev/null
echo done
