set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tl1; mkdir -p $O
B5="--no-cpu --no-crc --no-dropin --level 5 --kind novaseq --gb 4"
B3="--no-cpu --no-level5 --no-crc --no-dropin"
FQZ5_STEP_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt5 -o kt -- \
    python3 bench.py $B5 --steps 2 --warmup 1 > $O/kt5.json 2> $O/kt5.log || exit 1
FQZ5_STEP_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt3 -o kt -- \
    python3 bench.py $B3 --steps 2 --warmup 1 > $O/kt3.json 2> $O/kt3.log || exit 1
ls -la $O/kt5 $O/kt3
