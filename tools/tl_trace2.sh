# step traces of the -3 and -5 bench items (no profiler): tools/tl_trace2.sh TAG
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-tl2}; mkdir -p $O
FQZ5_STEP_TRACE=1 timeout -k 10 300 python3 bench.py --no-cpu --no-level5 --no-crc --no-dropin --steps 3 --warmup 1 > $O/b3.json 2> $O/b3.log || exit 1
FQZ5_STEP_TRACE=1 timeout -k 10 300 python3 bench.py --no-cpu --no-crc --no-dropin --level 5 --kind novaseq --gb 4 --steps 3 --warmup 1 > $O/b5.json 2> $O/b5.log || exit 1
grep -h "decode_sections: from\|\[bench\]" $O/b3.log $O/b5.log
