# File-path stages (FQZ5_FILE_TRACE) of fqz5file on the bench's 1 GB file,
# beside the reference CLI's -d on the same .fqz5: tools/file_trace.sh TAG [reps]
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
FQZ5_FILE_TRACE=1 timeout -k 10 400 python3 -u tools/file_path_check.py 1 3 ${2:-3} > $O/file.txt 2>&1 || { tail -20 $O/file.txt; exit 1; }
grep -v "^\[tid\|^names\|^decode\|^sections\|^tok3\|^fqz" $O/file.txt | tail -12
