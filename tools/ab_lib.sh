# A/B of a library variant (tools/ab/libfqz5_NAME.so) against the tree's
# library on the -3 and -5 bench items, step traces on, then optional tests:
#   tools/ab_lib.sh TAG NAME [steps] [test files...]
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
NAME=$2; ST=${3:-3}; shift 3 || shift $#
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || { echo "TESTS rc=$rc"; grep -E "FAIL|Error" $O/tests.log | head -20; exit 1; }
fi
for v in new base new base; do
  if [ $v = base ]; then export FQZ5_LIB_VARIANT=$PWD/tools/ab/libfqz5_$NAME.so; else unset FQZ5_LIB_VARIANT; fi
  FQZ5_STEP_TRACE=1 timeout -k 10 300 python3 bench.py --no-cpu --no-level5 --no-crc --no-dropin --steps $ST --warmup 1 > $O/b3$v.json 2> $O/b3$v.log || exit 1
  FQZ5_STEP_TRACE=1 timeout -k 10 300 python3 bench.py --no-cpu --no-crc --no-dropin --level 5 --kind novaseq --gb 4 --steps $ST --warmup 1 > $O/b5$v.json 2> $O/b5$v.log || exit 1
  echo "== $v"; grep -h "entry to exit\|names decode\|names encode" $O/b3$v.log $O/b5$v.log | tail -4
  python3 -c "
import json
for f in ('$O/b3$v.json','$O/b5$v.json'):
    d=json.load(open(f)); print(f, d['value'], d['enc_MBps'], d['dec_MBps'], d['enc_ms_per_step'], d['dec_ms_per_step'], d['config']['blocks_md5_by_rank'])"
done
