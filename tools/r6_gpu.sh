#!/bin/bash
# Round-6 GPU session steps: usage tools/r6_gpu.sh TAG STEP...
#   tests:FILES   pytest -m gpu on the listed test files (comma separated)
#   suite         the whole GPU suite
#   bench:ARGS    bench.py with ARGS (comma separated) -> gpurun_out/TAG_bench.json
#   dropin        tools/dropin_trace.sh -> gpurun_out/TAG_dropin/
#   smoke         __graft_entry__.smoke()
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
O=gpurun_out
mkdir -p $O
for st in "$@"; do
  case $st in
    tests:*) f=${st#tests:}; f=${f//,/ }
      timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $f > $O/${TAG}_tests.log 2>&1
      rc=$?; tail -3 $O/${TAG}_tests.log; [ $rc = 0 ] || { echo "TESTS rc=$rc"; grep -E "FAIL|Error" $O/${TAG}_tests.log | head -20; exit 1; } ;;
    suite)
      timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/${TAG}_suite.log 2>&1
      rc=$?; tail -3 $O/${TAG}_suite.log; [ $rc = 0 ] || { echo "SUITE rc=$rc"; grep -E "FAIL|Error" $O/${TAG}_suite.log | head -20; exit 1; } ;;
    bench*:*) a=${st#*:}; a=${a//,/ }; v=${st%%:*}; v=${v#bench}
      # benchNAME:ARGS with NAME a tools/ab/libfqz5_NAME.so variant (A/B)
      if [ -n "$v" ]; then export FQZ5_LIB_VARIANT=$PWD/tools/ab/libfqz5_$v.so; else unset FQZ5_LIB_VARIANT; fi
      TAGB=${TAG}${v}
      timeout -k 10 900 python -u bench.py $a > $O/${TAGB}_bench.json 2> $O/${TAGB}_bench.log
      rc=$?; unset FQZ5_LIB_VARIANT; [ $rc = 0 ] || { echo "BENCH rc=$rc"; tail -20 $O/${TAGB}_bench.log; exit 1; }
      python3 -c "
import json,sys; d=json.load(open('$O/${TAGB}_bench.json'))
def s(x): return {k:x.get(k) for k in ('value','enc_MBps','dec_MBps','enc_ms_min_max','dec_ms_min_max')}
print('main', s(d)); print('roof', {k:d['roofline'].get(k) for k in ('kernel','avg_launch_ms','frac','kernel_ms_per_step')}, d['roofline']['chains'])
for k in ('level5','level5_illumina'):
    if k in d: print(k, s(d[k]), d[k].get('cpu_baseline',{}).get('t1_file_md5_match'), d[k].get('cpu_baseline',{}).get('t1_blocks_matching'))
print('cpu', {k:d.get('cpu_baseline',{}).get(k) for k in ('value','enc_MBps','dec_MBps','blocks_match_gpu')})
print('dropin', json.dumps(d.get('dropin_cli'))[:900])
" ;;
    n2)   # the N = 2 path rehearsed on one GPU (gloo), strong scaling, beside
          # the one-process run's blocks split the same way
      FQZ5_BENCH_SPLIT=2 timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-level5 --no-dropin --no-cpu --no-crc > $O/${TAG}_n1split.json 2> $O/${TAG}_n1split.log || { echo N1SPLIT failed; tail -5 $O/${TAG}_n1split.log; exit 1; }
      FQZ5_BENCH_SHARE_GPU=1 timeout -k 10 900 python -u bench.py --gpus 2 --steps 3 --warmup 1 --scaling strong --no-level5 --no-dropin --no-cpu --no-crc > $O/${TAG}_n2.json 2> $O/${TAG}_n2.log || { echo N2 failed; tail -20 $O/${TAG}_n2.log; exit 1; }
      python3 -c "
import json; L=lambda f: json.loads(open(f).read().strip().splitlines()[-1]); a=L('$O/${TAG}_n1split.json'); b=L('$O/${TAG}_n2.json')
print('n1 split', a['config']['blocks_md5_by_rank'], a['value']); print('n2', b['config']['blocks_md5_by_rank'], b['value'], b['n_gpus'])
print('N2_BLOCKS_EQUAL', a['config']['blocks_md5_by_rank'] == b['config']['blocks_md5_by_rank'])" ;;
    dropin)
      timeout -k 10 600 bash tools/dropin_trace.sh $O/${TAG}_dropin > $O/${TAG}_dropin.log 2>&1
      rc=$?; tail -12 $O/${TAG}_dropin.log; [ $rc = 0 ] || { echo "DROPIN rc=$rc"; exit 1; } ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1
      rc=$?; tail -2 $O/${TAG}_smoke.log; [ $rc = 0 ] || { echo "SMOKE rc=$rc"; exit 1; } ;;
  esac
done
echo ALLDONE
