# A/B/A/B of an environment switch on the -3 and -5 bench items (step traces on):
#   tools/ab_env.sh TAG VAR=VALUE [steps]
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
ST=${3:-3}
for v in A B A2 B2; do
  case $v in B*) export "$2" ;; *) unset "${2%%=*}" ;; esac
  FQZ5_STEP_TRACE=1 timeout -k 10 300 python3 bench.py --no-cpu --no-level5 --no-crc --no-dropin --steps $ST --warmup 1 > $O/b3$v.json 2> $O/b3$v.log || exit 1
  FQZ5_STEP_TRACE=1 timeout -k 10 300 python3 bench.py --no-cpu --no-crc --no-dropin --level 5 --kind novaseq --gb 4 --steps $ST --warmup 1 > $O/b5$v.json 2> $O/b5$v.log || exit 1
  echo "== $v"; grep -h "entry to exit\|\[bench\] decode\|step:" $O/b3$v.log $O/b5$v.log | tail -16
  python3 -c "
import json
for f in ('$O/b3$v.json','$O/b5$v.json'):
    d=json.load(open(f)); print(f, d['value'], d['enc_MBps'], d['dec_MBps'], d['enc_ms_per_step'], d['dec_ms_per_step'])"
done
