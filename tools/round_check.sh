#!/bin/bash
# end-of-round check on the GPU box: the whole GPU suite, smoke(), then the
# driver's bench command (N=1)
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rc
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/rc/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/rc/tests.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rc/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/rc/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rc/bench.json 2> gpurun_out/rc/bench.log
rc=$?
echo "bench rc=$rc"; tail -c 600 gpurun_out/rc/bench.json
exit $rc
