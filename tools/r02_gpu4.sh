#!/bin/bash
# re-entry check: whole GPU suite, smoke, then the -3 step phases
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02d
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r02d/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r02d/tests.log | tail -15
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02d/smoke.log 2>&1 || exit $?
FQZ5_STEP_TRACE=1 timeout -k 10 300 python -u tools/step_timing.py 3 > gpurun_out/r02d/st3.log 2>&1 || exit $?
tail -40 gpurun_out/r02d/st3.log
