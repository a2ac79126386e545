#!/bin/bash
# the whole GPU suite and smoke(), as the driver runs them at round end
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/full
timeout -k 10 1100 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/full/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/full/tests.log | tail -15
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1
echo "smoke rc=$?"; tail -3 gpurun_out/full/smoke.log
