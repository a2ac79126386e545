#!/bin/bash
# Round-6 final tree: the rANS GPU tests (the LDS-tiled STRIPE), smoke, then
# the driver bench and the kernel traces (tools/profile.sh phase a).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_rans_gpu.py tests/test_dropin_gpu.py > gpurun_out/r06c_rans_tests.log 2>&1 || { tail -30 gpurun_out/r06c_rans_tests.log; exit 1; }
tail -1 gpurun_out/r06c_rans_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06c_smoke.log 2>&1 || { tail gpurun_out/r06c_smoke.log; exit 1; }
bash tools/profile.sh r06c a
