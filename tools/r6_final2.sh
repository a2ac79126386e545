#!/bin/bash
# Round-6 final tree (second pass): tok3 GPU tests, smoke, the driver bench
# and kernel traces (tools/profile.sh phase a), then the HBM traffic passes
# (phase b).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_tok3_gpu.py tests/test_tok3_search_gpu.py tests/test_fqz5file_gpu.py > gpurun_out/r06d_tests.log 2>&1 || { tail -30 gpurun_out/r06d_tests.log; exit 1; }
tail -1 gpurun_out/r06d_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06d_smoke.log 2>&1 || { tail gpurun_out/r06d_smoke.log; exit 1; }
bash tools/profile.sh r06d a && bash tools/profile.sh r06d b
