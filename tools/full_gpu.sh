set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/full
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/full/tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1
echo ok
