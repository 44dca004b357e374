#!/bin/bash
# full GPU test suite + smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== pytest gpu"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rs > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -12 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
