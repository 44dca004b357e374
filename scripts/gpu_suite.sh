#!/bin/bash
# GPU test tier + smoke (what the round driver runs):  PYTEST_K="halo or wgrad" bash scripts/gpu_suite.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== pytest gpu ${PYTEST_K:-all}"
timeout -k 10 ${TEST_TIMEOUT:-1100} python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
[ -n "$NO_SMOKE" ] && exit 0
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
