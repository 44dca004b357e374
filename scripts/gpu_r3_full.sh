#!/bin/bash
# full GPU suite, smoke, driver-style bench + kernel-trace profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_full.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_gpu_full.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_full.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
PROF=1 bash scripts/gpu_r3_cycle.sh
