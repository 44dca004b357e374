#!/bin/bash
# s2 wgrad candidate diagnostic, then the GPU suite without stopping at the first failure
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
timeout -k 10 180 python -u scripts/diag_s2_wgrad.py > gpurun_out/diag_s2.log 2>&1; rc=$?
cat gpurun_out/diag_s2.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 15 --timeout 120 --timeout-method thread -k "${PYTEST_K:-not trajectory}" > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -30
exit $rc
