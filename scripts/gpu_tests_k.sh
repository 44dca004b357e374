#!/bin/bash
# selected GPU tests only: PYTEST_K filter, verbose
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_k.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_k.log | tail -30
[ $rc -ne 0 ] && grep -E "^E " gpurun_out/pytest_k.log | head -30
exit $rc
