#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
timeout -k 10 300 python -u -m pytest tests/test_model_parity_gpu.py tests/test_filter_gpu.py -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1; rc=$?
grep -E "PASS|FAIL|^(losses|group|lowest|overfit|batched)|Error|assert" gpurun_out/pytest_parity.log | head -60
exit $rc
