#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_fp8.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_fp8.log; exit 1; }
tail -1 gpurun_out/pytest_fp8.log
bash scripts/gpu_r3_fp8ab.sh
