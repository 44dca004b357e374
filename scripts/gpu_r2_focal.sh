#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== tests"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_gpu.py tests/test_model_parity_gpu.py > gpurun_out/pytest_focal.log 2>&1 || { tail -30 gpurun_out/pytest_focal.log; exit 1; }
tail -1 gpurun_out/pytest_focal.log
bash scripts/gpu_r2_bench.sh
