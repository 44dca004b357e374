#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
MXR_POOL_K3S2=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_stem_gpu.py tests/test_model_parity_gpu.py > gpurun_out/pool_tests.log 2>&1; rc=$?; tail -3 gpurun_out/pool_tests.log; [ $rc -ne 0 ] && exit $rc
VALUES="MXR_AB=generic MXR_POOL_K3S2=1 MXR_AB=generic MXR_POOL_K3S2=1" bash scripts/gpu_r2_sweep.sh
