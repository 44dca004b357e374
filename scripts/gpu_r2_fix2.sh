#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_p8_gpu.py tests/test_halo_gpu.py tests/test_fp8_gpu.py tests/test_dgrad_s2_gpu.py tests/test_fused_gpu.py tests/test_model_parity_gpu.py tests/test_side_stream_gpu.py > gpurun_out/pytest_fix.log 2>&1 || { tail -30 gpurun_out/pytest_fix.log; exit 1; }
tail -2 gpurun_out/pytest_fix.log
echo "== microbench"
timeout -k 10 300 python scripts/bench_f8.py > gpurun_out/bench_f8.log 2>&1 || { tail -20 gpurun_out/bench_f8.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_f8.log | grep "bf16\|f8_6\|f8_7 "
bash scripts/gpu_r2_bench.sh
