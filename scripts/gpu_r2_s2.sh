#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== tests"
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_side_stream_gpu.py tests/test_dgrad_s2_gpu.py tests/test_p8_gpu.py tests/test_kernels_gpu.py tests/test_halo_gpu.py > gpurun_out/pytest_s2.log 2>&1 || { tail -40 gpurun_out/pytest_s2.log; exit 1; }
tail -2 gpurun_out/pytest_s2.log
echo "== microbench"
timeout -k 10 300 python scripts/bench_p8.py > gpurun_out/bench_p8.log 2>&1 || { tail -20 gpurun_out/bench_p8.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_p8.log
bash scripts/gpu_r2_bench.sh
