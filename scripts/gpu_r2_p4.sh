#!/bin/bash
# p4 (AGPR-pinned) kernel tests + microbench, then the side-stream tests / bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== p8/p4 tests"
timeout -k 10 300 python -u -m pytest tests/test_p8_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_p8.log 2>&1 || { tail -30 gpurun_out/pytest_p8.log; exit 1; }
tail -3 gpurun_out/pytest_p8.log
echo "== microbench"
timeout -k 10 300 python scripts/bench_p8.py > gpurun_out/bench_p8.log 2>&1 || { tail -20 gpurun_out/bench_p8.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_p8.log
bash scripts/gpu_r2_side.sh
