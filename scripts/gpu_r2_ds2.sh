#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== tests"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_p8_gpu.py > gpurun_out/pytest_ds.log 2>&1 || { tail -30 gpurun_out/pytest_ds.log; exit 1; }
tail -1 gpurun_out/pytest_ds.log
echo "== microbench"
timeout -k 10 300 python scripts/bench_f8.py > gpurun_out/bench_f8.log 2>&1 || { tail -20 gpurun_out/bench_f8.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_f8.log | grep "bf16"
echo "== bench"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-250
