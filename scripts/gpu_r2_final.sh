#!/bin/bash
# full GPU suite + smoke() + fp8 bench (+ the batched-filter timing printed by its test)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== pytest gpu"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rs > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
echo "== filter timing"
timeout -k 10 200 python -u -m pytest tests/test_filter_gpu.py -q -s -k production --timeout 120 --timeout-method thread > gpurun_out/filter_time.log 2>&1 || { tail -20 gpurun_out/filter_time.log; exit 1; }
grep "per batch" gpurun_out/filter_time.log
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-300
echo "== fp8 bench"
timeout -k 10 400 python bench.py --dtype fp8 > gpurun_out/bench_fp8.log 2>&1 || { tail -20 gpurun_out/bench_fp8.log; exit 1; }
tail -1 gpurun_out/bench_fp8.log | grep -o '"value": [0-9.]*, "unit": "[^"]*", "n_gpus": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*'
echo "== bf16 bench"
timeout -k 10 400 python bench.py > gpurun_out/bench_bf16.log 2>&1 || { tail -20 gpurun_out/bench_bf16.log; exit 1; }
tail -1 gpurun_out/bench_bf16.log | grep -o '"value": [0-9.]*, "unit": "[^"]*", "n_gpus": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*'
