#!/bin/bash
# conv_hx32_f8: numerics, head-shape microbench against the bf16 hx32 and the older fp8 kernels, fp8 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "${PYTEST_K:-hx8 or dequantized or dgrad or fused}" > gpurun_out/pytest_hx8.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_hx8.log; exit 1; }
tail -1 gpurun_out/pytest_hx8.log
timeout -k 10 300 python -u scripts/bench_f8.py > gpurun_out/bench_hx8.log 2>&1 || { echo "bench_f8 rc=$?"; tail -20 gpurun_out/bench_hx8.log; exit 1; }
cat gpurun_out/bench_hx8.log
if [ -n "$BENCH" ]; then
  MXR_SAVE_CONV_TABLE=gpurun_out/conv_table_fp8.json timeout -k 10 400 python -u bench.py --dtype fp8 > gpurun_out/bench_fp8.log 2> gpurun_out/bench_fp8.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench_fp8.err; exit 1; }
  tail -1 gpurun_out/bench_fp8.log
  timeout -k 10 900 python -u -m pytest tests/test_fp8_gpu.py -m gpu -q -x --timeout 600 --timeout-method thread -k "training or step" > gpurun_out/pytest_fp8_train.log 2>&1 || { echo "fp8 train rc=$?"; tail -30 gpurun_out/pytest_fp8_train.log; exit 1; }
  tail -1 gpurun_out/pytest_fp8_train.log
fi
