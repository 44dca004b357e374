#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== bench fp8"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table_f8.json timeout -k 10 600 python bench.py --dtype fp8 > gpurun_out/bench_fp8.log 2>&1 || { tail -20 gpurun_out/bench_fp8.log; exit 1; }
tail -1 gpurun_out/bench_fp8.log | cut -c1-300
echo "== fp8 tests"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fp8_gpu.py > gpurun_out/pytest_f8.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_f8.log | tail -30; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_f8.log | tail -2
