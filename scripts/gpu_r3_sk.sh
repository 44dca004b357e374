#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_hx32_pack_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_sk.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_sk.log; exit 1; }
tail -1 gpurun_out/pytest_sk.log
bash scripts/gpu_r3_fp8ab.sh
python3 scripts/conv_budget.py gpurun_out/conv_table_bf16.json 25 > gpurun_out/conv_budget_bf16.txt
grep -E "sk1|13\|21\|256\|256\|3\|2|25\|42\|2048\|256\|3\|2" gpurun_out/conv_budget_bf16.txt
