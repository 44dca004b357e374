#!/bin/bash
# round-4 kernel check: numerics of the new / changed kernels, wgrad microbench, counters of the head wgrad
# candidates, then the driver bench + per-kernel counters of the step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_wgrad_hx32_gpu.py tests/test_c1x1_gpu.py tests/test_fused_bias_gpu.py tests/test_kernels_gpu.py -k "wgrad or c1x1 or fused" > gpurun_out/pytest_5.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_5.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/bench_wgrad.py --only pyr > gpurun_out/bench_wgrad.log 2>&1; cat gpurun_out/bench_wgrad.log
timeout -k 10 600 bash scripts/gpu_pmc_pyr.sh "hxw 0" "wgrad 23" "wgrad 25" > gpurun_out/pmc_pyr.log 2>&1; grep -E "==|MFMA busy|WAIT|conflict|SQ_INSTS_LDS |SQ_INSTS_VALU |SQ_INSTS_MFMA |SQ_LDS_BANK|SQ_LDS_IDX" gpurun_out/pmc_pyr.log
rm -rf gpurun_out/pmc_pyr/*_[12]
[ -n "$NO_BENCH" ] && exit 0
TOP=24 timeout -k 10 1100 bash scripts/gpu_bench_pmc.sh
