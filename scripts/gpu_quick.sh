#!/bin/bash
# build -> GPU tests -> end-to-end bench (+ saved tuner table) -> rocprof kernel stats with that table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
python -m batchai_retinanet_horovod_coco_amd.build || exit 1
echo "== pytest gpu ${PYTEST_K:-all}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc -> stop"; exit $rc; fi
echo "== bench"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 400 python bench.py --steps 10 --warmup 3 --verbose > gpurun_out/bench_hip.log 2>&1 || { echo "bench rc=$?"; tail -30 gpurun_out/bench_hip.log; exit 1; }
tail -2 gpurun_out/bench_hip.log
python scripts/conv_budget.py gpurun_out/conv_table.json 13 > gpurun_out/conv_budget.txt && head -45 gpurun_out/conv_budget.txt
if [ -n "$FP8" ]; then
  echo "== bench fp8"
  MXR_SAVE_CONV_TABLE=gpurun_out/conv_table_fp8.json timeout -k 10 400 python bench.py --steps 10 --warmup 3 --dtype fp8 --verbose > gpurun_out/bench_fp8.log 2>&1 || { echo "bench fp8 rc=$?"; tail -30 gpurun_out/bench_fp8.log; exit 1; }
  tail -1 gpurun_out/bench_fp8.log
  python scripts/conv_budget.py gpurun_out/conv_table_fp8.json 13 > gpurun_out/conv_budget_fp8.txt && head -30 gpurun_out/conv_budget_fp8.txt
fi
if [ "${PROF:-1}" = "1" ]; then
  echo "== rocprof"
  R=$GRAFT_REPO_ROOT
  cd /tmp && export TMPDIR=/tmp
  MXR_CONV_TABLE=$R/gpurun_out/conv_table.json timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_hip -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3 > $R/gpurun_out/prof_hip.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $R/gpurun_out/prof_hip.log; exit 1; }
  python3 $R/scripts/prof_summary.py $R/gpurun_out/prof_hip/run_kernel_stats.csv --steps 6 > $R/gpurun_out/prof_summary.txt && cat $R/gpurun_out/prof_summary.txt
fi
