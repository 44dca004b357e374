#!/bin/bash
# Kernel-iteration run: build, GPU kernel tests, ablation + per-shape conv microbench, then the
# end-to-end bench with fresh tuning (table saved to gpurun_out/).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
python -m batchai_retinanet_horovod_coco_amd.build || exit 1
echo "== pytest gpu ${PYTEST_K:-all}"
timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc -> stop"; exit $rc; fi
if [ -z "$SKIP_MICRO" ]; then
  echo "== ablate"
  timeout -k 10 200 python scripts/ablate_conv.py > gpurun_out/ablate.log 2>&1 || { echo "ablate rc=$?"; tail -20 gpurun_out/ablate.log; exit 1; }
  cat gpurun_out/ablate.log
  echo "== conv microbench"
  timeout -k 10 500 python scripts/bench_conv.py ${BENCH_CONV_ARGS} > gpurun_out/bench_conv.log 2>&1 || { echo "bench_conv rc=$?"; tail -20 gpurun_out/bench_conv.log; exit 1; }
  cat gpurun_out/bench_conv.log
fi
echo "== bench"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 400 python bench.py --steps 10 --warmup 3 --verbose > gpurun_out/bench_hip.log 2>&1 || { echo "bench rc=$?"; tail -30 gpurun_out/bench_hip.log; exit 1; }
tail -2 gpurun_out/bench_hip.log
