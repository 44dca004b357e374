#!/bin/bash
# epilogue-prefetch check: conv numerics (unit + production-shape winners), bench, host pipeline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_p8_gpu.py tests/test_c1x1_gpu.py tests/test_dgrad_s2_gpu.py tests/test_fused_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_epi.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_epi.log; exit 1; }
tail -1 gpurun_out/pytest_epi.log
timeout -k 10 600 python -u -m pytest tests/test_winners_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/winners.log 2>&1 || { echo "winners rc=$?"; tail -30 gpurun_out/winners.log; exit 1; }
tail -1 gpurun_out/winners.log
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench.err; exit 1; }
tail -1 gpurun_out/bench.log
python scripts/conv_budget.py gpurun_out/conv_table.json 25 > gpurun_out/conv_budget.txt
for w in ${LOADER_WORKERS:-2 4}; do
  timeout -k 10 400 python -u -m batchai_retinanet_horovod_coco_amd.bin.train --bench 5 20 --workers $w --device-preprocess --loader process --batch-size 16 --no-weights --calibrate-bn --clip-mode global --no-evaluation synthetic --num-images 128 --height 800 --width 1333 > gpurun_out/pipe_w$w.log 2>&1 || { echo "pipeline rc=$?"; tail -20 gpurun_out/pipe_w$w.log; exit 1; }
  echo "workers $w: $(grep metric gpurun_out/pipe_w$w.log | tail -1)"
done
