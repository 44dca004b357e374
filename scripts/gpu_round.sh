#!/bin/bash
# Kernel numerics + conv shape-class microbench + end-to-end bench with the HIP kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== build"
python -m batchai_retinanet_horovod_coco_amd.build || exit 1
echo "== pytest gpu"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc -> stop"; exit $rc; fi
echo "== conv microbench"
timeout -k 10 400 python scripts/bench_conv.py --out gpurun_out/bench_conv.json > gpurun_out/bench_conv.log 2>&1 || { echo "bench_conv rc=$?"; tail -20 gpurun_out/bench_conv.log; exit 1; }
cat gpurun_out/bench_conv.log
echo "== bench (HIP)"
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --verbose > gpurun_out/bench_hip.log 2>&1; echo "bench rc=$?"
tail -5 gpurun_out/bench_hip.log
