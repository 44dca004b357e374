#!/bin/bash
# BASELINE configs beyond the headline: R101-FPN 1024x1024 bf16, and a 2-rank (gloo, one GPU) rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "== R101 1024x1024 bf16"
timeout -k 10 500 python bench.py --backbone resnet101 --height 1024 --width 1024 --steps 10 --warmup 3 > gpurun_out/cfg_r101.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/cfg_r101.log; exit 1; }
tail -1 gpurun_out/cfg_r101.log | cut -c1-260
echo "== 2 ranks gloo on one GPU"
MXR_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --batch-size 4 > gpurun_out/cfg_dist2.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/cfg_dist2.log; exit 1; }
tail -1 gpurun_out/cfg_dist2.log | cut -c1-200
