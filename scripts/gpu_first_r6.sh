#!/bin/bash
# round 6 first GPU call: small-batch sweep (eager vs graph + host issue), then a 2-rank gloo rehearsal of the
# full step on the one GPU (torch engine, side-stream wgrads, fused focal, bitmasks, TUNER.sync, Adam).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
MXR_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --comm torch --batch-size 4 --steps 10 --warmup 3 \
    > gpurun_out/gloo2.log 2>&1 || { echo "gloo2 rc=$?"; tail -30 gpurun_out/gloo2.log; exit 1; }
tail -1 gpurun_out/gloo2.log
bash scripts/gpu_batch_sweep.sh
