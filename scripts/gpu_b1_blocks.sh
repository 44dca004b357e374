#!/bin/bash
# B=1 graph replay vs the side-stream wgrad split-K grid target (MXR_WGRAD_PIPE_BLOCKS)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for nb in ${NBS:-64 128 192 384}; do
  MXR_WGRAD_PIPE_BLOCKS=$nb timeout -k 10 300 python -u bench.py --batch-size 1 --graph --steps 50 --warmup 5 > gpurun_out/b1.log 2> gpurun_out/b1.err || { echo "nb=$nb rc=$?"; tail -20 gpurun_out/b1.err; exit 1; }
  echo "B=1 graph MXR_WGRAD_PIPE_BLOCKS=$nb: $(tail -1 gpurun_out/b1.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], "img/s", r["ms_per_step"], "ms/step")')" | tee -a gpurun_out/b1_blocks.txt
done
