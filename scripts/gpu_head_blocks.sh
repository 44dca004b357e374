#!/bin/bash
# head weight-gradient grid: isolated time at 189 / 252 / 378 blocks, then the in-step sweep of MXR_WGRAD_HEAD_BLOCKS
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for b in 192 256 384; do
  echo "== isolated, MXR_WGRAD_HEAD_BLOCKS=$b"
  MXR_WGRAD_HEAD_BLOCKS=$b timeout -k 10 120 python -u scripts/bench_wgrad.py --only pyr > gpurun_out/wq_b$b.txt 2>&1 || exit 1
  grep -E "256->(256|720)" gpurun_out/wq_b$b.txt | cut -c1-120
done
for b in ${BLOCKS:-160 192 256 192 224}; do
  MXR_WGRAD_HEAD_BLOCKS=$b timeout -k 10 300 python -u bench.py > gpurun_out/hb_$b.log 2> gpurun_out/hb_$b.err || { tail -5 gpurun_out/hb_$b.err; exit 1; }
  echo "head blocks $b: $(tail -1 gpurun_out/hb_$b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
