#!/bin/bash
# usage: gpu_sweep.sh VAR v1 [v2 ...]: bench (tunes, saves the table), then one bench per VAR=v on that table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
VAR=$1; shift
echo "== bench (tunes)"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py --verbose > gpurun_out/bench_s0.log 2>&1 || { tail -30 gpurun_out/bench_s0.log; exit 1; }
tail -1 gpurun_out/bench_s0.log | cut -c1-200
for v in "$@"; do
  echo "== bench $VAR=$v"
  env $VAR=$v MXR_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py > gpurun_out/bench_s_$v.log 2>&1 || { tail -30 gpurun_out/bench_s_$v.log; exit 1; }
  tail -1 gpurun_out/bench_s_$v.log | cut -c1-200
done
