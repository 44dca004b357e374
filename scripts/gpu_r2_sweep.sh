#!/bin/bash
# bench under several environment settings (fresh tuning each): VALUES="K1=a,K2=b K1=c ..." (one run per token)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
i=0
for v in $VALUES; do
  i=$((i+1))
  echo "== $v"
  env ${v//,/ } timeout -k 10 400 python bench.py $BENCH_ARGS > gpurun_out/sweep_$i.log 2>&1 || { tail -20 gpurun_out/sweep_$i.log; exit 1; }
  tail -1 gpurun_out/sweep_$i.log | grep -o '"value": [0-9.]*, "unit": "[^"]*", "n_gpus": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*'
done
