#!/bin/bash
# bench under a few values of one environment knob (fresh tuning each): KNOB=name VALUES="a b c"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
for v in $VALUES; do
  echo "== $KNOB=$v"
  env $KNOB=$v timeout -k 10 400 python bench.py $BENCH_ARGS > gpurun_out/sweep_$v.log 2>&1 || { tail -20 gpurun_out/sweep_$v.log; exit 1; }
  tail -1 gpurun_out/sweep_$v.log | cut -c1-260
done
