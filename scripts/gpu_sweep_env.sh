#!/bin/bash
# bench.py under several values of one env var: SWEEP_VAR=name SWEEP_VALS="a b c"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in $SWEEP_VALS; do
  echo "== $SWEEP_VAR=$v"
  env "$SWEEP_VAR=$v" timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/sweep_$v.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/sweep_$v.log; exit 1; }
  tail -1 gpurun_out/sweep_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
