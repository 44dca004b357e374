#!/bin/bash
# tuning-noise study: 3 fresh tunings (tables saved), then each table re-run once
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2 3; do
  MXR_SAVE_CONV_TABLE=gpurun_out/tbl_$i.json timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/tbl_tune_$i.log 2>&1 || { echo "rc=$?"; exit 1; }
  echo "tune $i: $(tail -1 gpurun_out/tbl_tune_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
for i in 1 2 3; do
  MXR_CONV_TABLE=gpurun_out/tbl_$i.json timeout -k 10 300 python bench.py --steps 30 --warmup 3 > gpurun_out/tbl_run_$i.log 2>&1 || { echo "rc=$?"; exit 1; }
  echo "table $i: $(tail -1 gpurun_out/tbl_run_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
