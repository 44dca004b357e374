#!/bin/bash
# same-box A/B of scheduling knobs against the default bench: "NAME=VALUE ..." per arm (ARMS, ; separated)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table_ab.json timeout -k 10 400 python -u bench.py > gpurun_out/ab_0.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/ab_0.log; exit 1; }
echo "default: $(grep -o '"value": [0-9.]*' gpurun_out/ab_0.log)"
i=1
IFS=';' read -ra A <<< "$ARMS"
for arm in "${A[@]}"; do
  env $arm MXR_CONV_TABLE=gpurun_out/conv_table_ab.json timeout -k 10 300 python -u bench.py > gpurun_out/ab_$i.log 2>&1 || { echo "arm $arm rc=$?"; tail -20 gpurun_out/ab_$i.log; exit 1; }
  echo "$arm: $(grep -o '"value": [0-9.]*' gpurun_out/ab_$i.log)"
  i=$((i+1))
done
MXR_CONV_TABLE=gpurun_out/conv_table_ab.json timeout -k 10 300 python -u bench.py > gpurun_out/ab_last.log 2>&1 && echo "default (pinned table) again: $(grep -o '"value": [0-9.]*' gpurun_out/ab_last.log)"
