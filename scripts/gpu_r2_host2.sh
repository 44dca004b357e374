#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== bench"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-200
echo "== host issue per step"
MXR_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 300 python scripts/sync_probe.py > gpurun_out/sync_probe.log 2>&1 || { tail -20 gpurun_out/sync_probe.log; exit 1; }
grep "^step\|num_device" gpurun_out/sync_probe.log
echo "== host profile"
MXR_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 300 python scripts/host_profile.py 50 > gpurun_out/host_profile.txt 2>&1 || { tail -30 gpurun_out/host_profile.txt; exit 1; }
grep -A55 "Ordered by: internal time" gpurun_out/host_profile.txt | head -55 | cut -c1-150
