#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== host profile"
timeout -k 10 300 python scripts/host_profile.py 60 > gpurun_out/host_profile.txt 2>&1 || { tail -30 gpurun_out/host_profile.txt; exit 1; }
grep -A75 "Ordered by: internal time" gpurun_out/host_profile.txt | head -75
bash scripts/gpu_ab.sh MXR_AUTOGRAD_MT=0
