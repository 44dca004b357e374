#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash scripts/gpu_ab.sh MXR_CONV_EXCLUDE=miopen && \
  { echo "== op sources"; timeout -k 10 300 python scripts/op_sources.py > gpurun_out/op_sources.log 2>&1; rc=$?; head -60 gpurun_out/op_sources.log; exit $rc; }
