#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for e in "X=1" "MXR_COMM_TORCH_STREAM=1" "MXR_COMM_TORCH_STREAM=1 MXR_COMM_SKIP_RCCL=1" "MXR_COMM_SKIP_RCCL=1"; do
  echo "== $e"; env $e timeout -k 10 100 python scripts/probe_rccl.py native 2>&1 | grep "native  *chain_with\|buckets_only" || exit 1
done
