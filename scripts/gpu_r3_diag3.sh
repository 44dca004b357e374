#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/bench_halo.py --pipe "" --halo "" --hx32 "6,120,121,122,123,108,124" --only head_256 > gpurun_out/bench_hx32_diag3.log 2>&1; rc=$?
cat gpurun_out/bench_hx32_diag3.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 bash scripts/gpu_r3_pmc.sh "fwd hx32_6" "fwd hx32_120"
