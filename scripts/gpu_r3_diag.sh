#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/bench_halo.py --pipe "" --halo "7" --hx32 "2,4,5,100,101,102" > gpurun_out/bench_hx32_diag.log 2>&1; rc=$?
cat gpurun_out/bench_hx32_diag.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 bash scripts/gpu_r3_pmc.sh "fwd hx32_2" "fwd halo7" "fwd hx32_100"
