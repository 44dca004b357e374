#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/bench_halo.py --pipe "" --halo "" --hx32 "${V:-2,108,116,124,132,148}" --only "${ONLY:-head}" > gpurun_out/bench_hx32_diag2.log 2>&1; rc=$?
cat gpurun_out/bench_hx32_diag2.log
exit $rc
