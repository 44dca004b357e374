#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_halo_gpu.py -x -q -k "hx32" --timeout 120 --timeout-method thread > gpurun_out/pytest_hx32.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_hx32.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/bench_halo.py --pipe "" --halo "${HALO:-7}" --hx32 "${V:-0,1,2,3,101,102,103,108,111}" --only "${ONLY:-}" > gpurun_out/bench_hx32_diag4.log 2>&1; rc=$?
cat gpurun_out/bench_hx32_diag4.log
exit $rc
