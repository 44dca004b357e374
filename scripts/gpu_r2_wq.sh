#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/pytest_wq.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_wq.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/bench_p8.py wgrad 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench_wq.log
