#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
timeout -k 10 300 python -u -m pytest tests/test_halo_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_halo.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_halo.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/bench_p8.py 2>&1 | grep -v amdgpu.ids | grep pyramid | tee gpurun_out/bench_halo.log
