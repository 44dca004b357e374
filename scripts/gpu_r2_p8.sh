#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== p8/p4 tests"
timeout -k 10 300 python -u -m pytest tests/test_p8_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_p8.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_p8.log
[ $rc -ne 0 ] && exit $rc
echo "== microbench"
timeout -k 10 300 python scripts/bench_p8.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench_p8.log || exit 1
echo "== pmc"
bash scripts/gpu_pmc_p8.sh
