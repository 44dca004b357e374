#!/bin/bash
# halo kernel: numerics tests, then fwd/dgrad microbench against the pipelined kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== pytest halo"
timeout -k 10 300 python -u -m pytest tests/test_halo_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_halo.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_halo.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc -> stop"; exit $rc; fi
echo "== bench halo"
timeout -k 10 300 python -u scripts/bench_halo.py > gpurun_out/bench_halo.log 2>&1; rc=$?
cat gpurun_out/bench_halo.log
exit $rc
