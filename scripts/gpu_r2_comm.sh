#!/bin/bash
# Round 2: native comm engine tests + full GPU suite + default bench (native engine is only used at world>1)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== native comm tests"
timeout -k 10 300 python -u -m pytest tests/test_native_comm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_comm.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_comm.log
[ $rc -ne 0 ] && exit $rc
echo "== full gpu suite"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
echo "== bench 1 GPU with the native engine forced (one-rank communicator: comm timing evidence)"
MXR_COMM=native timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_native1.log 2>&1; rc=$?
tail -1 gpurun_out/bench_native1.log | cut -c1-2000
exit $rc
