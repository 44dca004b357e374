#!/bin/bash
# wgrad numerics (unit + production-shape winners) -> default bench (fresh tuning, table saved) -> op sources
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_kernels_gpu.py tests/test_winners_gpu.py} > gpurun_out/pytest_iter.log 2>&1; rc=$?
tail -6 gpurun_out/pytest_iter.log
[ $rc -ne 0 ] && exit $rc
echo "== bench"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py --verbose $BENCH_ARGS > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-400
if [ -n "$OPS" ]; then
  echo "== op sources"
  MXR_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 300 python scripts/op_sources.py > gpurun_out/op_sources.log 2>&1 || { tail -20 gpurun_out/op_sources.log; exit 1; }
  grep -v Warning gpurun_out/op_sources.log | head -60
fi
