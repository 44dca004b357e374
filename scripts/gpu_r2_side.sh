#!/bin/bash
# side-stream wgrad: ordering tests, then bench A/B (same tuned table) with it off / on
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== tests"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_side_stream_gpu.py > gpurun_out/pytest_side.log 2>&1 || { tail -40 gpurun_out/pytest_side.log; exit 1; }
tail -5 gpurun_out/pytest_side.log
echo "== bench (tunes, side on)"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py --verbose "$@" > gpurun_out/bench_side1.log 2>&1 || { tail -30 gpurun_out/bench_side1.log; exit 1; }
tail -1 gpurun_out/bench_side1.log | cut -c1-400
echo "== bench side off (same table)"
MXR_SIDE_WGRAD=0 MXR_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py "$@" > gpurun_out/bench_side0.log 2>&1 || { tail -30 gpurun_out/bench_side0.log; exit 1; }
tail -1 gpurun_out/bench_side0.log | cut -c1-400
echo "== bench side on (same table)"
MXR_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py "$@" > gpurun_out/bench_side1b.log 2>&1 || { tail -30 gpurun_out/bench_side1b.log; exit 1; }
tail -1 gpurun_out/bench_side1b.log | cut -c1-400
