#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== bench eager (tunes)"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py > gpurun_out/bench_e.log 2>&1 || { tail -30 gpurun_out/bench_e.log; exit 1; }
tail -1 gpurun_out/bench_e.log | cut -c1-300
echo "== bench graph"
MXR_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py --graph --verbose > gpurun_out/bench_g.log 2>&1 || { tail -30 gpurun_out/bench_g.log; exit 1; }
tail -1 gpurun_out/bench_g.log | cut -c1-300
grep warmup gpurun_out/bench_g.log | tail -3
echo "== bench graph fp8"
MXR_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py --graph --dtype fp8 > gpurun_out/bench_g8.log 2>&1 || { tail -30 gpurun_out/bench_g8.log; exit 1; }
tail -1 gpurun_out/bench_g8.log | cut -c1-300
