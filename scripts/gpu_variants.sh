#!/bin/bash
# bench variants on one box: eager (saved tuning table reused), HIP graph, fp8 forward
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "== eager (tune + save table)"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table_v.json timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/v_eager.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/v_eager.log; exit 1; }
tail -1 gpurun_out/v_eager.log | cut -c1-200
echo "== graph (same table)"
MXR_CONV_TABLE=gpurun_out/conv_table_v.json timeout -k 10 400 python bench.py --steps 20 --warmup 3 --graph > gpurun_out/v_graph.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/v_graph.log; exit 1; }
tail -1 gpurun_out/v_graph.log | cut -c1-200
echo "== eager again (same table)"
MXR_CONV_TABLE=gpurun_out/conv_table_v.json timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/v_eager2.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/v_eager2.log; exit 1; }
tail -1 gpurun_out/v_eager2.log | cut -c1-200
echo "== fp8"
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --dtype fp8 > gpurun_out/v_fp8.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/v_fp8.log; exit 1; }
tail -1 gpurun_out/v_fp8.log | cut -c1-200
