#!/bin/bash
# build -> GPU tests -> conv microbench -> bench with a FRESH tuner table (saved) -> bench with that table
# -> rocprof kernel stats with that table.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
python -m batchai_retinanet_horovod_coco_amd.build > /dev/null || exit 1
echo "== pytest gpu"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; echo "pytest rc=$rc -> stop"; exit $rc; fi
echo "== conv microbench"
timeout -k 10 600 python scripts/bench_conv.py > gpurun_out/bench_conv.log 2>&1 || { echo "bench_conv rc=$?"; tail -20 gpurun_out/bench_conv.log; exit 1; }
grep TOTALS gpurun_out/bench_conv.log
echo "== bench (fresh tuning)"
MXR_CONV_TABLE=none MXR_CONV_TUNE_REPS=3 MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_tune.log 2>&1 || { echo "bench rc=$?"; tail -30 gpurun_out/bench_tune.log; exit 1; }
tail -1 gpurun_out/bench_tune.log
echo "== bench (saved table)"
MXR_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 300 python bench.py > gpurun_out/bench_table.log 2>&1 || { echo "bench rc=$?"; tail -30 gpurun_out/bench_table.log; exit 1; }
tail -1 gpurun_out/bench_table.log
echo "== rocprof"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
MXR_CONV_TABLE=$R/gpurun_out/conv_table.json timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_hip -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3 > $R/gpurun_out/prof_hip.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $R/gpurun_out/prof_hip.log; exit 1; }
python3 $R/scripts/prof_summary.py $R/gpurun_out/prof_hip/run_kernel_stats.csv --steps 6 > $R/gpurun_out/prof_summary.txt && head -16 $R/gpurun_out/prof_summary.txt
