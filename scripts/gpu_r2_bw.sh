#!/bin/bash
# default bench (fresh tuning, table saved) -> production-shape numerics of that table's winners -> rocprof
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== bench"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py --verbose "$@" > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-1500
echo "== winners"
MXR_WINNER_TABLE=gpurun_out/conv_table.json timeout -k 10 500 python -u -m pytest tests/test_winners_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/winners.log 2>&1; rc=$?
tail -8 gpurun_out/winners.log
[ $rc -ne 0 ] && exit $rc
echo "== rocprof"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
MXR_CONV_TABLE=$R/gpurun_out/conv_table.json timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3 "$@" > $R/gpurun_out/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $R/gpurun_out/prof.log; exit 1; }
python3 $R/scripts/prof_summary.py $R/gpurun_out/prof/run_kernel_stats.csv --steps 6 > $R/gpurun_out/prof_summary.txt && head -40 $R/gpurun_out/prof_summary.txt
