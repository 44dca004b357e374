#!/bin/bash
# Why is the one-rank native engine slower than no reduction? A/B of comm-stream priority / event timing + kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export MXR_CONV_TABLE=$GRAFT_REPO_ROOT/tuning/conv_table_r2_387.json
run() { echo "== $1"; shift; env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }; tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config'].get('comm_engine'), d['config'].get('comm_ms'))"; }
run torch MXR_COMM=torch
run native MXR_COMM=native
run native_prio_normal MXR_COMM=native MXR_COMM_PRIORITY=normal
run native_notiming MXR_COMM=native MXR_COMM_TIMING=0
run native_nowatchdog MXR_COMM=native MXR_COMM_TIMEOUT=0
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
MXR_COMM=native timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_native -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3 > $R/gpurun_out/prof_native.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $R/gpurun_out/prof_native.log; exit 1; }
python3 $R/scripts/prof_summary.py $R/gpurun_out/prof_native/run_kernel_stats.csv --steps 6 > $R/gpurun_out/prof_native_summary.txt && head -30 $R/gpurun_out/prof_native_summary.txt
