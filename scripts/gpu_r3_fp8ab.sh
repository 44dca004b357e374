#!/bin/bash
# same-box A/B: bf16 bench, fp8 bench, then a kernel-trace profile of the fp8 run
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for d in bf16 fp8; do
  MXR_SAVE_CONV_TABLE=gpurun_out/conv_table_$d.json timeout -k 10 400 python -u bench.py --dtype $d > gpurun_out/bench_$d.log 2> gpurun_out/bench_$d.err || { echo "bench $d rc=$?"; tail -20 gpurun_out/bench_$d.err; exit 1; }
  echo "$d $(python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$d.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
MXR_CONV_TABLE=$R/gpurun_out/conv_table_fp8.json timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_fp8 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3 --dtype fp8 > $R/gpurun_out/prof_fp8.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $R/gpurun_out/prof_fp8.log; exit 1; }
python3 $R/scripts/steady_kernels.py $R/gpurun_out/prof_fp8/run_kernel_trace.csv 3 45 > $R/gpurun_out/steady_fp8.txt && head -60 $R/gpurun_out/steady_fp8.txt
