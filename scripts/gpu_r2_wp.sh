#!/bin/bash
# production-shape numerics of the committed table's winners -> rocprof kernel trace (steady-state table)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
R=$GRAFT_REPO_ROOT
T=${TABLE:-$R/tuning/conv_table.json}
if [ -z "$SKIP_WINNERS" ]; then
echo "== winners"
MXR_WINNER_TABLE=$T timeout -k 10 500 python -u -m pytest tests/test_winners_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/winners.log 2>&1; rc=$?
tail -15 gpurun_out/winners.log
[ $rc -gt 1 ] && exit $rc
fi
echo "== rocprof trace"
cd /tmp && export TMPDIR=/tmp
MXR_CONV_TABLE=$T timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/ktrace -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 3 "$@" > $R/gpurun_out/ktrace.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $R/gpurun_out/ktrace.log; exit 1; }
tail -1 $R/gpurun_out/ktrace.log | cut -c1-300
KT=$(ls $R/gpurun_out/ktrace/*kernel_trace.csv $R/gpurun_out/ktrace/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 $R/scripts/steady_kernels.py $KT 5 40 > $R/gpurun_out/steady.txt; head -70 $R/gpurun_out/steady.txt
gzip -f $KT
