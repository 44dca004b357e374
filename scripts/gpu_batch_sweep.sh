#!/bin/bash
# Small per-rank batches (the reference job runs --batch-size 1 per rank, train.py:365): bench.py eager vs
# --graph at B = 1 / 2 / 4 (and 16) for 800x1333 and 800x1067, plus the host issue cost of each eager step.
#   BATCHES="1 2 4" SIZES="800x1333 800x1067" bash scripts/gpu_batch_sweep.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/batch_sweep.txt
: > $OUT
for hw in ${SIZES:-800x1333 800x1067}; do
  H=${hw%x*}; W=${hw#*x}
  for B in ${BATCHES:-1 2 4}; do
    for mode in eager graph; do
      flag=""; [ $mode = graph ] && flag="--graph"
      timeout -k 10 300 python -u bench.py --batch-size $B --height $H --width $W --steps ${STEPS:-50} --warmup 5 $flag \
          > gpurun_out/bs.log 2> gpurun_out/bs.err || { echo "B=$B $hw $mode rc=$?"; tail -20 gpurun_out/bs.err; exit 1; }
      echo "B=$B $hw $mode: $(tail -1 gpurun_out/bs.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], "img/s", r["ms_per_step"], "ms/step")')" | tee -a $OUT
    done
    timeout -k 10 300 python -u scripts/host_time.py 3 --batch-size $B --height $H --width $W 2>&1 | tail -1 | tee -a $OUT || exit 1
  done
done
