#!/bin/bash
# Run-to-run spread on one box: three driver-equivalent bench.py runs, each with fresh tuning (tables saved as gpurun_out/t*.json)
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  MXR_SAVE_CONV_TABLE=gpurun_out/t$i.json timeout -k 10 400 python -u bench.py > gpurun_out/v$i.log 2> gpurun_out/v$i.err || exit 1
  echo "fresh $i: $(tail -1 gpurun_out/v$i.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
done
for i in 1 2 3; do
  MXR_CONV_TABLE=$PWD/gpurun_out/t$i.json timeout -k 10 400 python -u bench.py > gpurun_out/p$i.log 2> gpurun_out/p$i.err || exit 1
  echo "pinned t$i: $(tail -1 gpurun_out/p$i.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
done
