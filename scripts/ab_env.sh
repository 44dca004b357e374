#!/bin/bash
# Same-box A/B of environment settings on the driver-equivalent bench (fresh tuning per run):
#   bash scripts/ab_env.sh "MXR_WGRAD_HX_BLOCKS=256" "MXR_WGRAD_HX_BLOCKS=192" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for spec in "$@"; do
  env $spec timeout -k 10 400 python -u bench.py > gpurun_out/ab_bench.log 2> gpurun_out/ab_bench.err || { echo "$spec: rc=$?"; tail -5 gpurun_out/ab_bench.err; exit 1; }
  echo "$spec: $(tail -1 gpurun_out/ab_bench.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], "img/s", r["ms_per_step"], "ms/step")')"
done
