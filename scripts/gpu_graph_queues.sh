#!/bin/bash
# graph replay at batch 16 vs eager, with the HIP runtime's graph execution queue count forced (ROCm maps the
# captured step onto its own streams: by default the side-stream branch mostly lands on the compute queue)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {
  env $1 timeout -k 10 300 python -u bench.py $2 > gpurun_out/gq.log 2> gpurun_out/gq.err || { echo "$1 $2 rc=$?"; tail -5 gpurun_out/gq.err; exit 1; }
  echo "[$1 $2] $(tail -1 gpurun_out/gq.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], "img/s", r["ms_per_step"], "ms/step")')"
}
for rep in 1 2; do
  run "MXR_X=0" ""
  for q in ${QUEUES:-2 4}; do run "DEBUG_HIP_FORCE_GRAPH_QUEUES=$q" "--graph"; done
done
