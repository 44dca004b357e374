#!/bin/bash
# same-box sweep of the side-stream wgrad split-K grid target (MXR_WGRAD_PIPE_BLOCKS; VAR=MXR_WGRAD_HEAD_BLOCKS: the packed
# head layers only), bench.py defaults (+ ARGS, e.g. "--dtype fp8"); BLOCKS / REPS override the lists
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=${VAR:-MXR_WGRAD_PIPE_BLOCKS}
for rep in ${REPS:-1 2}; do
  for B in ${BLOCKS:-192 144 240 288}; do
    env $V=$B timeout -k 10 400 python -u bench.py ${ARGS:-} > gpurun_out/sw_${B}_${rep}.log 2> gpurun_out/sw_err.log || { echo "rc=$?"; tail -5 gpurun_out/sw_err.log; exit 1; }
    echo "blocks $B rep $rep: $(tail -1 gpurun_out/sw_${B}_${rep}.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"])')"
  done
done
