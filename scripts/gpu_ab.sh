#!/bin/bash
# A/B end-to-end benches on ONE box with the committed tuner table (box-to-box variance is large).
# Usage: AB="label1:ENV=val,ENV2=val;label2:ENV=val" bash scripts/gpu_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
python -m batchai_retinanet_horovod_coco_amd.build || exit 1
echo "== pytest gpu"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then tail -40 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc -> stop"; exit $rc; fi
IFS=';' read -ra ARMS <<< "${AB:-base:}"
for rep in 1 2; do
  for arm in "${ARMS[@]}"; do
    label="${arm%%:*}"; envs="${arm#*:}"
    echo "== bench $label (rep $rep) [$envs]"
    ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
      timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_${label}_${rep}.log 2>&1 ) || { echo "bench rc=$?"; tail -20 gpurun_out/bench_${label}_${rep}.log; exit 1; }
    tail -1 gpurun_out/bench_${label}_${rep}.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], 'img/s', d['ms_per_step'], 'ms/step')"
  done
done
