#!/bin/bash
# training throughput WITH the host data pipeline (Generator: random transform, resize to 800x1333,
# batching, enqueuer threads) -- train.py --bench on the synthetic dataset, batch 16
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
for w in ${WORKERS:-4 8}; do
  echo "== workers $w $EXTRA"
  timeout -k 10 500 python -m batchai_retinanet_horovod_coco_amd.bin.train --no-weights --calibrate-bn --batch-size 16 \
    --dtype bf16 --random-transform --workers $w $EXTRA --bench 5 20 synthetic --num-images ${NIMG:-128} --height 800 --width 1333 \
    > gpurun_out/hostpipe_$w.log 2>&1 || { tail -20 gpurun_out/hostpipe_$w.log; exit 1; }
  grep -o '{"metric".*' gpurun_out/hostpipe_$w.log | tail -1
done
