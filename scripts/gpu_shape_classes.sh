#!/bin/bash
# Real COCO-shaped batches at steady-state speed (VERDICT r4 Next #2): a ten-size COCO-layout JPEG fixture
# (scripts/make_coco_fixture.py --sizes coco) through train.py --bench with 2 decode workers, for each
# --pad-multiple in PADS (default "0 32 128"): value vs steady_value, raced / borrowed tuner keys, batch shapes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
FIX=/tmp/mxr_coco_fixture10
timeout -k 10 300 python -u scripts/make_coco_fixture.py $FIX --n ${NIMG:-2048} --workers 16 --sizes coco || exit 1
for P in ${PADS:-0 32 128}; do
  [ -n "$ALLOC" ] && export PYTORCH_HIP_ALLOC_CONF=$ALLOC
  timeout -k 10 ${RUN_TIMEOUT:-500} python -u -m batchai_retinanet_horovod_coco_amd.bin.train --bench ${WARM:-5} ${STEPS:-100} \
    --workers ${WORKERS:-2} --device-preprocess --loader process --batch-size 16 --no-weights --calibrate-bn \
    --clip-mode global --no-evaluation --tensorboard-dir '' --pad-multiple $P coco $FIX > gpurun_out/shapes_p$P.log 2>&1 \
    || { echo "pad $P rc=$?"; tail -20 gpurun_out/shapes_p$P.log; exit 1; }
  echo "pad $P: $(grep '^{' gpurun_out/shapes_p$P.log | tail -1)"
done
