#!/bin/bash
# Real-JPEG training throughput (VERDICT r3 Next #7): a COCO-layout JPEG fixture (scripts/make_coco_fixture.py)
# through train.py's host pipeline -- worker processes decode into shared memory, device preprocessing --
# at WORKERS (default "2 4 8"), next to bench.py's device-synthetic number on the same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
FIX=/tmp/mxr_coco_fixture
timeout -k 10 300 python -u scripts/make_coco_fixture.py $FIX --n ${NIMG:-1024} --workers 16 || exit 1
echo "cpus visible: $(nproc)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/jpeg_bench_ref.log 2>&1 || { tail -5 gpurun_out/jpeg_bench_ref.log; exit 1; }
echo "bench.py: $(tail -1 gpurun_out/jpeg_bench_ref.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], "img/s", r["ms_per_step"], "ms/step")')"
for W in ${WORKERS:-2 4 8}; do
  timeout -k 10 400 python -u -m batchai_retinanet_horovod_coco_amd.bin.train --bench 5 20 --workers $W \
    --device-preprocess --loader process --batch-size 16 --no-weights --calibrate-bn --clip-mode global \
    --no-evaluation --tensorboard-dir '' coco $FIX > gpurun_out/jpeg_w$W.log 2>&1 || { echo "workers $W rc=$?"; tail -20 gpurun_out/jpeg_w$W.log; exit 1; }
  echo "workers $W: $(grep '^{' gpurun_out/jpeg_w$W.log | tail -1)"
done
