#!/bin/bash
# Diagnose the process loader at W workers: CPU / thread snapshot of every process while train.py --bench runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
FIX=/tmp/mxr_coco_fixture
timeout -k 10 300 python -u scripts/make_coco_fixture.py $FIX --n ${NIMG:-512} --workers 16 > /dev/null || exit 1
W=${W:-8}
MXR_STACK_DUMP=${DUMP:-} timeout -k 10 ${LIM:-240} python -u -m batchai_retinanet_horovod_coco_amd.bin.train --bench ${BENCH:-5 20} --workers $W \
    --device-preprocess --loader process --batch-size 16 --no-weights --calibrate-bn --clip-mode global \
    --no-evaluation --tensorboard-dir '' coco $FIX > gpurun_out/jpeg_diag.log 2>&1 &
PID=$!
for t in ${TS:-40 70 100}; do
  sleep 30
  echo "== t=${t}s"
  ps -eo pid,ppid,nlwp,pcpu,rss,stat,comm --sort=-pcpu | head -14
  for p in $(ps -eo pid,comm | awk '$2=="python"{print $1}'); do
    n=$(ls -l /proc/$p/fd 2>/dev/null | grep -c kfd); echo "pid $p kfd_fds=$n threads=$(ls /proc/$p/task 2>/dev/null | wc -l)"
  done
done
wait $PID; rc=$?
echo "rc=$rc"; tail -3 gpurun_out/jpeg_diag.log
