#!/bin/bash
# Pipelined wgrad validation: build, GPU tests, conv microbench, PMC on head wgrad, bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
export PYTHONFAULTHANDLER=1
python -m batchai_retinanet_horovod_coco_amd.build || exit 1
echo "== pytest gpu"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc -> stop"; exit $rc; fi
echo "== conv microbench"
timeout -k 10 500 python scripts/bench_conv.py > gpurun_out/bench_conv.log 2>&1 || { echo "bench_conv rc=$?"; tail -20 gpurun_out/bench_conv.log; exit 1; }
cat gpurun_out/bench_conv.log
echo "== pmc"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for spec in "wgrad 3" "wgrad 4"; do
  set -- $spec
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d $R/gpurun_out/pmc/$1_$2_a -o run --output-format csv -- python3 $R/scripts/pmc_conv.py --op $1 --variant $2 > $R/gpurun_out/pmc/$1_$2_a.log 2>&1 || { echo "pmc rc=$?"; tail -5 $R/gpurun_out/pmc/$1_$2_a.log; exit 1; }
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc/$1_$2_b -o run --output-format csv -- python3 $R/scripts/pmc_conv.py --op $1 --variant $2 > $R/gpurun_out/pmc/$1_$2_b.log 2>&1 || { echo "pmc rc=$?"; tail -5 $R/gpurun_out/pmc/$1_$2_b.log; exit 1; }
done
cd $R
echo "== bench"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 400 python bench.py --steps 10 --warmup 3 --verbose > gpurun_out/bench_hip.log 2>&1 || { echo "bench rc=$?"; tail -30 gpurun_out/bench_hip.log; exit 1; }
tail -2 gpurun_out/bench_hip.log
