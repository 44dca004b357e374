#!/bin/bash
# First GPU contact: device info, pure-PyTorch (MIOpen) baseline, kernel-trace profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
python -c "import torch;print(torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0))" || exit 1
echo "== bench immediate-mode MIOpen (no find)"
MXR_CUDNN_BENCHMARK=0 timeout -k 10 420 python bench.py --steps 10 --warmup 3 --verbose > gpurun_out/bench_torch_immediate.log 2>&1; echo "exit $?"; tail -3 gpurun_out/bench_torch_immediate.log
echo "== bench MIOpen find mode"
MXR_CUDNN_BENCHMARK=1 timeout -k 10 600 python bench.py --steps 10 --warmup 3 --verbose > gpurun_out/bench_torch_find.log 2>&1; echo "exit $?"; tail -3 gpurun_out/bench_torch_find.log
