#!/bin/bash
# Host C++ runtime under AddressSanitizer + UndefinedBehaviorSanitizer: build the sanitized
# libmxr_cpu.so and run the tests that exercise it (every entry point + data pipeline + IO) with the
# sanitizer runtimes preloaded.  CPU only -- no GPU sanitizers on this pool.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
python -m batchai_retinanet_horovod_coco_amd.build --sanitize > /dev/null || exit 1
export MXR_CPU_LIB=$PWD/batchai_retinanet_horovod_coco_amd/_lib/asan/libmxr_cpu.so
ASAN_RT=$(gcc -print-file-name=libasan.so)
UBSAN_RT=$(gcc -print-file-name=libubsan.so)
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export PYTHONFAULTHANDLER=1
LD_PRELOAD="$ASAN_RT $UBSAN_RT" timeout -k 10 900 python -m pytest tests/test_cpu_native.py tests/test_data_io.py \
    -q -p no:cacheprovider -m "not gpu" "$@"
