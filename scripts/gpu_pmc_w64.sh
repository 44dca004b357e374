#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/scripts/bench_w64.py || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY -d $R/gpurun_out/pmc_w64 -o run --output-format csv -- python3 $R/scripts/bench_w64.py > $R/gpurun_out/pmc_w64.log 2>&1 || { tail -5 $R/gpurun_out/pmc_w64.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections, os
R = os.environ["GRAFT_REPO_ROOT"]
f = glob.glob(R + "/gpurun_out/pmc_w64/**/run_counter_collection.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
acc = collections.defaultdict(float); n = collections.Counter()
for r in rows:
    if "wgrad3x3" not in r["Kernel_Name"]:
        continue
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(acc):
    print("%-24s %.4g (per dispatch %.4g)" % (k, acc[k], acc[k] / max(1, n[k] / 1)))
PY
