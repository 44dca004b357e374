#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_pyr
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY"
G2="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
G3="FETCH_SIZE GRBM_GUI_ACTIVE"
G4="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
SPECS=("$@")
[ ${#SPECS[@]} -eq 0 ] && SPECS=("fwd halo12" "fwd p8_5" "fwd halo7" "wgrad 23" "wgrad 20")
TAGS=""
for spec in "${SPECS[@]}"; do
  set -- $spec
  tag=$1_$2
  TAGS="$TAGS $tag"
  for gi in ${PMC_GROUPS:-1 2}; do
    eval G=\$G$gi
    timeout -s KILL 90 rocprofv3 --pmc $G -d $R/gpurun_out/pmc_pyr/${tag}_$gi -o run --output-format csv -- python3 $R/scripts/pmc_pyr.py $1 $2 > $R/gpurun_out/pmc_pyr/${tag}_$gi.log 2>&1 || { echo "pmc $tag $gi failed"; tail -5 $R/gpurun_out/pmc_pyr/${tag}_$gi.log; exit 1; }
  done
done
TAGS="$TAGS" python3 - <<'PY'
import csv, glob, collections, os
R = os.environ["GRAFT_REPO_ROOT"]
for tag in os.environ["TAGS"].split():
    acc = collections.defaultdict(float); disp = collections.defaultdict(set); dur = {}
    for f in glob.glob(R + "/gpurun_out/pmc_pyr/%s_*/**/run_counter_collection.csv" % tag, recursive=True):
        for r in csv.DictReader(open(f)):
            kn = r["Kernel_Name"]
            if not ("conv" in kn and "kernel" in kn):
                continue
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
    print("==", tag)
    vals = {k: acc[k] / max(1, len(disp[k])) for k in acc}
    for k in sorted(vals):
        print("  %-26s per-dispatch %.4g" % (k, vals[k]))
    if "SQ_VALU_MFMA_BUSY_CYCLES" in vals and "GRBM_GUI_ACTIVE" in vals:
        print("  MFMA busy / (SIMD x cycles) = %.3f" % (vals["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (vals["GRBM_GUI_ACTIVE"] / 8)))
    if "TCC_HIT_sum" in vals:
        print("  L2 hit rate = %.3f" % (vals["TCC_HIT_sum"] / max(1.0, vals["TCC_HIT_sum"] + vals["TCC_MISS_sum"])))
    if "SQ_WAIT_ANY" in vals:
        print("  WAIT_ANY / WAVE_CYCLES = %.3f   WAIT_INST_ANY / WAVE_CYCLES = %.3f" % (
            vals["SQ_WAIT_ANY"] / vals["SQ_WAVE_CYCLES"], vals.get("SQ_WAIT_INST_ANY", 0) / vals["SQ_WAVE_CYCLES"]))
PY
