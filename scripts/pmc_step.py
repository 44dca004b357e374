#!/usr/bin/env python
"""Hardware counters of the training step, per kernel: MFMA busy, LDS bank-conflict share, HBM bytes.

Runs ``bench.py`` (pinned conv table, a few steps) once per counter pass under
``rocprofv3 --kernel-trace --pmc`` -- each pass a child process with its own time limit, the
program itself right after ``--`` -- and joins the passes by kernel name:

    python scripts/pmc_step.py run --out gpurun_out/pmc_step [--top 12] [-- extra bench.py args]
    python scripts/pmc_step.py summarize gpurun_out/pmc_step [--top 12]

Derived columns (per dispatch, averaged over the dispatches of a kernel):

* ``mfma``  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)
* ``ldsc``  = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (share of LDS-active cycles lost to conflicts)
* ``rd/wr`` = 2 x FETCH_SIZE and WRITE_SIZE in MB (gfx950 FETCH_SIZE tallies a 128-B streaming request as
  64 B: MI355X_MICROARCH.md §HBM; Infinity-Cache hits are counted too), ``TB/s`` = (rd + wr) / duration
* ``wait`` = SQ_WAIT_ANY / SQ_WAVE_CYCLES, ``l2hit`` = TCC_HIT / (TCC_HIT + TCC_MISS)

Counter-slot limits per pass (gfx950): 8 SQ, 4 TCC (FETCH_SIZE takes 3, WRITE_SIZE 2), 2 GRBM.
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import subprocess
import sys
from collections import defaultdict

PASSES = [
    "SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES "
    "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE",
    "FETCH_SIZE GRBM_GUI_ACTIVE",
    "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum",
    "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE",
]


def short(name: str) -> str:
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:70]


def run(args, extra) -> int:
    here = os.path.dirname(os.path.abspath(__file__))
    bench = os.path.join(os.path.dirname(here), "bench.py")
    out = os.path.abspath(args.out)
    os.makedirs(out, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    # the children run in /tmp: the pinned table path must be absolute (else the tuner re-times everything)
    env["MXR_CONV_TABLE"] = os.path.abspath(env.get("MXR_CONV_TABLE") or
                                            os.path.join(os.path.dirname(here), "tuning", "conv_table.json"))
    for i, grp in enumerate(PASSES):
        d = os.path.join(out, "pass%d" % i)
        cmd = ["timeout", "-s", "KILL", str(args.timeout), "rocprofv3", "--kernel-trace", "--pmc"] + grp.split() + \
              ["-d", d, "-o", "run", "--output-format", "csv", "--", sys.executable, bench,
               "--steps", str(args.steps), "--warmup", str(args.warmup)] + extra
        print("pass", i, grp, flush=True)
        with open(os.path.join(out, "pass%d.log" % i), "w") as log:
            rc = subprocess.call(cmd, cwd="/tmp", env=env, stdout=log, stderr=subprocess.STDOUT)
        if rc != 0:
            print("pass %d failed rc=%d (see %s/pass%d.log)" % (i, rc, out, i), flush=True)
            return rc
    summarize(out, args.top, args.steps)
    if not args.keep_raw:
        import shutil
        for i in range(len(PASSES)):
            shutil.rmtree(os.path.join(out, "pass%d" % i), ignore_errors=True)
    return 0


def _steady(ids_names, steps):
    """Dispatch ids of the last ``steps`` training steps (a step ends at the fused Adam kernel)."""
    ids_names = sorted(ids_names)
    ends = [i for i, (_, n) in enumerate(ids_names) if "adam_kernel" in n]
    if len(ends) < steps + 1:
        return {d for d, _ in ids_names}
    return {d for d, _ in ids_names[ends[-steps - 1] + 1:ends[-1] + 1]}


def load(out, steps):
    vals = defaultdict(lambda: defaultdict(list))     # kernel -> counter -> [per-dispatch values]
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(out, "pass*", "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        meta = {}
        for r in csv.DictReader(open(f)):
            key = (int(r["Dispatch_Id"]), r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            meta[int(r["Dispatch_Id"])] = r["Kernel_Name"]
        keep = _steady(meta.items(), steps)
        for (d, c), v in per.items():
            if d in keep:
                vals[short(meta[d])][c].append(v)
    for f in glob.glob(os.path.join(out, "pass0", "**", "*kernel_trace.csv"), recursive=True):
        rows = [(int(r["Dispatch_Id"]), r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                for r in csv.DictReader(open(f))]
        keep = _steady([(d, n) for d, n, _ in rows], steps)
        for d, n, t in rows:
            if d in keep:
                dur[short(n)].append(t * 1e-3 / steps)
    return vals, dur


def summarize(out, top=12, steps=3):
    vals, dur = load(out, steps)
    tot = {k: sum(v) for k, v in dur.items()}
    allt = sum(tot.values()) or 1.0
    rows = sorted(tot, key=lambda k: -tot[k])[:top]
    m = lambda k, c: (sum(vals[k][c]) / len(vals[k][c])) if vals[k].get(c) else float("nan")   # noqa: E731
    hdr = "{:>6} {:>5} {:>6} {:>5} {:>5} {:>5} {:>8} {:>8} {:>6} {:>5} {:>5}  {}".format(
        "us", "n", "share", "mfma", "ldsc", "wait", "rd MB", "wr MB", "TB/s", "l2hit", "GHz", "kernel")
    lines = ["# per-kernel hardware counters over the last %d training steps (scripts/pmc_step.py); n = dispatches "
             "per step, us = per dispatch (counters serialize the dispatches: isolated-kernel times); GHz = "
             "GRBM_GUI_ACTIVE / 8 XCDs / duration: the shader clock the power limit left the kernel" % steps, hdr]
    for k in rows:
        n = len(dur[k]) / steps           # dispatches per step
        us = tot[k] / len(dur[k]) * steps  # per dispatch
        grbm = m(k, "GRBM_GUI_ACTIVE")
        mf = m(k, "SQ_VALU_MFMA_BUSY_CYCLES") / (1024 * grbm / 8) if grbm == grbm and grbm > 0 else float("nan")
        idx = m(k, "SQ_LDS_IDX_ACTIVE")
        ldsc = m(k, "SQ_LDS_BANK_CONFLICT") / idx if idx and idx == idx else float("nan")
        wc = m(k, "SQ_WAVE_CYCLES")
        wait = m(k, "SQ_WAIT_ANY") / wc if wc and wc == wc else float("nan")
        rd = 2 * m(k, "FETCH_SIZE") / 1024.0      # FETCH_SIZE / WRITE_SIZE are in KB
        wr = m(k, "WRITE_SIZE") / 1024.0
        tbs = (rd + wr) * 1e6 / (us * 1e6) if us > 0 else float("nan")
        h, mi = m(k, "TCC_HIT_sum"), m(k, "TCC_MISS_sum")
        l2 = h / (h + mi) if (h + mi) > 0 else float("nan")
        ghz = grbm / 8 / (us * 1e-6) / 1e9 if grbm == grbm and us > 0 else float("nan")
        lines.append("{:6.1f} {:5.0f} {:5.1f}% {:5.2f} {:5.3f} {:5.2f} {:8.1f} {:8.1f} {:6.2f} {:5.2f} {:5.2f}  {}".format(
            us, n, 100 * tot[k] / allt, mf, ldsc, wait, rd, wr, tbs, l2, ghz, k))
    text = "\n".join(lines)
    print(text)
    with open(os.path.join(out, "summary.txt"), "w") as f:
        f.write(text + "\n")


def main():
    argv = sys.argv[1:]
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["run", "summarize"])
    ap.add_argument("out", nargs="?", default=None)
    ap.add_argument("--out", dest="out_opt", default="gpurun_out/pmc_step")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("--keep-raw", action="store_true", help="keep the per-pass csv files (large)")
    a = ap.parse_args(argv)
    a.out = a.out or a.out_opt
    if a.mode == "run":
        return run(a, extra)
    summarize(a.out, a.top, a.steps)
    return 0


if __name__ == "__main__":
    sys.exit(main())
