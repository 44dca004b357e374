#!/usr/bin/env python
"""Stream overlap of the last steps of a rocprofv3 --kernel-trace run: wall time, GPU-busy time (union of
kernel intervals), kernel-time sum (> busy when streams overlap), idle gaps, and busy time per stream.

usage: [TOPK=n] trace_overlap.py run_kernel_trace.csv [steps=3] [step_marker=adam_kernel] [run_hip_api_trace.csv]
TOPK: also the n largest kernels (summed time) of each queue
A step ends at each kernel whose name contains ``step_marker`` (the fused Adam kernel, once per step).  With the HIP
API trace, each large gap also says whether the kernel after it was launched by the host only after the
GPU went idle ("host late": the host was behind) or before ("queued": a dependency / stream wait)."""
import csv
import sys
from collections import defaultdict


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    marker = sys.argv[3] if len(sys.argv) > 3 else "adam_kernel"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"],
                         r.get("Correlation_Id")))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if marker in r[2]]
    if len(ends) < steps + 1:
        print("only %d step markers" % len(ends))
        return
    a, b = ends[-steps - 1] + 1, ends[-1] + 1
    win = rows[a:b]
    t0, t1 = win[0][0], max(r[1] for r in win)
    wall = t1 - t0
    busy = union([(s, e) for s, e, _, _, _ in win])
    ksum = sum(e - s for s, e, _, _, _ in win)
    print("steps %d  wall %.2f ms/step  busy %.2f ms/step (%.1f %%)  kernel-sum %.2f ms/step  overlap x%.2f"
          % (steps, wall / steps / 1e6, busy / steps / 1e6, 100.0 * busy / wall, ksum / steps / 1e6, ksum / max(busy, 1)))
    per_q = defaultdict(list)
    for s, e, n, q, _ in win:
        per_q[q].append((s, e))
    per_qk = defaultdict(lambda: defaultdict(float))
    for s, e, n, q, _ in win:
        per_qk[q][n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:90]] += e - s
    top = int(__import__("os").environ.get("TOPK", "0"))
    for q, iv in sorted(per_q.items()):
        print("  queue %s: %d kernels, busy %.2f ms/step" % (q, len(iv), union(iv) / steps / 1e6))
        for n, t in sorted(per_qk[q].items(), key=lambda kv: -kv[1])[:top]:
            print("      %7.3f ms/step  %s" % (t / steps / 1e6, n))
    launch = {}
    if len(sys.argv) > 4:
        with open(sys.argv[4]) as f:
            for r in csv.DictReader(f):
                if "Launch" in r.get("Function", ""):
                    launch[r["Correlation_Id"]] = int(r["Start_Timestamp"])
    gaps = []
    last_e, prev = t0, ""
    for s, e, n, q, cid in win:
        if s > last_e:
            gaps.append((s - last_e, n, prev, last_e, launch.get(cid)))
        if e >= last_e:
            prev = n
        last_e = max(last_e, e)
    gaps.sort(reverse=True)
    print("  idle %.2f ms/step in %d gaps; largest before:" % (sum(g[0] for g in gaps) / steps / 1e6, len(gaps)))
    late = sum(g[0] for g in gaps if g[4] is not None and g[4] > g[3])
    if launch:
        print("  of which host-late (next kernel launched after the GPU went idle): %.2f ms/step" % (late / steps / 1e6))
    for g, n, p, ge, lt in gaps[:int(__import__("os").environ.get("GAPS", "12"))]:
        tag = "" if lt is None else ("host late %+.0f us" % ((lt - ge) / 1e3) if lt > ge else "queued")
        print("    %7.1f us  %-18s %s  <-  %s" % (g / 1e3, tag, n[:70], p[:60]))


if __name__ == "__main__":
    main()
