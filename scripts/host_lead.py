#!/usr/bin/env python
"""How far ahead of the GPU the host is through a step: for every 12th kernel of the second-to-last
step of a rocprofv3 --kernel-trace --hip-runtime-trace run, (GPU start - host launch).  A lead near zero
means the GPU is waiting for the host's launches there.

usage: host_lead.py run_kernel_trace.csv run_hip_api_trace.csv[.gz] [every=12]"""
import csv
import gzip
import sys


def main():
    kt, ht = sys.argv[1], sys.argv[2]
    every = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    op = gzip.open if ht.endswith(".gz") else open
    api = {r["Correlation_Id"]: int(r["Start_Timestamp"]) for r in csv.DictReader(op(ht, "rt"))}
    kl = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:45], r["Correlation_Id"],
                 r["Queue_Id"]) for r in csv.DictReader(open(kt)))
    ad = [i for i, k in enumerate(kl) if k[2].startswith("(anonymous namespace)::adam_kernel")]
    a, b = ad[-3], ad[-2]
    t0 = kl[a][1]
    low = 0
    for i in range(a, b + 1):
        s, e, n, c, q = kl[i]
        if c in api and s - api[c] < 200000:
            low += 1
        if (i - a) % every == 0 and c in api:
            print("%7.2f ms  q%s lead %7.2f ms  %s" % ((s - t0) / 1e6, q, (s - api[c]) / 1e6, n))
    print("kernels launched < 0.2 ms before they started: %d of %d" % (low, b - a))


if __name__ == "__main__":
    main()
