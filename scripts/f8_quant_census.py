#!/usr/bin/env python
"""Which tensors still take a standalone fp8 quantisation pass (amax + quant) in an fp8 training step:
wraps ops.fp8.quantize / quantize_bf8, runs bench.py --dtype fp8 in-process, and prints per call site
(shape, callers) the count per step.

usage: f8_quant_census.py [bench args...]"""
import collections
import os
import runpy
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import fp8 as F8  # noqa: E402

SEEN = collections.Counter()


def wrap(name):
    real = getattr(F8, name)

    def f(x, *a, **k):
        st = [fr for fr in traceback.extract_stack()[:-1] if "batchai_retinanet" in fr.filename]
        site = " <- ".join("%s:%d %s" % (os.path.basename(fr.filename), fr.lineno, fr.name) for fr in st[-4:][::-1])
        SEEN[(name, tuple(x.shape), str(x.dtype), site)] += 1
        return real(x, *a, **k)
    setattr(F8, name, f)


for n in ("quantize", "quantize_bf8"):
    wrap(n)
steps = 4
sys.argv = ["bench.py", "--dtype", "fp8", "--steps", str(steps), "--warmup", "3"] + sys.argv[1:]
try:
    runpy.run_path(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"),
                   run_name="__main__")
finally:
    tot = steps + 3
    print("fp8 quantisation passes (count over %d steps incl. tuning):" % tot)
    for (name, shape, dt, site), c in SEEN.most_common():
        print("%4d  %-13s %-22s %s\n       %s" % (c, name, shape, dt, site))
