#!/usr/bin/env python
"""JPEG decode throughput of the loader (data.image.read_image_bgr = PIL decode + BGR flip) on a
PIL-generated COCO-sized fixture set: images/sec for one process and for N worker processes.
usage: bench_decode.py [--n 64] [--workers 1,2,4,8] [--hw 480,640]"""
import argparse
import multiprocessing as mp
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.data.image import read_image_bgr  # noqa: E402


def _decode(paths):
    n = 0
    for p in paths:
        n += read_image_bgr(p).shape[0] > 0
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--workers", default="1,2,4,8")
    ap.add_argument("--hw", default="480,640")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from PIL import Image
    h, w = (int(v) for v in a.hw.split(","))
    d = tempfile.mkdtemp(prefix="mxr_jpeg_")
    rng = np.random.default_rng(0)
    paths = []
    for i in range(a.n):
        # smooth random content (JPEG of pure noise is unrealistically large)
        base = rng.integers(0, 256, (h // 16, w // 16, 3), dtype=np.uint8)
        img = Image.fromarray(base).resize((w, h), Image.BILINEAR)
        p = os.path.join(d, "%04d.jpg" % i)
        img.save(p, quality=90)
        paths.append(p)
    mb = sum(os.path.getsize(p) for p in paths) / a.n / 1024
    print("fixture: %d JPEGs %dx%d, %.0f KiB each, cpus %d" % (a.n, w, h, mb, os.cpu_count()))
    ctx = mp.get_context("forkserver")
    for k in [int(v) for v in a.workers.split(",")]:
        best = 0.0
        for _ in range(a.reps):
            if k == 1:
                t0 = time.perf_counter()
                _decode(paths)
                el = time.perf_counter() - t0
            else:
                with ctx.Pool(k) as pool:
                    pool.map(_decode, [paths[:2]] * k)          # warm the workers
                    chunks = [paths[i::k] for i in range(k)]
                    t0 = time.perf_counter()
                    pool.map(_decode, chunks)
                    el = time.perf_counter() - t0
            best = max(best, a.n / el)
        print("workers %2d: %7.1f images/s decoded (%.1f per worker)" % (k, best, best / k), flush=True)
    for p in paths:
        os.remove(p)
    os.rmdir(d)


if __name__ == "__main__":
    main()
