#!/usr/bin/env python
"""Write a COCO-layout JPEG fixture (no dataset is reachable offline): ``<root>/images/<set>/*.jpg`` of
COCO-like sizes (``--sizes coco``: the ten most common COCO train2017 sizes -- 640 x 480 / 480 x 640,
640 x 427 / 427 x 640, 640 x 426, 640 x 360, 500 x 375 / 375 x 500, 640 x 512, 612 x 612 -- ten aspect ratios;
``--sizes two``: 640 x 480 and 480 x 640 only), smooth random content, PIL quality 90, ~60 KB
like COCO's JPEGs) and ``<root>/annotations/instances_<set>.json`` with 1-12 random boxes per image over the
80 COCO category ids (1..90 with COCO's gaps) -- the layout ``data/coco.py`` reads
(``/root/reference/train.py:197-214``).  Used by scripts/gpu_jpeg_pipeline.sh for the real-JPEG training
throughput (``train.py --bench ... coco <root>``).

usage: make_coco_fixture.py ROOT [--n 512] [--set train2017] [--workers 8] [--sizes coco|two]"""
import argparse
import json
import multiprocessing as mp
import os

import numpy as np

# (h, w), most frequent first (weights roughly COCO's)
SIZES = {"coco": [(480, 640)] * 6 + [(640, 480)] * 2 + [(427, 640)] * 2 + [(640, 427), (426, 640), (360, 640),
                                                                        (375, 500), (500, 375), (512, 640),
                                                                        (612, 612)],
         "two": [(480, 640), (480, 640), (640, 480)]}
COCO_IDS = [i for i in range(1, 91) if i not in (12, 26, 29, 30, 45, 66, 68, 69, 71, 83)]


def _write(args):
    path, h, w, seed = args
    from PIL import Image
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (h // 16, w // 16, 3), dtype=np.uint8)
    Image.fromarray(base).resize((w, h), Image.BILINEAR).save(path, quality=90)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--set", default="train2017")
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--sizes", choices=sorted(SIZES), default="coco")
    a = ap.parse_args()
    img_dir = os.path.join(a.root, "images", a.set)
    os.makedirs(img_dir, exist_ok=True)
    os.makedirs(os.path.join(a.root, "annotations"), exist_ok=True)
    rng = np.random.default_rng(1)
    images, anns, jobs = [], [], []
    aid = 1
    for i in range(a.n):
        h, w = SIZES[a.sizes][int(rng.integers(0, len(SIZES[a.sizes])))]
        fn = "%012d.jpg" % (i + 1)
        images.append({"id": i + 1, "file_name": fn, "height": h, "width": w})
        jobs.append((os.path.join(img_dir, fn), h, w, i))
        for _ in range(int(rng.integers(1, 13))):
            bw, bh = float(rng.uniform(8, w / 2)), float(rng.uniform(8, h / 2))
            x0, y0 = float(rng.uniform(0, w - bw)), float(rng.uniform(0, h - bh))
            anns.append({"id": aid, "image_id": i + 1, "category_id": int(rng.choice(COCO_IDS)),
                         "bbox": [x0, y0, bw, bh], "area": bw * bh, "iscrowd": 0})
            aid += 1
    cats = [{"id": c, "name": "class_%d" % c, "supercategory": "none"} for c in COCO_IDS]
    with open(os.path.join(a.root, "annotations", "instances_%s.json" % a.set), "w") as f:
        json.dump({"images": images, "annotations": anns, "categories": cats}, f)
    with mp.get_context("fork").Pool(a.workers) as pool:
        pool.map(_write, jobs, chunksize=8)
    kb = sum(os.path.getsize(j[0]) for j in jobs) / len(jobs) / 1024
    print("fixture %s: %d images (%.0f KiB each), %d boxes" % (a.root, a.n, kb, len(anns)))


if __name__ == "__main__":
    main()
