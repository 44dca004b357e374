"""Deterministic toy COCO GT / detection set for the evaluator's 12-stat fixture (tests/test_coco_eval.py):
4 categories over 12 images, boxes in all three area ranges, crowd regions, explicit ``ignore`` flags, images
with detections but no GT and GT but no detections, duplicate detections, score ties and more than 100
detections on one image (the maxDets cut)."""
import numpy as np


def build(seed: int = 7):
    rng = np.random.RandomState(seed)
    images = [{"id": i + 1, "width": 640, "height": 480} for i in range(12)]
    cats = [{"id": c} for c in (1, 3, 7, 11)]
    anns, dets = [], []
    aid = 1
    for img in images:
        if img["id"] == 5:
            continue                      # no GT at all: its detections are all false positives
        for _ in range(rng.randint(1, 9)):
            side = rng.choice([12.0, 24.0, 48.0, 80.0, 160.0])
            w, h = side * rng.uniform(0.6, 1.4), side * rng.uniform(0.6, 1.4)
            x, y = rng.uniform(0, 640 - w), rng.uniform(0, 480 - h)
            crowd = int(rng.rand() < 0.08)
            a = {"id": aid, "image_id": img["id"], "category_id": int(rng.choice([1, 3, 7, 11])),
                 "bbox": [round(x, 2), round(y, 2), round(w, 2), round(h, 2)], "area": round(w * h * 0.9, 2),
                 "iscrowd": crowd}
            if rng.rand() < 0.05:
                a["ignore"] = 1
            anns.append(a)
            aid += 1
    for a in anns:
        if a["image_id"] == 9:
            continue                      # GT but no detections
        for _ in range(rng.randint(0, 3)):
            x, y, w, h = a["bbox"]
            j = rng.normal(0, 0.06 * max(w, h), 4)
            dets.append({"image_id": a["image_id"], "category_id": a["category_id"] if rng.rand() < 0.85 else 3,
                         "bbox": [x + j[0], y + j[1], max(1.0, w + j[2]), max(1.0, h + j[3])],
                         "score": float(np.round(rng.uniform(0.05, 1.0), 2))})     # rounded: score ties
    for img in images:
        for _ in range(rng.randint(0, 6) + (120 if img["id"] == 2 else 0)):
            w, h = rng.uniform(8, 200), rng.uniform(8, 200)
            dets.append({"image_id": img["id"], "category_id": int(rng.choice([1, 3, 7, 11])),
                         "bbox": [rng.uniform(0, 600), rng.uniform(0, 440), w, h],
                         "score": float(np.round(rng.uniform(0.05, 0.7), 2))})
    return {"images": images, "categories": cats, "annotations": anns}, dets
