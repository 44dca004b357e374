"""COCO bbox evaluation (pycocotools ``COCOeval`` semantics, no pycocotools needed).

Reference: ``CocoEval`` callback (``/root/reference/train.py:135-138``) -> keras-retinanet
``evaluate_coco``: run the prediction model on every validation image, rescale boxes to the
original image, write ``<set>_bbox_results.json``, and compute the 12 COCO stats.

:class:`COCOeval` re-implements the bbox path of pycocotools: 10 IoU thresholds (.50:.05:.95),
101 recall points, maxDets (1, 10, 100), area ranges all/small/medium/large, crowd gt handled as
"ignore" with the intersection-over-detection-area IoU, greedy score-ordered matching, interpolated precision.
The IoU and the matching are native C++ (``csrc/cpu/runtime_cpu.cpp``: ``mxr_cpu_coco_iou``,
``mxr_cpu_coco_match``); see :class:`COCOeval` for the structure.
"""
from __future__ import annotations

import json
from collections import defaultdict
from typing import Dict, List, Optional

import numpy as np

from ..utils import cpu_native

STAT_NAMES = [
    "AP @[ IoU=0.50:0.95 | area=   all | maxDets=100 ]",
    "AP @[ IoU=0.50      | area=   all | maxDets=100 ]",
    "AP @[ IoU=0.75      | area=   all | maxDets=100 ]",
    "AP @[ IoU=0.50:0.95 | area= small | maxDets=100 ]",
    "AP @[ IoU=0.50:0.95 | area=medium | maxDets=100 ]",
    "AP @[ IoU=0.50:0.95 | area= large | maxDets=100 ]",
    "AR @[ IoU=0.50:0.95 | area=   all | maxDets=  1 ]",
    "AR @[ IoU=0.50:0.95 | area=   all | maxDets= 10 ]",
    "AR @[ IoU=0.50:0.95 | area=   all | maxDets=100 ]",
    "AR @[ IoU=0.50:0.95 | area= small | maxDets=100 ]",
    "AR @[ IoU=0.50:0.95 | area=medium | maxDets=100 ]",
    "AR @[ IoU=0.50:0.95 | area= large | maxDets=100 ]",
]


class Params:
    def __init__(self):
        self.imgIds: List[int] = []
        self.catIds: List[int] = []
        self.iouThrs = np.linspace(.5, 0.95, int(np.round((0.95 - .5) / .05)) + 1, endpoint=True)
        self.recThrs = np.linspace(.0, 1.00, int(np.round((1.00 - .0) / .01)) + 1, endpoint=True)
        self.maxDets = [1, 10, 100]
        self.areaRng = [[0 ** 2, 1e5 ** 2], [0 ** 2, 32 ** 2], [32 ** 2, 96 ** 2], [96 ** 2, 1e5 ** 2]]
        self.areaRngLbl = ["all", "small", "medium", "large"]
        self.useCats = 1


def load_results(coco_gt, results: List[Dict]):
    """``COCO.loadRes`` for bbox results: returns a CocoIndex with areas and ids filled in."""
    from ..data.coco import CocoIndex
    anns = []
    for i, r in enumerate(results):
        x, y, w, h = r["bbox"]
        a = dict(r)
        a["area"] = w * h
        a["id"] = i + 1
        a["iscrowd"] = 0
        anns.append(a)
    ds = {"images": list(coco_gt.dataset.get("images", [])), "categories": list(coco_gt.dataset.get("categories", [])),
          "annotations": anns}
    return CocoIndex(dataset=ds)


class _PairEval:
    """Per (image, category) evaluation record: detections in score order (cut at maxDet), and for every area range
    the (T, D) match / ignore masks and the number of regular gts."""
    __slots__ = ("scores", "matched", "dt_ignore", "n_gt")

    def __init__(self, scores, matched, dt_ignore, n_gt):
        self.scores, self.matched, self.dt_ignore, self.n_gt = scores, matched, dt_ignore, n_gt


class COCOeval:
    """bbox COCOeval: the 12 summary statistics of pycocotools' ``COCOeval(..., 'bbox')``.

    Re-designed rather than transcribed: each (image, category) pair is read ONCE -- detections stably sorted by
    score and cut at the largest maxDet, one native IoU matrix -- and the four area ranges reuse that matrix through a
    gt column order (regular gts first); the greedy matching of all ten IoU thresholds runs in C++
    (``mxr_cpu_coco_match``), and ``accumulate`` builds the precision envelope, recall and the 101-point sampling as
    array operations over the thresholds.  Semantics kept from pycocotools: gts with ``ignore`` / ``iscrowd`` or an
    area outside the range are ignored, crowd gts may be matched repeatedly, a detection never trades a regular gt for
    an ignored one, unmatched detections outside the area range are ignored, and ties in score break by image order
    then detection order (stable sorts).  Parity against pycocotools itself is unpinned (not installed here); the toy
    fixture in tests/test_coco_eval.py pins the 12 numbers of the previous, line-by-line formulation.
    """

    def __init__(self, cocoGt, cocoDt, iouType: str = "bbox"):
        if iouType != "bbox":
            raise NotImplementedError("only bbox evaluation is implemented")
        self.cocoGt, self.cocoDt = cocoGt, cocoDt
        self.params = Params()
        self.params.imgIds = sorted(cocoGt.getImgIds())
        self.params.catIds = sorted(cocoGt.getCatIds())
        self.pairs: Dict[tuple, _PairEval] = {}
        self.eval = {}
        self.stats = np.zeros(12)

    @staticmethod
    def _group(index, imgs, cats):
        out = defaultdict(list)
        for a in index.anns.values():              # insertion order: the detection order ties fall back on
            if a["image_id"] in imgs and a["category_id"] in cats:
                out[a["image_id"], a["category_id"]].append(a)
        return out

    def evaluate(self):
        p = self.params
        p.imgIds = [int(i) for i in np.unique(p.imgIds)]
        p.maxDets = sorted(p.maxDets)
        imgs, cats = set(p.imgIds), set(p.catIds)
        gts = self._group(self.cocoGt, imgs, cats)
        dts = self._group(self.cocoDt, imgs, cats)
        thr = np.asarray(p.iouThrs, dtype=np.float64)
        rng = np.asarray(p.areaRng, dtype=np.float64)
        max_det = p.maxDets[-1]
        self.pairs = {}
        for key in set(gts) | set(dts):
            g, d = gts.get(key, []), dts.get(key, [])
            g_box = np.array([a["bbox"] for a in g], dtype=np.float64).reshape(-1, 4)
            g_area = np.array([a["area"] if "area" in a else a["bbox"][2] * a["bbox"][3] for a in g], dtype=np.float64)
            g_flag = np.array([bool(a.get("ignore", 0) or a.get("iscrowd", 0)) for a in g], dtype=bool)
            crowd = np.array([int(a.get("iscrowd", 0)) for a in g], dtype=np.uint8)
            score = np.array([a["score"] for a in d], dtype=np.float64)
            keep = np.argsort(-score, kind="stable")[:max_det]
            score = score[keep]
            d_box = np.array([d[i]["bbox"] for i in keep], dtype=np.float64).reshape(-1, 4)
            d_area = np.array([d[i]["area"] for i in keep], dtype=np.float64)
            iou = cpu_native.coco_iou(d_box, g_box, crowd)
            per_range = []
            for lo, hi in rng:
                ig = g_flag | (g_area < lo) | (g_area > hi)
                order = np.argsort(ig, kind="stable").astype(np.int32)
                ig_o = ig[order]
                m = cpu_native.coco_match(iou, order, ig_o, crowd, thr)
                matched = m >= 0
                dt_ig = np.where(matched, ig_o[np.maximum(m, 0)] if len(g) else False, False)
                out = (d_area < lo) | (d_area > hi)
                dt_ig = dt_ig | (~matched & out[None, :])
                per_range.append((matched, dt_ig, int(np.count_nonzero(~ig))))
            self.pairs[key] = _PairEval(score, [r[0] for r in per_range], [r[1] for r in per_range],
                                        [r[2] for r in per_range])

    def accumulate(self):
        p = self.params
        T, R, K, A, M = len(p.iouThrs), len(p.recThrs), len(p.catIds), len(p.areaRng), len(p.maxDets)
        precision = -np.ones((T, R, K, A, M))
        recall = -np.ones((T, K, A, M))
        scores = -np.ones((T, R, K, A, M))
        rec_thr = np.asarray(p.recThrs)
        for k, cat in enumerate(p.catIds):
            recs = [self.pairs[i, cat] for i in p.imgIds if (i, cat) in self.pairs]   # image order: tie breaks
            if not recs:
                continue
            for a in range(A):
                n_gt = sum(r.n_gt[a] for r in recs)
                if n_gt == 0:
                    continue
                for mi, md in enumerate(p.maxDets):
                    sc = np.concatenate([r.scores[:md] for r in recs])
                    order = np.argsort(-sc, kind="stable")
                    sc = sc[order]
                    hit = np.concatenate([r.matched[a][:, :md] for r in recs], axis=1)[:, order]
                    ign = np.concatenate([r.dt_ignore[a][:, :md] for r in recs], axis=1)[:, order]
                    tp = np.cumsum(hit & ~ign, axis=1, dtype=np.float64)
                    fp = np.cumsum(~hit & ~ign, axis=1, dtype=np.float64)
                    nd = sc.shape[0]
                    if nd == 0:
                        recall[:, k, a, mi] = 0
                        precision[:, :, k, a, mi] = 0
                        scores[:, :, k, a, mi] = 0
                        continue
                    rc = tp / n_gt
                    pr = tp / (tp + fp + np.spacing(1))
                    pr = np.maximum.accumulate(pr[:, ::-1], axis=1)[:, ::-1]     # precision envelope
                    recall[:, k, a, mi] = rc[:, -1]
                    for t in range(T):
                        idx = np.searchsorted(rc[t], rec_thr, side="left")
                        ok = idx < nd
                        q = np.zeros(R)
                        ss = np.zeros(R)
                        q[ok] = pr[t, idx[ok]]
                        ss[ok] = sc[idx[ok]]
                        precision[t, :, k, a, mi] = q
                        scores[t, :, k, a, mi] = ss
        self.eval = {"params": p, "counts": [T, R, K, A, M], "precision": precision, "recall": recall,
                     "scores": scores}

    def _summarize(self, ap=1, iouThr=None, areaRng="all", maxDets=100):
        p = self.params
        aind = [i for i, a in enumerate(p.areaRngLbl) if a == areaRng]
        mind = [i for i, m in enumerate(p.maxDets) if m == maxDets]
        if ap == 1:
            s = self.eval["precision"]
            if iouThr is not None:
                s = s[np.where(iouThr == p.iouThrs)[0]]
            s = s[:, :, :, aind, mind]
        else:
            s = self.eval["recall"]
            if iouThr is not None:
                s = s[np.where(iouThr == p.iouThrs)[0]]
            s = s[:, :, aind, mind]
        return -1 if len(s[s > -1]) == 0 else float(np.mean(s[s > -1]))

    def summarize(self, verbose: bool = True):
        m = self.params.maxDets
        self.stats = np.array([
            self._summarize(1, maxDets=m[2]), self._summarize(1, iouThr=.5, maxDets=m[2]),
            self._summarize(1, iouThr=.75, maxDets=m[2]), self._summarize(1, areaRng="small", maxDets=m[2]),
            self._summarize(1, areaRng="medium", maxDets=m[2]), self._summarize(1, areaRng="large", maxDets=m[2]),
            self._summarize(0, maxDets=m[0]), self._summarize(0, maxDets=m[1]), self._summarize(0, maxDets=m[2]),
            self._summarize(0, areaRng="small", maxDets=m[2]), self._summarize(0, areaRng="medium", maxDets=m[2]),
            self._summarize(0, areaRng="large", maxDets=m[2])])
        if verbose:
            for name, v in zip(STAT_NAMES, self.stats):
                print(" Average {:<18} = {:0.3f}".format(name.replace(" @", "").split("[")[0].strip() and name, v))
        return self.stats


def predict_image(generator, prediction_model, index: int, device=None):
    """Load/preprocess/resize one image, run the prediction model, return boxes in image coords."""
    import torch
    image = generator.load_image(index)
    image = generator.preprocess_image(image)
    image, scale = generator.resize_image(image)
    dev = device or next(prediction_model.model.parameters()).device
    dt = getattr(prediction_model, "compute_dtype", None) or (torch.bfloat16 if dev.type == "cuda" else torch.float32)
    x = torch.from_numpy(image[None]).to(dev).to(dt)
    boxes, scores, labels = prediction_model(x)
    boxes = boxes[0].float().cpu().numpy() / scale
    return boxes, scores[0].float().cpu().numpy(), labels[0].cpu().numpy()


def evaluate_coco(generator, prediction_model, threshold: float = 0.05, results_path: Optional[str] = None,
                  verbose: bool = True):
    results, image_ids = [], []
    for index in range(generator.size()):
        boxes, scores, labels = predict_image(generator, prediction_model, index)
        boxes[:, 2] -= boxes[:, 0]
        boxes[:, 3] -= boxes[:, 1]
        for box, score, label in zip(boxes, scores, labels):
            if score < threshold:
                break
            results.append({"image_id": generator.image_ids[index],
                            "category_id": generator.label_to_coco_label(int(label)),
                            "score": float(score), "bbox": [float(v) for v in box]})
        image_ids.append(generator.image_ids[index])
    if not results:
        return None
    path = results_path or "{}_bbox_results.json".format(generator.set_name)
    with open(path, "w") as f:
        json.dump(results, f, indent=4)
    with open("{}_processed_image_ids.json".format(path.replace("_bbox_results.json", "")), "w") as f:
        json.dump(image_ids, f, indent=4)
    coco_pred = load_results(generator.coco, results)
    ev = COCOeval(generator.coco, coco_pred, "bbox")
    ev.params.imgIds = image_ids
    ev.evaluate()
    ev.accumulate()
    ev.summarize(verbose)
    return ev.stats
