"""COCO bbox evaluation (pycocotools ``COCOeval`` semantics, no pycocotools needed).

Reference: ``CocoEval`` callback (``/root/reference/train.py:135-138``) -> keras-retinanet
``evaluate_coco``: run the prediction model on every validation image, rescale boxes to the
original image, write ``<set>_bbox_results.json``, and compute the 12 COCO stats.

:class:`COCOeval` re-implements the bbox path of pycocotools: 10 IoU thresholds (.50:.05:.95),
101 recall points, maxDets (1, 10, 100), area ranges all/small/medium/large, crowd gt handled as
"ignore" with the intersection-over-detection-area IoU (native C++ IoU in
``csrc/cpu/runtime_cpu.cpp``), greedy score-ordered matching, interpolated precision.
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


class COCOeval:
    def __init__(self, cocoGt, cocoDt, iouType: str = "bbox"):
        if iouType != "bbox":
            raise NotImplementedError("only bbox evaluation is implemented")
        self.cocoGt, self.cocoDt = cocoGt, cocoDt
        self.params = Params()
        self.params.imgIds = sorted(cocoGt.getImgIds())
        self.params.catIds = sorted(cocoGt.getCatIds())
        self.evalImgs = []
        self.eval = {}
        self.stats = np.zeros(12)

    def _prepare(self):
        p = self.params
        self._gts = defaultdict(list)
        self._dts = defaultdict(list)
        imgs = set(p.imgIds)
        cats = set(p.catIds)
        for a in self.cocoGt.anns.values():
            if a["image_id"] in imgs and a["category_id"] in cats:
                g = dict(a)
                g.setdefault("area", g["bbox"][2] * g["bbox"][3])
                g["ignore"] = g.get("ignore", 0) or g.get("iscrowd", 0)
                self._gts[g["image_id"], g["category_id"]].append(g)
        for a in self.cocoDt.anns.values():
            if a["image_id"] in imgs and a["category_id"] in cats:
                self._dts[a["image_id"], a["category_id"]].append(a)

    def evaluate(self):
        p = self.params
        p.imgIds = list(np.unique(p.imgIds))
        p.maxDets = sorted(p.maxDets)
        self._prepare()
        maxDet = p.maxDets[-1]
        self.evalImgs = [self.evaluateImg(imgId, catId, areaRng, maxDet)
                         for catId in p.catIds for areaRng in p.areaRng for imgId in p.imgIds]

    def computeIoU(self, gt, dt):
        if len(gt) == 0 or len(dt) == 0:
            return np.zeros((len(dt), len(gt)))
        g = np.array([x["bbox"] for x in gt], dtype=np.float64)
        d = np.array([x["bbox"] for x in dt], dtype=np.float64)
        crowd = [int(o.get("iscrowd", 0)) for o in gt]
        return cpu_native.coco_iou(d, g, crowd)

    def evaluateImg(self, imgId, catId, aRng, maxDet):
        p = self.params
        gt = self._gts[imgId, catId]
        dt = self._dts[imgId, catId]
        if len(gt) == 0 and len(dt) == 0:
            return None
        for g in gt:
            g["_ignore"] = 1 if (g["ignore"] or (g["area"] < aRng[0] or g["area"] > aRng[1])) else 0
        gtind = np.argsort([g["_ignore"] for g in gt], kind="mergesort")
        gt = [gt[i] for i in gtind]
        dtind = np.argsort([-d["score"] for d in dt], kind="mergesort")
        dt = [dt[i] for i in dtind[0:maxDet]]
        iscrowd = [int(o.get("iscrowd", 0)) for o in gt]
        ious = self.computeIoU(gt, dt)
        T, G, D = len(p.iouThrs), len(gt), len(dt)
        gtm = np.zeros((T, G))
        dtm = np.zeros((T, D))
        gtIg = np.array([g["_ignore"] for g in gt])
        dtIg = np.zeros((T, D))
        if len(ious):
            for tind, t in enumerate(p.iouThrs):
                for dind, d in enumerate(dt):
                    iou = min([t, 1 - 1e-10])
                    m = -1
                    for gind, g in enumerate(gt):
                        if gtm[tind, gind] > 0 and not iscrowd[gind]:
                            continue
                        if m > -1 and gtIg[m] == 0 and gtIg[gind] == 1:
                            break
                        if ious[dind, gind] < iou:
                            continue
                        iou = ious[dind, gind]
                        m = gind
                    if m == -1:
                        continue
                    dtIg[tind, dind] = gtIg[m]
                    dtm[tind, dind] = gt[m]["id"]
                    gtm[tind, m] = d["id"]
        a = np.array([d["area"] < aRng[0] or d["area"] > aRng[1] for d in dt]).reshape((1, len(dt)))
        dtIg = np.logical_or(dtIg, np.logical_and(dtm == 0, np.repeat(a, T, 0)))
        return {"image_id": imgId, "category_id": catId, "aRng": aRng, "maxDet": maxDet,
                "dtIds": [d["id"] for d in dt], "gtIds": [g["id"] for g in gt], "dtMatches": dtm, "gtMatches": gtm,
                "dtScores": [d["score"] for d in dt], "gtIgnore": gtIg, "dtIgnore": dtIg}

    def accumulate(self):
        p = self.params
        T, R, K, A, M = len(p.iouThrs), len(p.recThrs), len(p.catIds), len(p.areaRng), len(p.maxDets)
        precision = -np.ones((T, R, K, A, M))
        recall = -np.ones((T, K, A, M))
        scores = -np.ones((T, R, K, A, M))
        I0, A0 = len(p.imgIds), len(p.areaRng)
        for k in range(K):
            Nk = k * A0 * I0
            for a in range(A):
                Na = a * I0
                for m, maxDet in enumerate(p.maxDets):
                    E = [self.evalImgs[Nk + Na + i] for i in range(I0)]
                    E = [e for e in E if e is not None]
                    if len(E) == 0:
                        continue
                    dtScores = np.concatenate([e["dtScores"][0:maxDet] for e in E])
                    inds = np.argsort(-dtScores, kind="mergesort")
                    dtScoresSorted = dtScores[inds]
                    dtm = np.concatenate([e["dtMatches"][:, 0:maxDet] for e in E], axis=1)[:, inds]
                    dtIg = np.concatenate([e["dtIgnore"][:, 0:maxDet] for e in E], axis=1)[:, inds]
                    gtIg = np.concatenate([e["gtIgnore"] for e in E])
                    npig = np.count_nonzero(gtIg == 0)
                    if npig == 0:
                        continue
                    tps = np.logical_and(dtm, np.logical_not(dtIg))
                    fps = np.logical_and(np.logical_not(dtm), np.logical_not(dtIg))
                    tp_sum = np.cumsum(tps, axis=1).astype(dtype=np.float64)
                    fp_sum = np.cumsum(fps, axis=1).astype(dtype=np.float64)
                    for t, (tp, fp) in enumerate(zip(tp_sum, fp_sum)):
                        nd = len(tp)
                        rc = tp / npig
                        pr = tp / (fp + tp + np.spacing(1))
                        q = np.zeros((R,))
                        ss = np.zeros((R,))
                        recall[t, k, a, m] = rc[-1] if nd else 0
                        pr = pr.tolist()
                        for i in range(nd - 1, 0, -1):
                            if pr[i] > pr[i - 1]:
                                pr[i - 1] = pr[i]
                        inds2 = np.searchsorted(rc, p.recThrs, side="left")
                        try:
                            for ri, pi in enumerate(inds2):
                                q[ri] = pr[pi]
                                ss[ri] = dtScoresSorted[pi]
                        except IndexError:
                            pass
                        precision[t, :, k, a, m] = np.array(q)
                        scores[t, :, k, a, m] = np.array(ss)
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
