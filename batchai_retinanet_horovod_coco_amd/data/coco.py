"""COCO detection generator (keras-retinanet ``CocoGenerator`` behaviour; pycocotools not needed).

Reference: ``CocoGenerator(args.coco_path, 'train2017' | 'val2017', ...)``
(``/root/reference/train.py:197-214``).  Layout: ``<data_dir>/annotations/instances_<set>.json``
and ``<data_dir>/images/<set>/<file_name>``.  Category ids map to contiguous labels in sorted-id
order (0..79 for COCO); boxes are xywh -> x1y1x2y2; crowd boxes and boxes with w or h < 1 are
skipped.  :class:`CocoIndex` is a minimal json index (the subset of ``pycocotools.coco.COCO``
the generator and the evaluator use).
"""
from __future__ import annotations

import json
import os
from collections import defaultdict
from typing import Dict, List

import numpy as np

from .generator import Generator
from .image import read_image_bgr


class CocoIndex:
    """Minimal COCO annotation index: imgs, anns, cats, imgToAnns."""

    def __init__(self, annotation_file: str = None, dataset: dict = None):
        if dataset is None:
            with open(annotation_file) as f:
                dataset = json.load(f)
        self.dataset = dataset
        self.imgs: Dict[int, dict] = {img["id"]: img for img in dataset.get("images", [])}
        self.anns: Dict[int, dict] = {}
        self.cats: Dict[int, dict] = {c["id"]: c for c in dataset.get("categories", [])}
        self.imgToAnns: Dict[int, List[dict]] = defaultdict(list)
        for a in dataset.get("annotations", []):
            self.anns[a["id"]] = a
            self.imgToAnns[a["image_id"]].append(a)

    def getImgIds(self) -> List[int]:
        return list(self.imgs.keys())

    def getCatIds(self) -> List[int]:
        return list(self.cats.keys())

    def loadCats(self, ids) -> List[dict]:
        return [self.cats[i] for i in ids]

    def loadImgs(self, ids) -> List[dict]:
        return [self.imgs[i] for i in (ids if isinstance(ids, (list, tuple)) else [ids])]

    def getAnnIds(self, imgIds=None, catIds=None, iscrowd=None) -> List[int]:
        ids = imgIds if isinstance(imgIds, (list, tuple)) else ([imgIds] if imgIds is not None else None)
        anns = [a for i in ids for a in self.imgToAnns.get(i, [])] if ids is not None else list(self.anns.values())
        if catIds:
            anns = [a for a in anns if a["category_id"] in set(catIds)]
        if iscrowd is not None:
            anns = [a for a in anns if bool(a.get("iscrowd", 0)) == bool(iscrowd)]
        return [a["id"] for a in anns]

    def loadAnns(self, ids) -> List[dict]:
        return [self.anns[i] for i in ids]


class CocoGenerator(Generator):
    def __init__(self, data_dir: str, set_name: str, **kwargs):
        self.data_dir = data_dir
        self.set_name = set_name
        self.coco = CocoIndex(os.path.join(data_dir, "annotations", "instances_" + set_name + ".json"))
        self.image_ids = self.coco.getImgIds()
        self.load_classes()
        super().__init__(**kwargs)

    def load_classes(self):
        categories = self.coco.loadCats(self.coco.getCatIds())
        categories.sort(key=lambda x: x["id"])
        self.classes, self.coco_labels, self.coco_labels_inverse = {}, {}, {}
        for c in categories:
            self.coco_labels[len(self.classes)] = c["id"]
            self.coco_labels_inverse[c["id"]] = len(self.classes)
            self.classes[c["name"]] = len(self.classes)
        self.labels = {v: k for k, v in self.classes.items()}

    def size(self) -> int:
        return len(self.image_ids)

    def num_classes(self) -> int:
        return len(self.classes)

    def name_to_label(self, name):
        return self.classes[name]

    def label_to_name(self, label):
        return self.labels[label]

    def coco_label_to_label(self, coco_label):
        return self.coco_labels_inverse[coco_label]

    def coco_label_to_name(self, coco_label):
        return self.label_to_name(self.coco_label_to_label(coco_label))

    def label_to_coco_label(self, label):
        return self.coco_labels[label]

    def image_aspect_ratio(self, image_index) -> float:
        image = self.coco.loadImgs(self.image_ids[image_index])[0]
        return float(image["width"]) / float(image["height"])

    def image_path(self, image_index) -> str:
        info = self.coco.loadImgs(self.image_ids[image_index])[0]
        return os.path.join(self.data_dir, "images", self.set_name, info["file_name"])

    def load_image(self, image_index):
        return read_image_bgr(self.image_path(image_index))

    def load_annotations(self, image_index):
        ids = self.coco.getAnnIds(imgIds=self.image_ids[image_index], iscrowd=False)
        annotations = np.zeros((0, 5))
        if len(ids) == 0:
            return annotations
        for a in self.coco.loadAnns(ids):
            if a["bbox"][2] < 1 or a["bbox"][3] < 1:
                continue
            box = np.zeros((1, 5))
            box[0, :4] = a["bbox"]
            box[0, 4] = self.coco_label_to_label(a["category_id"])
            annotations = np.append(annotations, box, axis=0)
        annotations[:, 2] = annotations[:, 0] + annotations[:, 2]
        annotations[:, 3] = annotations[:, 1] + annotations[:, 3]
        return annotations
