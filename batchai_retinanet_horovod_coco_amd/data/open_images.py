"""Open Images generator (keras-retinanet ``OpenImagesGenerator`` behaviour).

Reference: ``OpenImagesGenerator(args.main_dir, subset='train' | 'validation', version,
labels_filter, annotation_cache_dir, fixed_labels, ...)`` (``/root/reference/train.py:252-276``).

Layout (v4): ``<main_dir>/2018_04/class-descriptions-boxable.csv``,
``<main_dir>/2018_04/<subset>/<subset>-annotations-bbox.csv``, images at
``<main_dir>/images/<subset>/<ImageID>.jpg``; challenge2018 uses
``challenge-2018-class-descriptions-500.csv``; v3 uses ``2017_11`` with ``classes-bbox-trainable.txt``.
Boxes are stored normalised; they are scaled by the image size (read once from the image header
and cached in ``<annotation_cache_dir>/<subset>.json``).  ``labels_filter`` keeps only the listed
class descriptions (re-indexed; in the given order when ``fixed_labels``).
"""
from __future__ import annotations

import csv
import json
import os
import warnings

import numpy as np

from .generator import Generator
from .image import read_image_bgr, read_image_size

_META = {"v4": "2018_04", "challenge2018": "challenge2018", "v3": "2017_11"}


def get_labels(metadata_dir: str, version: str = "v4"):
    id_to_labels, cls_index = {}, {}
    if version in ("v4", "challenge2018"):
        name = "class-descriptions-boxable.csv" if version == "v4" else "challenge-2018-class-descriptions-500.csv"
        with open(os.path.join(metadata_dir, name)) as f:
            i = 0
            for row in csv.reader(f):
                if not row:
                    continue
                label, description = row[0], row[1].replace('"', "").replace("'", "").replace("`", "")
                id_to_labels[i] = description
                cls_index[label] = i
                i += 1
    else:
        with open(os.path.join(metadata_dir, "classes-bbox-trainable.txt")) as f:
            trainable = [l.strip() for l in f if l.strip()]
        desc = {}
        with open(os.path.join(metadata_dir, "class-descriptions.csv")) as f:
            for row in csv.reader(f):
                if row:
                    desc[row[0]] = row[1]
        for i, label in enumerate(trainable):
            id_to_labels[i] = desc.get(label, label)
            cls_index[label] = i
    return id_to_labels, cls_index


def generate_images_annotations_json(main_dir, metadata_dir, subset, cls_index, version="v4"):
    if version == "challenge2018":
        ann_file = os.path.join(metadata_dir, subset, "challenge-2018-{}-annotations-bbox.csv".format(subset))
    else:
        ann_file = os.path.join(metadata_dir, subset, "{}-annotations-bbox.csv".format(subset))
    if not os.path.exists(ann_file):
        ann_file = os.path.join(metadata_dir, "{}-annotations-bbox.csv".format(subset))
    images = {}
    sizes = {}
    with open(ann_file) as f:
        reader = csv.DictReader(f)
        for row in reader:
            image_id = row["ImageID"]
            label = row["LabelName"]
            if label not in cls_index:
                continue
            x1, x2 = float(row["XMin"]), float(row["XMax"])
            y1, y2 = float(row["YMin"]), float(row["YMax"])
            if x2 <= x1 or y2 <= y1:
                warnings.warn("image {} has a degenerate box ({}, {}, {}, {})".format(image_id, x1, y1, x2, y2))
                continue
            if image_id not in images:
                p = os.path.join(main_dir, "images", subset, image_id + ".jpg")
                if image_id not in sizes:
                    try:
                        sizes[image_id] = read_image_size(p)
                    except OSError:
                        warnings.warn("image {} not found, skipping".format(p))
                        sizes[image_id] = None
                if sizes[image_id] is None:
                    continue
                h, w = sizes[image_id]
                images[image_id] = {"w": w, "h": h, "boxes": []}
            images[image_id]["boxes"].append({"cls_id": cls_index[label], "x1": x1, "x2": x2, "y1": y1, "y2": y2})
    return images


class OpenImagesGenerator(Generator):
    def __init__(self, main_dir: str, subset: str, version: str = "v4", labels_filter=None,
                 annotation_cache_dir: str = ".", fixed_labels: bool = False, **kwargs):
        metadata_dir = os.path.join(main_dir, _META.get(version, version))
        self.base_dir = main_dir
        self.image_dir = os.path.join(main_dir, "images", subset)
        self.id_to_labels, cls_index = get_labels(metadata_dir, version)
        cache = os.path.join(annotation_cache_dir, "{}.json".format(subset))
        if os.path.exists(cache):
            with open(cache) as f:
                self.annotations = json.load(f)
        else:
            self.annotations = generate_images_annotations_json(main_dir, metadata_dir, subset, cls_index, version)
            os.makedirs(annotation_cache_dir or ".", exist_ok=True)
            with open(cache, "w") as f:
                json.dump(self.annotations, f)
        if labels_filter is not None:
            self.id_to_labels, self.annotations = self._filter(labels_filter, fixed_labels)
        self.id_to_image_id = {i: k for i, k in enumerate(sorted(self.annotations))}
        self.labels = self.id_to_labels
        self.classes = {v: k for k, v in self.id_to_labels.items()}
        super().__init__(**kwargs)

    def _filter(self, labels_filter, fixed_labels):
        if fixed_labels:
            wanted = list(labels_filter)
        else:
            wanted = [d for _, d in sorted(self.id_to_labels.items()) if d in set(labels_filter)]
        old_by_desc = {d: i for i, d in self.id_to_labels.items()}
        remap = {old_by_desc[d]: new for new, d in enumerate(wanted) if d in old_by_desc}
        id_to_labels = {new: d for new, d in enumerate(wanted)}
        filtered = {}
        for image_id, ann in self.annotations.items():
            boxes = [dict(b, cls_id=remap[b["cls_id"]]) for b in ann["boxes"] if b["cls_id"] in remap]
            if boxes:
                filtered[image_id] = {"w": ann["w"], "h": ann["h"], "boxes": boxes}
        return id_to_labels, filtered

    def size(self):
        return len(self.annotations)

    def num_classes(self):
        return len(self.id_to_labels)

    def has_label(self, label):
        return label in self.id_to_labels

    def name_to_label(self, name):
        return self.classes[name]

    def label_to_name(self, label):
        return self.id_to_labels[label]

    def image_aspect_ratio(self, image_index):
        ann = self.annotations[self.id_to_image_id[image_index]]
        return float(ann["w"]) / float(ann["h"])

    def image_path(self, image_index):
        return os.path.join(self.image_dir, self.id_to_image_id[image_index] + ".jpg")

    def load_image(self, image_index):
        return read_image_bgr(self.image_path(image_index))

    def load_annotations(self, image_index):
        ann = self.annotations[self.id_to_image_id[image_index]]
        boxes = ann["boxes"]
        h, w = ann["h"], ann["w"]
        out = np.zeros((len(boxes), 5))
        for idx, b in enumerate(boxes):
            out[idx] = [b["x1"] * w, b["y1"] * h, b["x2"] * w, b["y2"] * h, b["cls_id"]]
        return out
