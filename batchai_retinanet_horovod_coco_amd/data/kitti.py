"""KITTI generator (keras-retinanet ``KittiGenerator`` behaviour).

Reference: ``KittiGenerator(args.kitti_path, subset='train' | 'val', ...)``
(``/root/reference/train.py:277-293``).  Layout: ``<base>/<subset>/labels/*.txt`` and
``<base>/<subset>/images/*.png``; label lines are
``type truncated occluded alpha left top right bottom h w l x y z rotation_y``.
"""
from __future__ import annotations

import csv
import os

import numpy as np
from PIL import Image

from .generator import Generator
from .image import read_image_bgr

kitti_classes = {
    "Car": 0, "Van": 1, "Truck": 2, "Pedestrian": 3, "Person_sitting": 4, "Cyclist": 5, "Tram": 6, "Misc": 7,
    "DontCare": 7,
}


class KittiGenerator(Generator):
    def __init__(self, base_dir: str, subset: str = "train", **kwargs):
        self.base_dir = base_dir
        label_dir = os.path.join(base_dir, subset, "labels")
        image_dir = os.path.join(base_dir, subset, "images")
        self.id_to_labels = {}
        for label, id_ in kitti_classes.items():
            self.id_to_labels.setdefault(id_, label)
        self.classes = kitti_classes
        self.labels = self.id_to_labels
        self.image_data = {}
        self.images = []
        for i, fn in enumerate(sorted(os.listdir(label_dir))):
            path = os.path.join(label_dir, fn)
            self.images.append(os.path.join(image_dir, fn.replace(".txt", ".png")))
            boxes = []
            with open(path, "r") as f:
                reader = csv.reader(f, delimiter=" ")
                for row in reader:
                    if not row:
                        continue
                    obj_type = row[0]
                    if obj_type not in kitti_classes:
                        raise ValueError("unknown KITTI class '{}' in {}".format(obj_type, path))
                    x1, y1, x2, y2 = (float(v) for v in row[4:8])
                    boxes.append({"cls_id": kitti_classes[obj_type], "x1": x1, "y1": y1, "x2": x2, "y2": y2})
            self.image_data[i] = boxes
        super().__init__(**kwargs)

    def size(self):
        return len(self.images)

    def num_classes(self):
        return max(kitti_classes.values()) + 1

    def name_to_label(self, name):
        return kitti_classes[name]

    def label_to_name(self, label):
        return self.id_to_labels[label]

    def image_aspect_ratio(self, image_index):
        with Image.open(self.images[image_index]) as image:
            return float(image.width) / float(image.height)

    def load_image(self, image_index):
        return read_image_bgr(self.images[image_index])

    def load_annotations(self, image_index):
        annots = self.image_data[image_index]
        boxes = np.zeros((len(annots), 5))
        for idx, a in enumerate(annots):
            boxes[idx] = [a["x1"], a["y1"], a["x2"], a["y2"], a["cls_id"]]
        return boxes
