"""CSV generator (keras-retinanet ``CSVGenerator`` behaviour).

Reference: ``CSVGenerator(args.annotations, args.classes, ...)`` with optional
``--val-annotations`` (``/root/reference/train.py:232-251``).

* classes file: ``class_name,id`` per line (ids must be unique);
* annotations file: ``path/to/image.jpg,x1,y1,x2,y2,class_name`` per box, or
  ``path/to/image.jpg,,,,,`` for an image without boxes; relative paths are resolved against
  the annotations file's directory (or ``base_dir``).  Malformed lines raise ``ValueError`` with
  the line number.
"""
from __future__ import annotations

import csv
import os
from collections import OrderedDict

import numpy as np
from PIL import Image

from .generator import Generator
from .image import read_image_bgr


def _parse(value, function, fmt):
    try:
        return function(value)
    except ValueError as e:
        raise ValueError(fmt.format(e)) from None


def _read_classes(csv_reader):
    result = OrderedDict()
    for line, row in enumerate(csv_reader):
        line += 1
        try:
            class_name, class_id = row
        except ValueError:
            raise ValueError("line {}: format should be 'class_name,class_id'".format(line)) from None
        class_id = _parse(class_id, int, "line {}: malformed class ID: {{}}".format(line))
        if class_name in result:
            raise ValueError("line {}: duplicate class name: '{}'".format(line, class_name))
        result[class_name] = class_id
    return result


def _read_annotations(csv_reader, classes):
    result = OrderedDict()
    for line, row in enumerate(csv_reader):
        line += 1
        try:
            img_file, x1, y1, x2, y2, class_name = row[:6]
        except ValueError:
            raise ValueError("line {}: format should be 'img_file,x1,y1,x2,y2,class_name' or 'img_file,,,,,'".format(
                line)) from None
        if img_file not in result:
            result[img_file] = []
        if (x1, y1, x2, y2, class_name) == ("", "", "", "", ""):
            continue
        x1 = _parse(x1, int, "line {}: malformed x1: {{}}".format(line))
        y1 = _parse(y1, int, "line {}: malformed y1: {{}}".format(line))
        x2 = _parse(x2, int, "line {}: malformed x2: {{}}".format(line))
        y2 = _parse(y2, int, "line {}: malformed y2: {{}}".format(line))
        if x2 <= x1:
            raise ValueError("line {}: x2 ({}) must be higher than x1 ({})".format(line, x2, x1))
        if y2 <= y1:
            raise ValueError("line {}: y2 ({}) must be higher than y1 ({})".format(line, y2, y1))
        if class_name not in classes:
            raise ValueError("line {}: unknown class name: '{}' (classes: {})".format(line, class_name, classes))
        result[img_file].append({"x1": x1, "x2": x2, "y1": y1, "y2": y2, "class": class_name})
    return result


def _open_for_csv(path):
    return open(path, "r", newline="")


class CSVGenerator(Generator):
    def __init__(self, csv_data_file: str, csv_class_file: str, base_dir: str = None, **kwargs):
        self.image_names = []
        self.image_data = {}
        self.base_dir = base_dir
        if self.base_dir is None:
            self.base_dir = os.path.dirname(csv_data_file)
        try:
            with _open_for_csv(csv_class_file) as file:
                self.classes = _read_classes(csv.reader(file, delimiter=","))
        except ValueError as e:
            raise ValueError("invalid CSV class file: {}: {}".format(csv_class_file, e)) from None
        self.labels = {v: k for k, v in self.classes.items()}
        try:
            with _open_for_csv(csv_data_file) as file:
                self.image_data = _read_annotations(csv.reader(file, delimiter=","), self.classes)
        except ValueError as e:
            raise ValueError("invalid CSV annotations file: {}: {}".format(csv_data_file, e)) from None
        self.image_names = list(self.image_data.keys())
        super().__init__(**kwargs)

    def size(self):
        return len(self.image_names)

    def num_classes(self):
        return max(self.classes.values()) + 1

    def name_to_label(self, name):
        return self.classes[name]

    def label_to_name(self, label):
        return self.labels[label]

    def image_path(self, image_index):
        return os.path.join(self.base_dir, self.image_names[image_index])

    def image_aspect_ratio(self, image_index):
        with Image.open(self.image_path(image_index)) as image:
            return float(image.width) / float(image.height)

    def load_image(self, image_index):
        return read_image_bgr(self.image_path(image_index))

    def load_annotations(self, image_index):
        path = self.image_names[image_index]
        annots = self.image_data[path]
        boxes = np.zeros((len(annots), 5))
        for idx, annot in enumerate(annots):
            boxes[idx, 0] = float(annot["x1"])
            boxes[idx, 1] = float(annot["y1"])
            boxes[idx, 2] = float(annot["x2"])
            boxes[idx, 3] = float(annot["y2"])
            boxes[idx, 4] = self.name_to_label(annot["class"])
        return boxes
