"""Pascal VOC generator (keras-retinanet ``PascalVocGenerator`` behaviour).

Reference: ``PascalVocGenerator(args.pascal_path, 'trainval' | 'test', ...)``
(``/root/reference/train.py:215-231``).  Layout: ``VOCdevkit/VOC20xx``-style directory with
``ImageSets/Main/<set>.txt``, ``Annotations/<name>.xml`` and ``JPEGImages/<name>.jpg``; 20 classes;
1-based pixel boxes are converted to 0-based.
"""
from __future__ import annotations

import os
import xml.etree.ElementTree as ET

import numpy as np
from PIL import Image

from .generator import Generator
from .image import read_image_bgr

voc_classes = {
    "aeroplane": 0, "bicycle": 1, "bird": 2, "boat": 3, "bottle": 4, "bus": 5, "car": 6, "cat": 7, "chair": 8,
    "cow": 9, "diningtable": 10, "dog": 11, "horse": 12, "motorbike": 13, "person": 14, "pottedplant": 15,
    "sheep": 16, "sofa": 17, "train": 18, "tvmonitor": 19,
}


def _findNode(parent, name, debug_name=None, parse=None):
    if debug_name is None:
        debug_name = name
    result = parent.find(name)
    if result is None:
        raise ValueError("missing element '{}'".format(debug_name))
    if parse is not None:
        try:
            return parse(result.text)
        except ValueError as e:
            raise ValueError("illegal value for '{}': {}".format(debug_name, e)) from None
    return result


class PascalVocGenerator(Generator):
    def __init__(self, data_dir: str, set_name: str, classes=voc_classes, image_extension: str = ".jpg",
                 skip_truncated: bool = False, skip_difficult: bool = False, **kwargs):
        self.data_dir = data_dir
        self.set_name = set_name
        self.classes = classes
        with open(os.path.join(data_dir, "ImageSets", "Main", set_name + ".txt")) as f:
            self.image_names = [line.strip().split(None, 1)[0] for line in f if line.strip()]
        self.image_extension = image_extension
        self.skip_truncated = skip_truncated
        self.skip_difficult = skip_difficult
        self.labels = {v: k for k, v in self.classes.items()}
        super().__init__(**kwargs)

    def size(self):
        return len(self.image_names)

    def num_classes(self):
        return len(self.classes)

    def name_to_label(self, name):
        return self.classes[name]

    def label_to_name(self, label):
        return self.labels[label]

    def image_path(self, image_index):
        return os.path.join(self.data_dir, "JPEGImages", self.image_names[image_index] + self.image_extension)

    def image_aspect_ratio(self, image_index):
        with Image.open(self.image_path(image_index)) as image:
            return float(image.width) / float(image.height)

    def load_image(self, image_index):
        return read_image_bgr(self.image_path(image_index))

    def __parse_annotation(self, element):
        truncated = _findNode(element, "truncated", parse=int) if element.find("truncated") is not None else 0
        difficult = _findNode(element, "difficult", parse=int) if element.find("difficult") is not None else 0
        class_name = _findNode(element, "name").text
        if class_name not in self.classes:
            raise ValueError("class name '{}' not found in classes: {}".format(class_name, list(self.classes.keys())))
        box = np.zeros((1, 5))
        box[0, 4] = self.name_to_label(class_name)
        bndbox = _findNode(element, "bndbox")
        box[0, 0] = _findNode(bndbox, "xmin", "bndbox.xmin", parse=float) - 1
        box[0, 1] = _findNode(bndbox, "ymin", "bndbox.ymin", parse=float) - 1
        box[0, 2] = _findNode(bndbox, "xmax", "bndbox.xmax", parse=float) - 1
        box[0, 3] = _findNode(bndbox, "ymax", "bndbox.ymax", parse=float) - 1
        return truncated, difficult, box

    def __parse_annotations(self, xml_root):
        boxes = np.zeros((0, 5))
        for i, element in enumerate(xml_root.iter("object")):
            try:
                truncated, difficult, box = self.__parse_annotation(element)
            except ValueError as e:
                raise ValueError("could not parse object #{}: {}".format(i, e)) from None
            if truncated and self.skip_truncated:
                continue
            if difficult and self.skip_difficult:
                continue
            boxes = np.append(boxes, box, axis=0)
        return boxes

    def load_annotations(self, image_index):
        filename = self.image_names[image_index] + ".xml"
        try:
            tree = ET.parse(os.path.join(self.data_dir, "Annotations", filename))
            return self.__parse_annotations(tree.getroot())
        except ET.ParseError as e:
            raise ValueError("invalid annotations file: {}: {}".format(filename, e)) from None
        except ValueError as e:
            raise ValueError("invalid annotations file: {}: {}".format(filename, e)) from None
