"""Generator protocol (keras-retinanet ``preprocessing.generator.Generator`` behaviour).

Every dataset generator the reference builds (``/root/reference/train.py:197-293``; SURVEY
§2.8.9) derives from :class:`Generator`:

* groups images by aspect ratio (``group_method='ratio'``) into ``batch_size`` groups (wrapping
  around to fill the last group), shuffles the groups at the start of each pass (thread-locked);
* per group: load images + annotations, drop invalid boxes (with a warning), caffe-preprocess,
  random affine transform (image warp + box AABB), resize (min/max side), scale boxes;
* ``compute_inputs`` zero-pads to the batch's max shape, top-left aligned -- rounded up to a multiple of
  ``pad_multiple`` when set (``--pad-multiple``): real COCO batches then fall into a few shape classes
  instead of one H x W per batch, and the extra anchors lie outside every image's region, so they are
  ignored exactly like the batch-max padding's (``tests/test_pad_classes.py``).

Output differs from the Keras generator in one deliberate way: instead of dense anchor targets
(65 MB/image of one-hot labels) ``next()`` returns the padded boxes, and the trainer computes the
targets on the GPU.  ``compute_targets()`` still produces the reference-format dense targets via
the numpy oracle (``compute_anchor_targets`` is overridable as in the reference,
``train.py:430-432``).
"""
from __future__ import annotations

import random
import threading
import warnings
from typing import Dict, List, Optional

import numpy as np
import torch

from ..ops.anchors import anchor_targets_bbox, guess_shapes
from .image import TransformParameters, apply_transform, preprocess_image, resize_image
from .transform import adjust_transform_for_image, transform_aabb


def pad_shape(shape, multiple: int):
    """``shape`` (H, W, ...) with H and W rounded up to ``multiple`` (0 / 1: unchanged)."""
    if not multiple or multiple <= 1:
        return tuple(shape)
    m = int(multiple)
    return (-(-int(shape[0]) // m) * m, -(-int(shape[1]) // m) * m) + tuple(shape[2:])


class Generator:
    def __init__(self, transform_generator=None, batch_size: int = 1, group_method: str = "ratio",
                 shuffle_groups: bool = True, image_min_side: int = 800, image_max_side: int = 1333,
                 transform_parameters: Optional[TransformParameters] = None,
                 compute_anchor_targets=anchor_targets_bbox, compute_shapes=guess_shapes,
                 preprocess_image=preprocess_image, seed: Optional[int] = None, shard: Optional[tuple] = None,
                 pad_multiple: int = 0):
        self.transform_generator = transform_generator
        self.batch_size = int(batch_size)
        self.group_method = group_method
        self.shuffle_groups = shuffle_groups
        self.image_min_side = image_min_side
        self.image_max_side = image_max_side
        self.transform_parameters = transform_parameters or TransformParameters()
        self.compute_anchor_targets = compute_anchor_targets
        self.compute_shapes = compute_shapes
        self.preprocess_image = preprocess_image
        self.rng = random.Random(seed)
        self.shard = shard            # (rank, world) -> rank-strided groups (--shard-data)
        self.pad_multiple = int(pad_multiple or 0)
        self.group_index = 0
        self.lock = threading.Lock()
        self._transform_lock = threading.Lock()
        self.device_preprocessor = None
        self.group_images()

    # ------------------------------------------------------------------ pickling (process loader workers)
    def __getstate__(self):
        """What a loader worker process needs: the dataset index and the box / resize settings.  Locks,
        the transform generator (drawn in the parent, in order) and the device preprocessor stay behind."""
        st = dict(self.__dict__)
        for k in ("lock", "_transform_lock", "transform_generator", "device_preprocessor"):
            st[k] = None
        return st

    def __setstate__(self, st):
        self.__dict__.update(st)
        self.lock = threading.Lock()
        self._transform_lock = threading.Lock()

    def enable_device_preprocess(self, device, mode: str = "caffe", dtype=torch.float32):
        """Normalise / warp / resize / pad on ``device`` (HIP kernels) instead of the host.

        Only the stock ``preprocess_image`` is mirrored on the device; a custom one keeps the
        host path.
        """
        from .device_preprocess import DevicePreprocessor
        if self.preprocess_image is not preprocess_image:
            return False
        self.device_preprocessor = DevicePreprocessor(device, self.image_min_side, self.image_max_side, mode, dtype,
                                                      pad_multiple=self.pad_multiple)
        return True

    # ------------------------------------------------------------------ abstract
    def size(self) -> int:
        raise NotImplementedError("size method not implemented")

    def num_classes(self) -> int:
        raise NotImplementedError("num_classes method not implemented")

    def has_label(self, label) -> bool:
        return label in self.labels

    def has_name(self, name) -> bool:
        return name in self.classes

    def name_to_label(self, name):
        raise NotImplementedError("name_to_label method not implemented")

    def label_to_name(self, label):
        raise NotImplementedError("label_to_name method not implemented")

    def image_aspect_ratio(self, image_index) -> float:
        raise NotImplementedError("image_aspect_ratio method not implemented")

    def load_image(self, image_index) -> np.ndarray:
        raise NotImplementedError("load_image method not implemented")

    def load_annotations(self, image_index) -> np.ndarray:
        raise NotImplementedError("load_annotations method not implemented")

    # ------------------------------------------------------------------ loading
    def load_annotations_group(self, group):
        return [np.asarray(self.load_annotations(i), dtype=np.float64).reshape(-1, 5) for i in group]

    def load_image_group(self, group):
        return [self.load_image(i) for i in group]

    def filter_annotations(self, image_group, annotations_group, group):
        for index, (image, annotations) in enumerate(zip(image_group, annotations_group)):
            invalid = np.where(
                (annotations[:, 2] <= annotations[:, 0]) |
                (annotations[:, 3] <= annotations[:, 1]) |
                (annotations[:, 0] < 0) |
                (annotations[:, 1] < 0) |
                (annotations[:, 2] > image.shape[1]) |
                (annotations[:, 3] > image.shape[0])
            )[0]
            if len(invalid):
                warnings.warn("Image with id {} (shape {}) contains the following invalid boxes: {}.".format(
                    group[index], image.shape, annotations[invalid, :].tolist()))
                annotations_group[index] = np.delete(annotations, invalid, axis=0)
        return image_group, annotations_group

    # ------------------------------------------------------------------ preprocessing
    def random_transform_group_entry(self, image, annotations):
        if self.transform_generator is not None:
            with self._transform_lock:     # python generators are not re-entrant across workers
                raw = next(self.transform_generator)
            transform = adjust_transform_for_image(raw, image, self.transform_parameters.relative_translation)
            image = apply_transform(transform, image, self.transform_parameters)
            annotations = annotations.copy()
            for index in range(annotations.shape[0]):
                annotations[index, :4] = transform_aabb(transform, annotations[index, :4])
        return image, annotations

    def resize_image(self, image):
        return resize_image(image, min_side=self.image_min_side, max_side=self.image_max_side)

    def preprocess_group_entry(self, image, annotations):
        image = self.preprocess_image(image)
        image, annotations = self.random_transform_group_entry(image, annotations)
        image, image_scale = self.resize_image(image)
        annotations = annotations.copy()
        annotations[:, :4] *= image_scale
        return image, annotations

    def preprocess_group(self, image_group, annotations_group):
        for index in range(len(image_group)):
            image_group[index], annotations_group[index] = self.preprocess_group_entry(image_group[index],
                                                                                      annotations_group[index])
        return image_group, annotations_group

    # ------------------------------------------------------------------ grouping
    def group_images(self):
        order = list(range(self.size()))
        if self.group_method == "random":
            self.rng.shuffle(order)
        elif self.group_method == "ratio":
            order.sort(key=lambda x: self.image_aspect_ratio(x))
        if not order:
            self.groups = []
            return
        self.groups = [[order[x % len(order)] for x in range(i, i + self.batch_size)]
                       for i in range(0, len(order), self.batch_size)]
        if self.shard is not None:
            r, w = self.shard
            mine = self.groups[r::w]
            self.groups = mine if mine else self.groups[:1]

    # ------------------------------------------------------------------ batching
    def padded_shape(self, image_group):
        """(H, W, C) of the batch: the largest image's, H and W rounded up to ``pad_multiple``."""
        return pad_shape(tuple(max(image.shape[x] for image in image_group) for x in range(3)), self.pad_multiple)

    def compute_inputs(self, image_group):
        max_shape = self.padded_shape(image_group)
        image_batch = np.zeros((self.batch_size,) + max_shape, dtype=np.float32)
        for i, image in enumerate(image_group):
            image_batch[i, :image.shape[0], :image.shape[1], :image.shape[2]] = image
        return image_batch

    def compute_targets(self, image_group, annotations_group):
        """Reference-format dense targets: regression (B, A, 5), labels (B, A, C+1) (state last)."""
        max_shape = self.padded_shape(image_group)
        regs, labs = [], []
        for image, annotations in zip(image_group, annotations_group):
            labels, reg, state = self.compute_anchor_targets(max_shape, annotations, self.num_classes(),
                                                             mask_shape=image.shape)
            regs.append(np.concatenate([reg, state[:, None]], axis=1))
            labs.append(np.concatenate([labels, state[:, None]], axis=1))
        return [np.stack(regs).astype(np.float32), np.stack(labs).astype(np.float32)]

    def compute_batch(self, image_group, annotations_group) -> Dict[str, torch.Tensor]:
        images = self.compute_inputs(image_group)
        G = max(1, max(a.shape[0] for a in annotations_group))
        B = self.batch_size
        gt = np.full((B, G, 5), -1.0, dtype=np.float32)
        cnt = np.zeros((B,), dtype=np.int32)
        hw = np.zeros((B, 2), dtype=np.int32)
        for i, (img, ann) in enumerate(zip(image_group, annotations_group)):
            n = ann.shape[0]
            gt[i, :n] = ann
            cnt[i] = n
            hw[i] = img.shape[:2]
        for i in range(len(image_group), B):    # short final group: repeat-free padding image
            hw[i] = images.shape[1:3]
        return {"images": torch.from_numpy(images), "gt": torch.from_numpy(gt), "gt_count": torch.from_numpy(cnt),
                "image_hw": torch.from_numpy(hw)}

    def compute_input_output(self, group) -> Dict[str, torch.Tensor]:
        if self.device_preprocessor is not None:
            from .device_preprocess import compute_input_output_device
            return compute_input_output_device(self, group)
        image_group = self.load_image_group(group)
        annotations_group = self.load_annotations_group(group)
        image_group, annotations_group = self.filter_annotations(image_group, annotations_group, group)
        image_group, annotations_group = self.preprocess_group(image_group, annotations_group)
        return self.compute_batch(image_group, annotations_group)

    def __len__(self) -> int:
        return len(self.groups)

    def __iter__(self):
        return self

    def __next__(self) -> Dict[str, torch.Tensor]:
        return self.next()

    def next(self) -> Dict[str, torch.Tensor]:
        with self.lock:
            if self.group_index == 0 and self.shuffle_groups:
                self.rng.shuffle(self.groups)
            group = self.groups[self.group_index]
            self.group_index = (self.group_index + 1) % len(self.groups)
        return self.compute_input_output(group)

    def __getitem__(self, index: int) -> Dict[str, torch.Tensor]:
        return self.compute_input_output(self.groups[index])
