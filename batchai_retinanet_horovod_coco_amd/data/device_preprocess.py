"""Device-side batch assembly for real data (HIP normalise + affine warp + bilinear resize + pad).

The reference does all of this on the CPU per image (keras-retinanet ``preprocess_group_entry``:
caffe preprocess -> ``apply_transform`` (cv2.warpAffine) -> ``resize_image`` (cv2.resize) ->
``compute_inputs`` zero padding; SURVEY §2.6 K22, reached from ``/root/reference/train.py:179-193``)
and ships 12.8 MB of float32 per 800x1333 image host->device.  Here the host only decodes the
JPEG and draws the random transform; the uint8 image (4x smaller) goes to the GPU and
``csrc/kernels/image.hip`` does the rest directly into the padded NHWC batch.  Box arithmetic
(transform_aabb, scale) stays on the host, exactly as in the CPU path, so annotations are
bit-identical between the two paths.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..utils import cpu_native
from .image import CAFFE_MEAN_BGR, compute_resize_scale


def normalization(mode: str = "caffe"):
    """(scale, mean) such that ``x*scale - mean`` == ``preprocess_image(x, mode)``."""
    if mode == "caffe":
        return 1.0, CAFFE_MEAN_BGR
    if mode == "tf":
        return 1.0 / 127.5, (1.0, 1.0, 1.0)
    return 1.0, (0.0, 0.0, 0.0)


class DevicePreprocessor:
    """Builds the zero-padded (B, Hmax, Wmax, 3) batch on ``device`` from uint8 BGR images."""

    def __init__(self, device: torch.device, min_side: int = 800, max_side: int = 1333, mode: str = "caffe",
                 dtype: torch.dtype = torch.float32, pad_multiple: int = 0):
        self.device = torch.device(device)
        self.pad_multiple = int(pad_multiple or 0)
        self.min_side, self.max_side = min_side, max_side
        self.scale, self.mean = normalization(mode)
        self.dtype = dtype

    def output_size(self, hw: Sequence[int]):
        s = compute_resize_scale(hw, min_side=self.min_side, max_side=self.max_side)
        return (int(round(hw[0] * s)), int(round(hw[1] * s))), s

    def __call__(self, images: List[np.ndarray], matrices: List[Optional[np.ndarray]], batch_size: int,
                 params=None) -> torch.Tensor:
        from ..ops import native
        sizes = [self.output_size(im.shape[:2])[0] for im in images]
        from .generator import pad_shape
        Hm, Wm = pad_shape((max(s[0] for s in sizes), max(s[1] for s in sizes)), self.pad_multiple)
        batch = torch.zeros((batch_size, Hm, Wm, 3), dtype=self.dtype, device=self.device)
        interp = cpu_native.INTERP[params.interpolation] if params is not None else 1
        border = cpu_native.BORDER[params.fill_mode] if params is not None else 1
        cval = float(params.cval) if params is not None else 0.0
        for i, (im, M, (oh, ow)) in enumerate(zip(images, matrices, sizes)):
            host = torch.from_numpy(np.ascontiguousarray(im, dtype=np.uint8))
            if self.device.type == "cuda":
                host = host.pin_memory()
            src = host.to(self.device, non_blocking=True)
            f = native.image_warp_normalize(src, M, None, interp, border, cval, self.scale, self.mean)
            native.image_resize_into(f, batch, i, (oh, ow))
        return batch


def compute_input_output_device(gen, group) -> Dict[str, torch.Tensor]:
    """``Generator.compute_input_output`` with the image work on the device (see module doc)."""
    from .transform import adjust_transform_for_image, transform_aabb
    image_group = gen.load_image_group(group)
    annotations_group = gen.load_annotations_group(group)
    image_group, annotations_group = gen.filter_annotations(image_group, annotations_group, group)
    pre: DevicePreprocessor = gen.device_preprocessor
    matrices, sized_shapes = [], []
    for i, (image, ann) in enumerate(zip(image_group, annotations_group)):
        M = None
        ann = ann.copy()
        if gen.transform_generator is not None:
            with gen._transform_lock:
                raw = next(gen.transform_generator)
            M = adjust_transform_for_image(raw, image, gen.transform_parameters.relative_translation)
            for j in range(ann.shape[0]):
                ann[j, :4] = transform_aabb(M, ann[j, :4])
        (oh, ow), s = pre.output_size(image.shape[:2])
        ann[:, :4] *= s
        annotations_group[i] = ann
        matrices.append(M)
        sized_shapes.append((oh, ow))
    images = pre(image_group, matrices, gen.batch_size, gen.transform_parameters)
    B = gen.batch_size
    G = max(1, max(a.shape[0] for a in annotations_group))
    gt = np.full((B, G, 5), -1.0, dtype=np.float32)
    cnt = np.zeros((B,), dtype=np.int32)
    hw = np.zeros((B, 2), dtype=np.int32)
    for i, ann in enumerate(annotations_group):
        gt[i, :ann.shape[0]] = ann
        cnt[i] = ann.shape[0]
        hw[i] = sized_shapes[i]
    for i in range(len(image_group), B):
        hw[i] = images.shape[1:3]
    return {"images": images, "gt": torch.from_numpy(gt), "gt_count": torch.from_numpy(cnt),
            "image_hw": torch.from_numpy(hw)}
