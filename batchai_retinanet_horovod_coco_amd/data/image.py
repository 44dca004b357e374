"""Image I/O and preprocessing (keras-retinanet ``utils.image`` behaviour).

Reached from every generator the reference builds (``/root/reference/train.py:197-293``;
SURVEY §2.2 E-KR-image):

* ``read_image_bgr`` -- PIL decode -> RGB -> BGR uint8;
* ``preprocess_image`` -- caffe mode: float32, subtract BGR mean [103.939, 116.779, 123.68];
* ``compute_resize_scale`` / ``resize_image`` -- shortest side to ``min_side`` unless the longest
  side would exceed ``max_side``; bilinear resize (native C++ replacement for cv2.resize);
* ``TransformParameters`` / ``apply_transform`` -- affine warp about the given matrix (native C++
  replacement for cv2.warpAffine; fill modes constant / nearest / reflect / wrap).
"""
from __future__ import annotations

import numpy as np
from PIL import Image

from ..utils import cpu_native

CAFFE_MEAN_BGR = (103.939, 116.779, 123.68)


def read_image_bgr(path: str) -> np.ndarray:
    image = np.asarray(Image.open(path).convert("RGB"))
    return image[:, :, ::-1].copy()


def read_image_size(path: str):
    with Image.open(path) as im:
        w, h = im.size
    return h, w


def preprocess_image(x: np.ndarray, mode: str = "caffe") -> np.ndarray:
    x = x.astype(np.float32)
    if mode == "tf":
        x /= 127.5
        x -= 1.0
    elif mode == "caffe":
        x[..., 0] -= CAFFE_MEAN_BGR[0]
        x[..., 1] -= CAFFE_MEAN_BGR[1]
        x[..., 2] -= CAFFE_MEAN_BGR[2]
    return x


def compute_resize_scale(image_shape, min_side: int = 800, max_side: int = 1333) -> float:
    rows, cols = image_shape[0], image_shape[1]
    smallest = min(rows, cols)
    scale = min_side / smallest
    largest = max(rows, cols)
    if largest * scale > max_side:
        scale = max_side / largest
    return scale


def resize_image(img: np.ndarray, min_side: int = 800, max_side: int = 1333):
    scale = compute_resize_scale(img.shape, min_side=min_side, max_side=max_side)
    oh = int(round(img.shape[0] * scale))
    ow = int(round(img.shape[1] * scale))
    return cpu_native.resize_bilinear(img, oh, ow), scale


class TransformParameters:
    """How an affine transform is applied to an image (defaults match keras-retinanet)."""

    def __init__(self, fill_mode: str = "nearest", interpolation: str = "linear", cval: float = 0,
                 data_format=None, relative_translation: bool = True):
        if fill_mode not in cpu_native.BORDER:
            raise ValueError("invalid fill_mode {}".format(fill_mode))
        if interpolation not in cpu_native.INTERP:
            raise ValueError("invalid interpolation {}".format(interpolation))
        self.fill_mode = fill_mode
        self.cval = cval
        self.interpolation = interpolation
        self.relative_translation = relative_translation
        self.data_format = data_format


def apply_transform(matrix: np.ndarray, image: np.ndarray, params: TransformParameters) -> np.ndarray:
    """Warp ``image`` (H, W, C float) by the 3x3 ``matrix`` (source -> destination)."""
    return cpu_native.warp_affine(image, matrix, (image.shape[0], image.shape[1]), params.interpolation,
                                  params.fill_mode, params.cval)
