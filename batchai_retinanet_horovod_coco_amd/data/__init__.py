"""Data pipeline: Generator protocol, COCO / Pascal VOC / CSV / KITTI / Open Images generators,
synthetic COCO-shaped batches, image ops, random affine transforms, prefetching enqueuer."""
from .generator import Generator  # noqa: F401
from .image import (TransformParameters, apply_transform, preprocess_image, read_image_bgr,  # noqa: F401
                    resize_image, compute_resize_scale)
from .transform import random_transform_generator, transform_aabb  # noqa: F401


def CocoGenerator(*args, **kwargs):
    from .coco import CocoGenerator as G
    return G(*args, **kwargs)


def PascalVocGenerator(*args, **kwargs):
    from .pascal_voc import PascalVocGenerator as G
    return G(*args, **kwargs)


def CSVGenerator(*args, **kwargs):
    from .csv_generator import CSVGenerator as G
    return G(*args, **kwargs)


def KittiGenerator(*args, **kwargs):
    from .kitti import KittiGenerator as G
    return G(*args, **kwargs)


def OpenImagesGenerator(*args, **kwargs):
    from .open_images import OpenImagesGenerator as G
    return G(*args, **kwargs)
