"""Random affine augmentation (keras-retinanet ``utils.transform`` behaviour).

The reference builds ``random_transform_generator(flip_x_chance=0.5)`` by default and the full
rotation/translation/shear/scale/flip version with ``--random-transform``
(``/root/reference/train.py:179-193``).  Matrices are 3x3 homogeneous, composed as
rotation . translation . shear . scaling . flip and re-centred on the image centre.
"""
from __future__ import annotations

import numpy as np

DEFAULT_PRNG = np.random


def colvec(*args):
    return np.array([args]).T


def transform_aabb(transform: np.ndarray, aabb) -> list:
    """Axis-aligned bounding box of the transformed corners of ``aabb`` = [x1, y1, x2, y2]."""
    x1, y1, x2, y2 = aabb
    points = transform.dot([[x1, x2, x1, x2], [y1, y2, y2, y1], [1, 1, 1, 1]])
    mn = points.min(axis=1)
    mx = points.max(axis=1)
    return [mn[0], mn[1], mx[0], mx[1]]


def _random_vector(mn, mx, prng=DEFAULT_PRNG):
    mn = np.array(mn)
    mx = np.array(mx)
    assert mn.shape == mx.shape
    assert len(mn.shape) == 1
    return prng.uniform(mn, mx)


def rotation(angle: float) -> np.ndarray:
    return np.array([[np.cos(angle), -np.sin(angle), 0], [np.sin(angle), np.cos(angle), 0], [0, 0, 1]])


def random_rotation(min, max, prng=DEFAULT_PRNG):  # noqa: A002
    return rotation(prng.uniform(min, max))


def translation(translation) -> np.ndarray:
    return np.array([[1, 0, translation[0]], [0, 1, translation[1]], [0, 0, 1]])


def random_translation(min, max, prng=DEFAULT_PRNG):  # noqa: A002
    return translation(_random_vector(min, max, prng))


def shear(angle: float) -> np.ndarray:
    return np.array([[1, -np.sin(angle), 0], [0, np.cos(angle), 0], [0, 0, 1]])


def random_shear(min, max, prng=DEFAULT_PRNG):  # noqa: A002
    return shear(prng.uniform(min, max))


def scaling(factor) -> np.ndarray:
    return np.array([[factor[0], 0, 0], [0, factor[1], 0], [0, 0, 1]])


def random_scaling(min, max, prng=DEFAULT_PRNG):  # noqa: A002
    return scaling(_random_vector(min, max, prng))


def random_flip(flip_x_chance, flip_y_chance, prng=DEFAULT_PRNG):
    flip_x = prng.uniform(0, 1) < flip_x_chance
    flip_y = prng.uniform(0, 1) < flip_y_chance
    return scaling((1 - 2 * flip_x, 1 - 2 * flip_y))


def change_transform_origin(transform, center):
    center = np.array(center)
    return np.linalg.multi_dot([translation(center), transform, translation(-center)])


def random_transform(min_rotation=0, max_rotation=0, min_translation=(0, 0), max_translation=(0, 0), min_shear=0,
                     max_shear=0, min_scaling=(1, 1), max_scaling=(1, 1), flip_x_chance=0, flip_y_chance=0,
                     prng=DEFAULT_PRNG):
    return np.linalg.multi_dot([
        random_rotation(min_rotation, max_rotation, prng),
        random_translation(min_translation, max_translation, prng),
        random_shear(min_shear, max_shear, prng),
        random_scaling(min_scaling, max_scaling, prng),
        random_flip(flip_x_chance, flip_y_chance, prng),
    ])


def random_transform_generator(prng=None, **kwargs):
    """Infinite generator of random 3x3 transforms."""
    if prng is None:
        prng = np.random.RandomState()
    while True:
        yield random_transform(prng=prng, **kwargs)


def adjust_transform_for_image(transform, image, relative_translation):
    """Scale relative translation by the image size and move the origin to the image centre."""
    height, width = image.shape[0], image.shape[1]
    result = np.array(transform, dtype=np.float64)
    if relative_translation:
        result[0:2, 2] *= [width, height]
    return change_transform_origin(result, (0.5 * width, 0.5 * height))
