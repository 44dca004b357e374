"""Operators: anchors/targets, box ops, losses, NHWC convolution front-end, HIP bindings."""
from . import anchors, boxes, conv, losses, native  # noqa: F401
