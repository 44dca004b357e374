"""Model registry: ``backbone(name)`` -> object with ``.retinanet()``, ``.download_imagenet()``,
``.validate()``; ``load_model(path, backbone_name)``.

Mirrors the ``models`` API the reference drives at ``/root/reference/train.py:390,406,413,91``
(keras-retinanet ``models.backbone`` / ``models.load_model``; SURVEY §2.2 E-KR-models).
"""
from __future__ import annotations

import os
from typing import Callable, Optional

from .layers import Conv2D, FrozenBatchNormalization  # noqa: F401
from .retinanet import RetinaNet, RetinaNetBBox, retinanet_bbox  # noqa: F401
from .resnet import ResNet  # noqa: F401

IMAGENET_CACHE_DIRS = ("~/.keras/models", "~/.cache/batchai_retinanet_horovod_coco_amd")


class Backbone:
    """Backbone descriptor (keras-retinanet ``Backbone`` protocol)."""

    allowed = ()

    def __init__(self, name: str):
        self.backbone = name
        self.validate()

    @property
    def custom_objects(self):
        # Keras needed these to deserialize the graph; our checkpoints rebuild the model from
        # the backbone name, so the mapping documents the layer types that exist.
        from ..ops import losses
        return {"UpsampleLike": "ops.conv.upsample_like", "PriorProbability": "models.layers.prior_probability_bias",
                "RegressBoxes": "ops.boxes.bbox_transform_inv", "FilterDetections": "ops.boxes.filter_detections",
                "Anchors": "ops.anchors.anchors_for_shape", "ClipBoxes": "ops.boxes.clip_boxes",
                "_smooth_l1": losses.smooth_l1_keras, "_focal": losses.focal_keras}

    def validate(self):
        if self.backbone not in self.allowed:
            raise ValueError("Backbone ('{}') not in allowed backbones ({}).".format(self.backbone, self.allowed))

    def retinanet(self, num_classes: int, modifier: Optional[Callable] = None, **kwargs) -> RetinaNet:
        raise NotImplementedError

    def imagenet_filename(self) -> str:
        raise NotImplementedError

    def download_imagenet(self) -> str:
        """Locate ImageNet weights offline (the reference downloads them, train.py:412-413)."""
        fname = self.imagenet_filename()
        for d in IMAGENET_CACHE_DIRS:
            p = os.path.join(os.path.expanduser(d), fname)
            if os.path.exists(p):
                return p
        raise FileNotFoundError(
            "ImageNet weights '{}' not found in {} and there is no network access; pass --weights <file> "
            "or --no-weights.".format(fname, ", ".join(IMAGENET_CACHE_DIRS)))


class ResNetBackbone(Backbone):
    allowed = ("resnet18", "resnet34", "resnet50", "resnet101", "resnet152")

    def retinanet(self, num_classes: int, modifier: Optional[Callable] = None, **kwargs) -> RetinaNet:
        model = RetinaNet(num_classes, backbone=self.backbone, **kwargs)
        if modifier is not None:
            model = modifier(model) or model
        return model

    def imagenet_filename(self) -> str:
        depth = int(self.backbone.replace("resnet", ""))
        return "ResNet-{}-model.keras.h5".format(depth)


def backbone(backbone_name: str) -> Backbone:
    """Registry lookup by substring, like keras-retinanet (``'resnet' in name``)."""
    if "resnet" in backbone_name:
        return ResNetBackbone(backbone_name)
    from . import extra_backbones
    return extra_backbones.lookup(backbone_name)


def freeze(model: RetinaNet) -> RetinaNet:
    """``utils.model.freeze``: make every backbone layer non-trainable."""
    model.freeze_backbone()
    return model


def load_model(filepath: str, backbone_name: str = "resnet50", **kwargs):
    """Rebuild a RetinaNet from a checkpoint written by :mod:`io.keras_h5` (or safetensors)."""
    from ..io import checkpoint
    return checkpoint.load_model(filepath, backbone_name=backbone_name, **kwargs)
