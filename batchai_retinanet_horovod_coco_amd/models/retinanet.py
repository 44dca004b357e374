"""RetinaNet = backbone -> FPN (P3..P7) -> shared classification / regression heads.

Spec: keras-retinanet ``models.retinanet.retinanet`` / ``__create_pyramid_features`` /
``default_classification_model`` / ``default_regression_model`` / ``retinanet_bbox``, built
by ``backbone.retinanet(num_classes, modifier)`` at ``/root/reference/train.py:91`` and
``retinanet_bbox(model=model)`` at ``train.py:95,408``.

Training outputs follow the Keras model's output names: ``regression`` (B, A, 4) and
``classification`` (B, A, C).  Unlike the Keras model the classification output is returned
as *logits*: the sigmoid is fused into the focal-loss kernel; :class:`RetinaNetBBox` applies
it for inference.  Anchor order is level (P3..P7) -> row -> column -> anchor (ratio-major),
and the head channel index is ``anchor * C + class`` -- identical to the reference.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import os

import torch
import torch.nn as nn

from ..ops import anchors as anchor_ops
from ..ops import boxes as box_ops
from ..ops import conv as conv_ops
from .layers import Conv2D, prior_probability_bias
from .resnet import ResNet


class FPN(nn.Module):
    """Feature pyramid (feature_size 256; glorot_uniform kernels, zero bias)."""

    def __init__(self, c3: int, c4: int, c5: int, feature_size: int = 256):
        super().__init__()
        f = feature_size
        self.C5_reduced = Conv2D("C5_reduced", c5, f, 1, 1, "same")
        self.P5 = Conv2D("P5", f, f, 3, 1, "same")
        self.C4_reduced = Conv2D("C4_reduced", c4, f, 1, 1, "same")
        self.P4 = Conv2D("P4", f, f, 3, 1, "same")
        self.C3_reduced = Conv2D("C3_reduced", c3, f, 1, 1, "same")
        self.P3 = Conv2D("P3", f, f, 3, 1, "same")
        self.P6 = Conv2D("P6", c5, f, 3, 2, "same")
        self.P7 = Conv2D("P7", f, f, 3, 2, "same")

    def forward(self, C3, C4, C5, joins=None) -> List[torch.Tensor]:
        """``joins``: {1: C3, 2: C4, 3: C5 GradJoin} shared with the backbone (RetinaNet.features)."""
        j = joins or {}
        P5r = self.C5_reduced(C5, join=j.get(3))
        P4m = conv_ops.upsample_add(P5r, self.C4_reduced(C4, join=j.get(2)))      # P5_upsampled + C4_reduced
        P3m = conv_ops.upsample_add(P4m, self.C3_reduced(C3, join=j.get(1)))      # P4_upsampled + C3_reduced
        P5 = self.P5(P5r)
        P4 = self.P4(P4m)
        P3 = self.P3(P3m)
        P6 = self.P6(C5, join=j.get(3))
        P7 = self.P7(torch.relu(P6))                               # C6_relu -> P7
        return [P3, P4, P5, P6, P7]

    def convs(self) -> List[Conv2D]:
        return [self.C5_reduced, self.P5, self.C4_reduced, self.P4, self.C3_reduced, self.P3, self.P6, self.P7]


class Submodel(nn.Module):
    """Shared head tower: 4 x (3x3 conv 256 + ReLU) + final 3x3 conv."""

    def __init__(self, name: str, prefix: str, cin: int, width: int, out_channels: int, final_bias: float):
        super().__init__()
        self.keras_name = name
        self.tower = nn.ModuleList(
            [Conv2D(f"{prefix}_{i}", cin if i == 0 else width, width, 3, 1, "same", True, True, "normal001")
             for i in range(4)])
        self.final = Conv2D(prefix, width, out_channels, 3, 1, "same", True, False, "normal001", bias_value=final_bias)
        if os.environ.get("MXR_HEAD_MAIN_WGRAD", "0") == "1":
            # the head weight gradients on the compute stream, serial with the data gradients (an A/B of the
            # side-stream overlap for the biggest weight gradients: profiles/r6_head_main_wgrad_ab.txt)
            for c in self.convs():
                c.weight.mxr_main_wgrad = True

    def forward(self, feats: List[torch.Tensor]) -> List[torch.Tensor]:
        x = feats
        for c in self.tower:
            w, b = c.effective(x[0].dtype)
            x = conv_ops.pyramid_conv(x, w, b, relu=True)
        w, b = self.final.effective(x[0].dtype)
        return conv_ops.pyramid_conv(x, w, b, relu=False)

    def forward_packed(self, x: torch.Tensor, shapes, pad_sink=None, join=None) -> torch.Tensor:
        """All 5 levels as ONE ragged GEMM per layer on packed [B, P, C] features.

        ``pad_sink``: dict through which the loss may hand the final layer its gradient already in
        zero-padded rows (see :attr:`RetinaNet.cls_pad_sink`)."""
        from ..ops import native_conv
        from ..ops import fp8
        # each tower output feeds only the next layer: its relu backward is fused into that layer's
        # data-gradient epilogue (mask_input_grad) and skipped in its own backward (grad_premasked); out_f8 when
        # that next layer runs fp8 (the regression final's 36 outputs do not)
        for i, c in enumerate(self.tower):
            nxt = self.tower[i + 1] if i + 1 < len(self.tower) else self.final
            x = native_conv.pyramid_conv_layer(x, shapes, c, True, mask_input_grad=i > 0, grad_premasked=True,
                                               join=join if i == 0 else None,
                                               out_f8=fp8.eligible(nxt.cin, nxt.cout))
        return native_conv.pyramid_conv_layer(x, shapes, self.final, False, mask_input_grad=True,
                                              pad_sink=pad_sink)

    def convs(self) -> List[Conv2D]:
        return list(self.tower) + [self.final]


class RetinaNet(nn.Module):
    """Training model.  ``forward(images NHWC) -> {'regression', 'classification'}``."""

    def __init__(self, num_classes: int, backbone: str = "resnet50", num_anchors: int = 9,
                 feature_size: int = 256, prior_probability: float = 0.01):
        super().__init__()
        self.num_classes = num_classes
        self.num_anchors = num_anchors
        self.backbone_name = backbone
        if "resnet" in backbone:
            self.backbone = ResNet(backbone)
        else:
            from .extra_backbones import make_backbone
            self.backbone = make_backbone(backbone)
        c3, c4, c5 = self.backbone.out_channels[1:]
        self.fpn = FPN(c3, c4, c5, feature_size)
        self.regression_submodel = Submodel("regression_submodel", "pyramid_regression", feature_size, 256,
                                            num_anchors * 4, 0.0)
        self.classification_submodel = Submodel("classification_submodel", "pyramid_classification", feature_size,
                                                256, num_anchors * num_classes,
                                                prior_probability_bias(prior_probability))

    def features(self, images: torch.Tensor) -> List[torch.Tensor]:
        joins = self._grad_joins(images)
        if joins is None:
            C3, C4, C5 = self.backbone(images)
            return self.fpn(C3, C4, C5)
        C3, C4, C5 = self.backbone(images, joins=joins)
        return self.fpn(C3, C4, C5, joins=joins if self.backbone.joins_active else None)

    def _grad_joins(self, images: torch.Tensor):
        """GradJoins for C3 / C4 / C5 (two HIP consumers each: next stage + lateral, lateral + P6) when the
        whole path runs on fused HIP nodes; None otherwise (MXR_GRAD_JOIN=0 disables)."""
        if not (torch.is_grad_enabled() and isinstance(self.backbone, ResNet) and images.is_cuda
                and os.environ.get("MXR_GRAD_JOIN", "1") == "1" and conv_ops.get_conv_backend() != "torch"):
            return None
        from ..ops import native, native_conv
        if not native.available():
            return None
        dt = torch.bfloat16
        fpn = [self.fpn.C3_reduced, self.fpn.C4_reduced, self.fpn.C5_reduced, self.fpn.P6]
        if images.dtype != dt or not all(native_conv.hip_conv_ok(c.cin, c.cout, dt) for c in fpn):
            return None
        return {1: native_conv.GradJoin(2), 2: native_conv.GradJoin(2), 3: native_conv.GradJoin(2)}

    def forward(self, images: torch.Tensor) -> Dict[str, torch.Tensor]:
        feats = self.features(images)
        B = images.shape[0]
        if conv_ops.use_packed_heads(feats[0]):
            from ..ops import native
            packed, shapes = native.pyramid_pack(feats)
            # both towers' first layers read `packed`: their data gradients share one buffer (GradJoin)
            from ..ops import native_conv
            join = native_conv.GradJoin(2) if (torch.is_grad_enabled() and
                                               os.environ.get("MXR_GRAD_JOIN", "1") == "1") else None
            # the regression final layer (36 outputs) runs on 64-padded rows the same way as the
            # classification one: smooth-L1 may write its gradient straight into them.  (Both towers stay on
            # the compute stream: a second stream for the regression tower measured 461.7 vs 468.8-473.2
            # img/s with hx32, profiles/r3_ab_knobs.txt, and was removed.)
            self.reg_pad_sink = {} if torch.is_grad_enabled() else None
            reg = self.regression_submodel.forward_packed(packed, shapes, self.reg_pad_sink, join=join)
            # The classification final layer's data gradient runs on 64-padded rows (720 -> 768): a
            # loss kernel may write its gradient there directly (Trainer._losses_backward) instead of
            # autograd handing over (B, A, 80) rows that then get padded -- one 0.5 GB copy per step.
            self.cls_pad_sink = {} if torch.is_grad_enabled() else None
            req = getattr(self, "focal_request", None)
            if self.cls_pad_sink is not None and req is not None:
                # the Trainer's targets: the final layer may fuse the focal loss into its forward
                # (ops.conv_launch.FocalRequest)
                self.cls_pad_sink["focal"] = req
            cls = self.classification_submodel.forward_packed(packed, shapes, self.cls_pad_sink, join=join)
            return {"regression": reg.reshape(B, -1, 4), "classification": cls.reshape(B, -1, self.num_classes)}
        self.cls_pad_sink = self.reg_pad_sink = None
        reg = self.regression_submodel(feats)
        cls = self.classification_submodel(feats)
        regression = torch.cat([r.reshape(B, -1, 4) for r in reg], dim=1)
        classification = torch.cat([c.reshape(B, -1, self.num_classes) for c in cls], dim=1)
        return {"regression": regression, "classification": classification}

    # ------------------------------------------------------------------ helpers
    def convs(self) -> List[Conv2D]:
        return (self.backbone.convs() + self.fpn.convs() + self.regression_submodel.convs()
                + self.classification_submodel.convs())

    def pyramid_shapes(self, image_hw: Sequence[int]) -> List[Tuple[int, int]]:
        """Real P3..P7 shapes (used by ``make_shapes_callback``)."""
        c = self.backbone.feature_shapes(image_hw)
        C3, C4, C5 = c[1], c[2], c[3]
        p6 = self.fpn.P6.out_hw(C5)
        p7 = self.fpn.P7.out_hw(p6)
        return [tuple(C3), tuple(C4), tuple(C5), tuple(p6), tuple(p7)]

    def backbone_parameters(self):
        return list(self.backbone.parameters())

    def freeze_backbone(self) -> None:
        """``utils.model.freeze`` on the backbone (``--freeze-backbone``, train.py:82,375)."""
        for p in self.backbone.parameters():
            p.requires_grad_(False)


class RetinaNetBBox(nn.Module):
    """Prediction model: anchors -> RegressBoxes -> ClipBoxes -> sigmoid -> FilterDetections.

    Returns ``boxes (B, D, 4)``, ``scores (B, D)``, ``labels (B, D)`` padded with -1.
    """

    def __init__(self, model: RetinaNet, nms: bool = True, class_specific_filter: bool = True,
                 nms_threshold: float = 0.5, score_threshold: float = 0.05, max_detections: int = 300):
        super().__init__()
        self.model = model
        self.nms = nms
        self.class_specific_filter = class_specific_filter
        self.nms_threshold = nms_threshold
        self.score_threshold = score_threshold
        self.max_detections = max_detections
        self._anchors = anchor_ops.AnchorCache()

    @torch.no_grad()
    def forward(self, images: torch.Tensor):
        out = self.model(images)
        H, W = images.shape[1], images.shape[2]
        anchors = self._anchors.get((H, W), images.device, shapes_callback=anchor_ops.make_shapes_callback(self.model))
        from ..ops import native
        if (self.nms and self.class_specific_filter and images.is_cuda and native.available()
                and self.max_detections <= 512):
            # batched device path: threshold + per-class NMS for the whole batch in two launches,
            # decode + clip fused (only candidates are decoded), one top-k (csrc/kernels/filter.hip)
            return native.filter_detections_batched(anchors, out["regression"], out["classification"], H, W,
                                                    self.score_threshold, self.nms_threshold, self.max_detections)
        boxes = box_ops.bbox_transform_inv(anchors[None], out["regression"].float())
        boxes = box_ops.clip_boxes(boxes, H, W)
        cls = torch.sigmoid(out["classification"].float())
        res_b, res_s, res_l = [], [], []
        for i in range(images.shape[0]):
            b, s, l = box_ops.filter_detections(boxes[i], cls[i], self.nms, self.class_specific_filter,
                                                self.nms_threshold, self.score_threshold, self.max_detections)
            res_b.append(b)
            res_s.append(s)
            res_l.append(l)
        return torch.stack(res_b), torch.stack(res_s), torch.stack(res_l)


def retinanet_bbox(model: RetinaNet, **kwargs) -> RetinaNetBBox:
    return RetinaNetBBox(model, **kwargs)
