"""Experimental backbones of the keras-retinanet registry: VGG16/19, MobileNet (v1), DenseNet.

The reference accepts any registered backbone name (``--backbone``, ``/root/reference/train.py:364``)
and warns that only ResNet-50 is properly tested (``train.py:323-324``); for vgg/densenet it
measures the real pyramid shapes with ``make_shapes_callback(model)`` (``train.py:428-432``).
Layer names follow keras.applications so ``--weights`` by-name loading lines up:

* VGG16/19: ``block{b}_conv{i}`` (3x3 same + bias + ReLU), ``block{b}_pool``; C3..C5 =
  block3_pool / block4_pool / block5_pool;
* MobileNet(alpha): ``conv1`` 3x3/s2 + ``conv1_bn``, 13 depthwise-separable blocks
  ``conv_dw_{i}`` / ``conv_pw_{i}`` (+ ``_bn``, ReLU6); C3..C5 = conv_pw_5/11/13 outputs;
* DenseNet121/169/201: ``conv1/conv`` 7x7/s2, pool, dense blocks ``conv{s}_block{i}`` (BN-ReLU-1x1
  (4k)-BN-ReLU-3x3(k), concat), transitions ``pool{s}`` (BN-ReLU-1x1, avg-pool 2); C3..C5 = the
  outputs of dense blocks 2, 3, 4.

As in keras.applications, BN in MobileNet/DenseNet is ordinary (trainable, batch statistics in
training).  VGG convs run through the same conv front-end as ResNet (HIP implicit GEMM when the
shape class is covered); depthwise and BN-heavy backbones use PyTorch/MIOpen ops.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .layers import Conv2D


def _nchw(x):
    return x.permute(0, 3, 1, 2)


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _bn_weights(name, bnact):
    b = bnact.bn
    return [(name + "/gamma:0", b.weight, "plain"), (name + "/beta:0", b.bias, "plain"),
            (name + "/moving_mean:0", b.running_mean, "plain"), (name + "/moving_variance:0", b.running_var, "plain")]


def _autocast(x):
    """Run torch-op backbones in the trainer's compute dtype (BN statistics stay fp32)."""
    return torch.autocast(device_type=x.device.type, dtype=x.dtype, enabled=x.dtype != torch.float32)


class _ShapeProbe:
    """Pyramid shapes measured with a real (no-grad) forward, cached per input size."""

    def feature_shapes_probe(self, image_hw: Sequence[int]) -> List[Tuple[int, int]]:
        key = (int(image_hw[0]), int(image_hw[1]))
        cache = self.__dict__.setdefault("_shape_cache", {})
        if key not in cache:
            p = next(self.parameters())
            with torch.no_grad():
                x = torch.zeros((1, key[0], key[1], 3), device=p.device, dtype=torch.float32)
                was = self.training
                self.eval()
                outs = self(x)
                self.train(was)
            cache[key] = [(int(o.shape[1]), int(o.shape[2])) for o in outs]
        return cache[key]


class VGG(nn.Module, _ShapeProbe):
    CFG = {"vgg16": [2, 2, 3, 3, 3], "vgg19": [2, 2, 4, 4, 4]}

    def __init__(self, name: str = "vgg16"):
        super().__init__()
        self.name = name
        widths = [64, 128, 256, 512, 512]
        blocks = []
        cin = 3
        for b, (n, w) in enumerate(zip(self.CFG[name], widths)):
            layers = nn.ModuleList()
            for i in range(n):
                layers.append(Conv2D("block{}_conv{}".format(b + 1, i + 1), cin, w, 3, 1, "same", True, True,
                                     "glorot_uniform"))
                cin = w
            blocks.append(layers)
        self.blocks = nn.ModuleList(blocks)
        self.out_channels = [128, 256, 512, 512]

    def forward(self, x):
        outs = []
        for b, layers in enumerate(self.blocks):
            for c in layers:
                x = c(x)
            x = _nhwc(F.max_pool2d(_nchw(x), 2, 2))
            if b >= 2:
                outs.append(x)
        return outs

    def convs(self):
        return [c for layers in self.blocks for c in layers]

    def keras_layers(self):
        return [(c.keras_name, [(c.keras_name + "/kernel:0", c.weight, "kernel"),
                                (c.keras_name + "/bias:0", c.bias, "plain")]) for c in self.convs()]

    def feature_shapes(self, image_hw):
        h, w = image_hw
        shapes = []
        for b in range(5):
            h, w = h // 2, w // 2
            shapes.append((h, w))
        return [shapes[0]] + shapes[2:5]


class _BNAct(nn.Module):
    def __init__(self, c, act="relu", eps=1e-3, momentum=0.01):
        super().__init__()
        self.bn = nn.BatchNorm2d(c, eps=eps, momentum=momentum)
        self.act = act

    def forward(self, x):    # NCHW
        x = self.bn(x)
        if self.act == "relu6":
            return F.relu6(x)
        if self.act == "relu":
            return F.relu(x)
        return x


class MobileNet(nn.Module, _ShapeProbe):
    STRIDES = [1, 2, 1, 2, 1, 2, 1, 1, 1, 1, 1, 2, 1]
    FILTERS = [64, 128, 128, 256, 256, 512, 512, 512, 512, 512, 512, 1024, 1024]

    def __init__(self, alpha: float = 1.0):
        super().__init__()
        c = int(32 * alpha)
        self.conv1 = nn.Conv2d(3, c, 3, 2, 0, bias=False)
        self.conv1_bn = _BNAct(c, "relu6")
        self.dw, self.dw_bn, self.pw, self.pw_bn, self.strides = (nn.ModuleList(), nn.ModuleList(), nn.ModuleList(),
                                                                   nn.ModuleList(), [])
        for s, f in zip(self.STRIDES, self.FILTERS):
            f = int(f * alpha)
            self.dw.append(nn.Conv2d(c, c, 3, s, 0, groups=c, bias=False))
            self.dw_bn.append(_BNAct(c, "relu6"))
            self.pw.append(nn.Conv2d(c, f, 1, 1, 0, bias=False))
            self.pw_bn.append(_BNAct(f, "relu6"))
            self.strides.append(s)
            c = f
        self.out_channels = [0, int(256 * alpha), int(512 * alpha), int(1024 * alpha)]

    def forward(self, x):
        dt = x.dtype
        with _autocast(x):
            x = _nchw(x)
            x = F.pad(x, (0, 1, 0, 1))                   # keras: ZeroPadding2D(((0,1),(0,1))) + valid s2
            x = self.conv1_bn(self.conv1(x))
            outs = []
            for i in range(13):
                x = F.pad(x, (1, 1, 1, 1)) if self.strides[i] == 1 else F.pad(x, (0, 1, 0, 1))
                x = self.dw_bn[i](self.dw[i](x))
                x = self.pw_bn[i](self.pw[i](x))
                if i + 1 in (5, 11, 13):
                    outs.append(_nhwc(x).to(dt))
        return outs

    def convs(self):
        return []

    def keras_layers(self):
        out = [("conv1", [("conv1/kernel:0", self.conv1.weight, "oihw")]), ("conv1_bn", _bn_weights("conv1_bn",
                                                                                                    self.conv1_bn))]
        for i in range(13):
            n = i + 1
            out.append(("conv_dw_%d" % n, [("conv_dw_%d/depthwise_kernel:0" % n, self.dw[i].weight, "dw")]))
            out.append(("conv_dw_%d_bn" % n, _bn_weights("conv_dw_%d_bn" % n, self.dw_bn[i])))
            out.append(("conv_pw_%d" % n, [("conv_pw_%d/kernel:0" % n, self.pw[i].weight, "oihw")]))
            out.append(("conv_pw_%d_bn" % n, _bn_weights("conv_pw_%d_bn" % n, self.pw_bn[i])))
        return out

    def feature_shapes(self, image_hw):
        return [(1, 1)] + self.feature_shapes_probe(image_hw)


class _DenseLayer(nn.Module):
    def __init__(self, cin, growth):
        super().__init__()
        self.bn1 = _BNAct(cin, "relu", eps=1.001e-5)
        self.conv1 = nn.Conv2d(cin, 4 * growth, 1, bias=False)
        self.bn2 = _BNAct(4 * growth, "relu", eps=1.001e-5)
        self.conv2 = nn.Conv2d(4 * growth, growth, 3, padding=1, bias=False)

    def forward(self, x):
        y = self.conv2(self.bn2(self.conv1(self.bn1(x))))
        return torch.cat([x, y], dim=1)


class DenseNet(nn.Module, _ShapeProbe):
    BLOCKS = {"densenet121": [6, 12, 24, 16], "densenet169": [6, 12, 32, 32], "densenet201": [6, 12, 48, 32]}

    def __init__(self, name: str = "densenet121", growth: int = 32):
        super().__init__()
        blocks = self.BLOCKS[name]
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 0, bias=False)
        self.conv1_bn = _BNAct(64, "relu", eps=1.001e-5)
        c = 64
        self.dense = nn.ModuleList()
        self.trans = nn.ModuleList()
        outs = []
        for i, n in enumerate(blocks):
            layers = nn.ModuleList()
            for _ in range(n):
                layers.append(_DenseLayer(c, growth))
                c += growth
            self.dense.append(layers)
            outs.append(c)
            if i != len(blocks) - 1:
                self.trans.append(nn.ModuleDict({"bn": _BNAct(c, "relu", eps=1.001e-5),
                                                 "conv": nn.Conv2d(c, c // 2, 1, bias=False)}))
                c = c // 2
        self.out_channels = outs

    def forward(self, x):
        dt = x.dtype
        with _autocast(x):
            x = _nchw(x)
            x = self.conv1_bn(self.conv1(F.pad(x, (3, 3, 3, 3))))
            x = F.max_pool2d(F.pad(x, (1, 1, 1, 1)), 3, 2)
            outs = []
            for i, layers in enumerate(self.dense):
                for l in layers:
                    x = l(x)
                if i >= 1:
                    outs.append(_nhwc(x).to(dt))
                if i < len(self.trans):
                    t = self.trans[i]
                    x = F.avg_pool2d(t["conv"](t["bn"](x)), 2, 2)
        return outs

    def convs(self):
        return []

    def keras_layers(self):
        out = [("conv1/conv", [("conv1/conv/kernel:0", self.conv1.weight, "oihw")]),
               ("conv1/bn", _bn_weights("conv1/bn", self.conv1_bn))]
        for s, layers in enumerate(self.dense):
            for i, l in enumerate(layers):
                p = "conv{}_block{}".format(s + 2, i + 1)
                out += [(p + "_0_bn", _bn_weights(p + "_0_bn", l.bn1)),
                        (p + "_1_conv", [(p + "_1_conv/kernel:0", l.conv1.weight, "oihw")]),
                        (p + "_1_bn", _bn_weights(p + "_1_bn", l.bn2)),
                        (p + "_2_conv", [(p + "_2_conv/kernel:0", l.conv2.weight, "oihw")])]
            if s < len(self.trans):
                p = "pool{}".format(s + 2)
                t = self.trans[s]
                out += [(p + "_bn", _bn_weights(p + "_bn", t["bn"])),
                        (p + "_conv", [(p + "_conv/kernel:0", t["conv"].weight, "oihw")])]
        return out

    def feature_shapes(self, image_hw):
        return [(1, 1)] + self.feature_shapes_probe(image_hw)


def make_backbone(name: str) -> nn.Module:
    if name in VGG.CFG:
        return VGG(name)
    if name.startswith("mobilenet"):
        # keras-retinanet names: mobilenet{128,160,192,224}_{alpha}
        alpha = float(name.split("_")[1]) if "_" in name else 1.0
        return MobileNet(alpha)
    if name in DenseNet.BLOCKS:
        return DenseNet(name)
    raise ValueError("Backbone '{}' not recognized.".format(name))


from . import Backbone  # noqa: E402  (models/__init__ imports this module lazily)


class _GenericBackbone(Backbone):
    def validate(self):
        ok = self.backbone in self.allowed or any(self.backbone.startswith(a) for a in self.allowed if a.endswith("_"))
        if not ok:
            raise ValueError("Backbone ('{}') not in allowed backbones ({}).".format(self.backbone, self.allowed))

    def retinanet(self, num_classes, modifier=None, **kwargs):
        from .retinanet import RetinaNet
        model = RetinaNet(num_classes, backbone=self.backbone, **kwargs)
        if modifier is not None:
            model = modifier(model) or model
        return model

    def imagenet_filename(self):
        return "{}_weights_tf_dim_ordering_tf_kernels_notop.h5".format(self.backbone)


class VGGBackbone(_GenericBackbone):
    allowed = ("vgg16", "vgg19")


class MobileNetBackbone(_GenericBackbone):
    allowed = ("mobilenet128_", "mobilenet160_", "mobilenet192_", "mobilenet224_")


class DenseNetBackbone(_GenericBackbone):
    allowed = ("densenet121", "densenet169", "densenet201")


def lookup(name: str):
    if "vgg" in name:
        return VGGBackbone(name)
    if "mobilenet" in name:
        return MobileNetBackbone(name)
    if "densenet" in name:
        return DenseNetBackbone(name)
    raise NotImplementedError("Backbone class for  '{}' not implemented.".format(name))
