"""Caffe-style ResNet backbones (keras-resnet semantics) with Keras layer names.

Spec: keras-resnet ``ResNet18/34/50/101/152`` as built by keras-retinanet's
``resnet_retinanet`` for ``--backbone resnet50|resnet101|resnet152`` (reference flag
``/root/reference/train.py:364``):

* stem: ZeroPadding2D(3) -> conv1 7x7/s2 valid (no bias) -> bn_conv1 -> ReLU ->
  pool1 MaxPool 3x3/s2 'same';
* bottleneck: branch2a 1x1 with the stage stride (Caffe style), branch2b 3x3 (pad 1),
  branch2c 1x1 x4, shortcut branch1 1x1 + BN on block 0 of every stage, add, ReLU;
* basic (R18/R34): branch2a 3x3 stride s, branch2b 3x3, shortcut on block 0;
* frozen BN (eps 1e-5), conv kernels he_normal, no conv bias;
* R101/R152 stages 3-4 name blocks ``a, b1, b2, ...``.

Outputs C3, C4, C5.  All convs execute through ``ops.conv`` (HIP implicit GEMM on the GPU)
with the frozen BN folded into the conv epilogue and the residual add + ReLU fused into the
branch2c conv.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from ..ops import conv as conv_ops
from .layers import Conv2D

_SPECS = {
    "resnet18": ("basic", [2, 2, 2, 2], [False, False, False, False]),
    "resnet34": ("basic", [3, 4, 6, 3], [False, False, False, False]),
    "resnet50": ("bottleneck", [3, 4, 6, 3], [False, False, False, False]),
    "resnet101": ("bottleneck", [3, 4, 23, 3], [False, True, True, False]),
    "resnet152": ("bottleneck", [3, 8, 36, 3], [False, True, True, False]),
}


def _names(stage: int, block: int, numerical: bool) -> Tuple[str, str]:
    stage_char = str(stage + 2)
    if block == 0 or not numerical:
        block_char = chr(ord("a") + block)
    else:
        block_char = "b{}".format(block)
    return stage_char, block_char


class Block(nn.Module):
    def __init__(self, kind: str, cin: int, filters: int, stage: int, block: int, numerical: bool):
        super().__init__()
        s, b = _names(stage, block, numerical)
        self.name = "res{}{}".format(s, b)
        stride = 1 if (block != 0 or stage == 0) else 2
        self.kind = kind
        if kind == "bottleneck":
            self.branch2a = Conv2D(f"res{s}{b}_branch2a", cin, filters, 1, stride, 0, False, True, "he_normal",
                                   bn_name=f"bn{s}{b}_branch2a")
            self.branch2b = Conv2D(f"res{s}{b}_branch2b", filters, filters, 3, 1, 1, False, True, "he_normal",
                                   bn_name=f"bn{s}{b}_branch2b")
            self.branch2c = Conv2D(f"res{s}{b}_branch2c", filters, filters * 4, 1, 1, 0, False, True, "he_normal",
                                   bn_name=f"bn{s}{b}_branch2c")
            cout = filters * 4
        else:
            self.branch2a = Conv2D(f"res{s}{b}_branch2a", cin, filters, 3, stride, 1, False, True, "he_normal",
                                   bn_name=f"bn{s}{b}_branch2a")
            self.branch2b = Conv2D(f"res{s}{b}_branch2b", filters, filters, 3, 1, 1, False, True, "he_normal",
                                   bn_name=f"bn{s}{b}_branch2b")
            self.branch2c = None
            cout = filters
        self.branch1 = None
        if block == 0:
            self.branch1 = Conv2D(f"res{s}{b}_branch1", cin, cout, 1, stride, 0, False, False, "he_normal",
                                  bn_name=f"bn{s}{b}_branch1")
        self.cout = cout

    def chain(self) -> List[Conv2D]:
        return [self.branch2a, self.branch2b] + ([self.branch2c] if self.branch2c is not None else [])

    def forward(self, x: torch.Tensor, mask_input_grad: bool = False, grad_premasked: bool = False,
                join=None) -> torch.Tensor:
        chain = self.chain()
        if conv_ops.fused_blocks(x, chain + [self.branch1]):
            from ..ops import native_conv
            return native_conv.residual_block(x, chain, self.branch1, mask_input_grad, grad_premasked, join)
        if join is not None:
            raise RuntimeError("GradJoin needs the fused HIP block path")
        shortcut = self.branch1(x) if self.branch1 is not None else x
        y = self.branch2a(x)
        if self.branch2c is not None:
            y = self.branch2b(y)
            return self.branch2c(y, residual=shortcut, relu=True)
        return self.branch2b(y, residual=shortcut, relu=True)

    def convs(self) -> List[Conv2D]:
        return [c for c in (self.branch2a, self.branch2b, self.branch2c, self.branch1) if c is not None]


class ResNet(nn.Module):
    """Caffe-style ResNet returning [C3, C4, C5] (NHWC)."""

    def __init__(self, name: str = "resnet50"):
        super().__init__()
        if name not in _SPECS:
            raise ValueError("Backbone '{}' not recognized.".format(name))
        kind, blocks, numerical = _SPECS[name]
        self.name = name
        self.conv1 = Conv2D("conv1", 3, 64, 7, 2, 3, False, True, "he_normal", bn_name="bn_conv1")
        stages = []
        cin = 64
        self.out_channels: List[int] = []
        for stage_id, n in enumerate(blocks):
            filters = 64 * 2 ** stage_id
            stage = nn.ModuleList()
            for block_id in range(n):
                blk = Block(kind, cin, filters, stage_id, block_id, block_id > 0 and numerical[stage_id])
                stage.append(blk)
                cin = blk.cout
            self.out_channels.append(cin)
            stages.append(stage)
        self.stages = nn.ModuleList(stages)
        # weight gradients of these blocks stay on the compute stream (ops.conv_wgrad._side): they are the
        # last of the backward, and behind the side stream's backlog they would run while the compute
        # stream sits idle before the optimizer -- split between the two streams the tail shortens
        main_blocks = set(filter(None, os.environ.get("MXR_MAIN_WGRAD_BLOCKS", "res2c").split(",")))
        for stage in self.stages:
            for blk in stage:
                if blk.name in main_blocks:
                    for c in blk.chain() + ([blk.branch1] if blk.branch1 is not None else []):
                        c.weight.mxr_main_wgrad = True

    def forward(self, x: torch.Tensor, joins: Optional[Dict[int, object]] = None) -> List[torch.Tensor]:
        """``joins``: {stage index: ops.native_conv.GradJoin} for stage outputs with several HIP consumers
        (RetinaNet: C3 / C4 / C5 also feed the FPN); the next stage's first block joins that gradient and
        the producing block skips its relu backward.  Only honoured on the fused block path."""
        if conv_ops.stem_fused(x, self.conv1):
            # conv1 + bn_conv1 + relu + pool1 as one HIP node (ops/stem.py)
            from ..ops import stem as _stem
            x = _stem.stem(x, self.conv1, conv_ops.same_pads(self.conv1.out_hw(x.shape[1:3]), 3, 2))
        else:
            x = self.conv1(x)
            x = conv_ops.maxpool_same(x, 3, 2)
        outs = []
        fused = conv_ops.fused_blocks(x, [c for st in self.stages for b in st for c in b.convs()])
        joins = joins if fused else None
        self.joins_active = joins is not None
        for si, stage in enumerate(self.stages):
            for j, blk in enumerate(stage):
                if fused:
                    # inside a stage a block's output feeds only the next block: that block fuses
                    # this block's output-relu backward into its own last dgrad.  C2 (stage 0's output)
                    # is not a pyramid input, so the same holds across the res2 -> res3 boundary; C3..C5
                    # also feed the FPN: with a GradJoin the last consumer applies the mask, else the
                    # producing block keeps its own relu backward.
                    last = j == len(stage) - 1
                    jin = joins.get(si - 1) if (joins and j == 0) else None
                    jout = joins.get(si) if (joins and last) else None
                    x = blk(x, mask_input_grad=j > 0 or si == 1, grad_premasked=not last or si == 0 or jout is not None,
                            join=jin)
                else:
                    x = blk(x)
            outs.append(x)
        return outs[1:]

    def convs(self) -> List[Conv2D]:
        out = [self.conv1]
        for stage in self.stages:
            for blk in stage:
                out.extend(blk.convs())
        return out

    def feature_shapes(self, image_hw: Sequence[int]) -> List[Tuple[int, int]]:
        """Shapes of C2..C5 for an input of ``image_hw`` (pure arithmetic, no forward)."""
        hw = self.conv1.out_hw(image_hw)
        pads = conv_ops.same_pads(hw, 3, 2)
        hw = conv_ops.out_hw(hw, 3, 2, pads)
        shapes = []
        for stage in self.stages:
            for blk in stage:
                hw = blk.branch2a.out_hw(hw)
                hw = blk.branch2b.out_hw(hw)
            shapes.append(hw)
        return shapes
