"""Anchor generation and anchor-target assignment.

Behavioural spec: keras-retinanet ``utils.anchors`` as imported by the reference at
``/root/reference/train.py:51`` (``anchor_targets_bbox``, ``make_shapes_callback``) and used
implicitly by every generator built at ``train.py:197-293``.  SURVEY §2.8.4-2.8.5.

Two implementations live here:

* a float64 numpy *oracle* (``anchor_targets_bbox``) that reproduces the reference
  semantics literally (IoU with the "+1 pixel" convention, 0.4/0.5 thresholds,
  outside-centre ignore, corner-offset regression with std 0.2);
* a batched torch implementation (``anchor_targets_torch``) that runs on the GPU (or CPU)
  with compact outputs -- per-anchor ``state`` (-1 ignore / 0 negative / 1 positive),
  ``label`` (class id of the matched box) and ``regression`` (A, 4) -- instead of the
  reference's 65 MB/image one-hot tensor.  The fused HIP kernel in
  ``csrc/kernels/targets.hip`` implements the same contract.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch


@dataclass
class AnchorParameters:
    """Anchor configuration (keras-retinanet ``AnchorParameters.default``)."""

    sizes: Sequence[float] = (32, 64, 128, 256, 512)
    strides: Sequence[int] = (8, 16, 32, 64, 128)
    ratios: Sequence[float] = (0.5, 1.0, 2.0)
    scales: Sequence[float] = (2.0 ** 0.0, 2.0 ** (1.0 / 3.0), 2.0 ** (2.0 / 3.0))

    def num_anchors(self) -> int:
        return len(self.ratios) * len(self.scales)


AnchorParameters.default = AnchorParameters()  # type: ignore[attr-defined]

PYRAMID_LEVELS = (3, 4, 5, 6, 7)
BOX_STD = 0.2
BOX_MEAN = 0.0
POSITIVE_OVERLAP = 0.5
NEGATIVE_OVERLAP = 0.4


def generate_anchors(base_size: float = 16, ratios=None, scales=None) -> np.ndarray:
    """Reference anchors (centred at the origin) for one pyramid level.

    Ordering is ratio-major, scale-minor, which is also the channel ordering of the
    regression/classification heads.
    """
    ratios = np.asarray(AnchorParameters.default.ratios if ratios is None else ratios, dtype=np.float64)
    scales = np.asarray(AnchorParameters.default.scales if scales is None else scales, dtype=np.float64)
    rr = np.repeat(ratios, len(scales))          # ratio for anchor i
    ss = np.tile(scales, len(ratios))            # scale for anchor i
    side = base_size * ss
    area = side * side
    w = np.sqrt(area / rr)
    h = w * rr
    out = np.stack([-0.5 * w, -0.5 * h, 0.5 * w, 0.5 * h], axis=1)
    return out


def shift(shape: Tuple[int, int], stride: int, anchors: np.ndarray) -> np.ndarray:
    """Tile ``anchors`` over a (H, W) feature map; centres at (i + 0.5) * stride.

    Result is (H*W*A, 4), position-major (row-major over y then x), anchor-minor.
    """
    h, w = int(shape[0]), int(shape[1])
    sx = (np.arange(w, dtype=np.float64) + 0.5) * stride
    sy = (np.arange(h, dtype=np.float64) + 0.5) * stride
    gx, gy = np.meshgrid(sx, sy)
    shifts = np.stack([gx.ravel(), gy.ravel(), gx.ravel(), gy.ravel()], axis=1)
    return (shifts[:, None, :] + anchors[None, :, :]).reshape(-1, 4)


def guess_shapes(image_shape: Sequence[int], pyramid_levels=PYRAMID_LEVELS) -> List[Tuple[int, int]]:
    """Closed-form feature-map shapes for the ResNet backbone: ceil(size / 2**level)."""
    h, w = int(image_shape[0]), int(image_shape[1])
    return [((h + 2 ** x - 1) // (2 ** x), (w + 2 ** x - 1) // (2 ** x)) for x in pyramid_levels]


def anchors_for_shape(image_shape: Sequence[int], pyramid_levels=PYRAMID_LEVELS,
                      anchor_params: Optional[AnchorParameters] = None,
                      shapes_callback=None) -> np.ndarray:
    """All anchors (float64) for an input image of ``image_shape`` (H, W[, C])."""
    p = anchor_params or AnchorParameters.default
    shapes = (shapes_callback or guess_shapes)(image_shape[:2], pyramid_levels)
    out = []
    for idx, lvl in enumerate(pyramid_levels):
        base = generate_anchors(p.sizes[idx], p.ratios, p.scales)
        out.append(shift(shapes[idx], p.strides[idx], base))
    return np.concatenate(out, axis=0)


def level_sizes(image_shape, pyramid_levels=PYRAMID_LEVELS) -> List[int]:
    """Number of anchors on each pyramid level."""
    A = AnchorParameters.default.num_anchors()
    return [h * w * A for (h, w) in guess_shapes(image_shape, pyramid_levels)]


def make_shapes_callback(model):
    """Shape oracle that measures the real feature-map shapes of ``model``.

    The reference swaps this in for vgg/densenet backbones (``train.py:428-432``).
    ``model`` must expose ``pyramid_shapes(image_shape)``.
    """
    def get_shapes(image_shape, pyramid_levels=PYRAMID_LEVELS):
        return model.pyramid_shapes(tuple(image_shape[:2]))
    return get_shapes


# ----------------------------------------------------------------------------------------
# numpy oracle
# ----------------------------------------------------------------------------------------

def compute_overlap(boxes: np.ndarray, query_boxes: np.ndarray) -> np.ndarray:
    """IoU matrix (N, K) with the reference's "+1 pixel" convention.

    Replaces the Cython ``compute_overlap.pyx``; the native C++ version lives in
    ``csrc/cpu/boxes_cpu.cpp`` and is used when the CPU extension is built.
    """
    boxes = np.asarray(boxes, dtype=np.float64)
    q = np.asarray(query_boxes, dtype=np.float64)
    if q.shape[0] == 0 or boxes.shape[0] == 0:
        return np.zeros((boxes.shape[0], q.shape[0]), dtype=np.float64)
    area_q = (q[:, 2] - q[:, 0] + 1) * (q[:, 3] - q[:, 1] + 1)
    iw = np.minimum(boxes[:, None, 2], q[None, :, 2]) - np.maximum(boxes[:, None, 0], q[None, :, 0]) + 1
    ih = np.minimum(boxes[:, None, 3], q[None, :, 3]) - np.maximum(boxes[:, None, 1], q[None, :, 1]) + 1
    iw = np.clip(iw, 0, None)
    ih = np.clip(ih, 0, None)
    inter = iw * ih
    ua = (boxes[:, None, 2] - boxes[:, None, 0] + 1) * (boxes[:, None, 3] - boxes[:, None, 1] + 1) + area_q[None, :] - inter
    out = np.where((iw > 0) & (ih > 0), inter / ua, 0.0)
    return out


def bbox_transform(anchors: np.ndarray, gt_boxes: np.ndarray, mean=BOX_MEAN, std=BOX_STD) -> np.ndarray:
    """Corner-offset regression targets normalised by anchor width/height."""
    aw = anchors[:, 2] - anchors[:, 0]
    ah = anchors[:, 3] - anchors[:, 1]
    t = np.stack([(gt_boxes[:, 0] - anchors[:, 0]) / aw,
                  (gt_boxes[:, 1] - anchors[:, 1]) / ah,
                  (gt_boxes[:, 2] - anchors[:, 2]) / aw,
                  (gt_boxes[:, 3] - anchors[:, 3]) / ah], axis=1)
    return (t - mean) / std


def anchor_targets_bbox(image_shape, annotations: np.ndarray, num_classes: int, mask_shape=None,
                        negative_overlap=NEGATIVE_OVERLAP, positive_overlap=POSITIVE_OVERLAP,
                        shapes_callback=None, anchors: Optional[np.ndarray] = None):
    """Reference-semantics targets for one image.

    Returns ``(labels (A, C) with -1 rows for ignore, regression (A, 4), state (A,))``.
    """
    if anchors is None:
        anchors = anchors_for_shape(image_shape, shapes_callback=shapes_callback)
    A = anchors.shape[0]
    annotations = np.asarray(annotations, dtype=np.float64).reshape(-1, 5)
    labels = np.full((A, num_classes), -1.0)
    state = np.full((A,), -1.0)
    if annotations.shape[0]:
        overlaps = compute_overlap(anchors, annotations[:, :4])
        arg = np.argmax(overlaps, axis=1)
        mx = overlaps[np.arange(A), arg]
        neg = mx < negative_overlap
        labels[neg, :] = 0
        state[neg] = 0
        matched = annotations[arg]
        pos = mx >= positive_overlap
        labels[pos, :] = 0
        labels[pos, matched[pos, 4].astype(int)] = 1
        state[pos] = 1
    else:
        labels[:] = 0
        state[:] = 0
        matched = np.zeros((A, 5))
        matched[:, :4] = anchors
    mh, mw = (image_shape if mask_shape is None else mask_shape)[:2]
    cx = (anchors[:, 0] + anchors[:, 2]) / 2
    cy = (anchors[:, 1] + anchors[:, 3]) / 2
    outside = (cx >= mw) | (cy >= mh)
    labels[outside, :] = -1
    state[outside] = -1
    regression = bbox_transform(anchors, matched[:, :4])
    return labels, regression, state


# ----------------------------------------------------------------------------------------
# batched torch implementation (device-resident targets)
# ----------------------------------------------------------------------------------------

def centers_round_down(anchors64: np.ndarray) -> np.ndarray:
    """Anchor centres (A, 2) as the largest float32 <= the float64 centre.

    The reference tests ``cx >= W`` in float64; rounding the centre DOWN to float32 keeps every
    comparison against an integer image size identical (e.g. 95.99999999999999 must not become 96).
    """
    c64 = np.stack([(anchors64[:, 0] + anchors64[:, 2]) / 2, (anchors64[:, 1] + anchors64[:, 3]) / 2], axis=1)
    c32 = c64.astype(np.float32)
    up = c32.astype(np.float64) > c64
    c32[up] = np.nextafter(c32[up], np.float32(-np.inf))
    return c32


class AnchorCache:
    """Per-(padded shape, device) cache of anchors (float32 (A, 4)) and their centres (A, 2)."""

    def __init__(self, anchor_params: Optional[AnchorParameters] = None):
        self.p = anchor_params or AnchorParameters.default
        self._cache = {}

    def _entry(self, image_shape, device, shapes_callback):
        key = (int(image_shape[0]), int(image_shape[1]), str(device))
        t = self._cache.get(key)
        if t is None:
            a = anchors_for_shape(image_shape, anchor_params=self.p, shapes_callback=shapes_callback)
            t = (torch.from_numpy(a.astype(np.float32)).to(device),
                 torch.from_numpy(centers_round_down(a)).to(device))
            self._cache[key] = t
        return t

    def get(self, image_shape, device, shapes_callback=None) -> torch.Tensor:
        return self._entry(image_shape, device, shapes_callback)[0]

    def centers(self, image_shape, device, shapes_callback=None) -> torch.Tensor:
        return self._entry(image_shape, device, shapes_callback)[1]


def anchor_targets_torch(anchors: torch.Tensor, gt: torch.Tensor, gt_count: torch.Tensor,
                         mask_hw: torch.Tensor,
                         negative_overlap=NEGATIVE_OVERLAP, positive_overlap=POSITIVE_OVERLAP,
                         centers: Optional[torch.Tensor] = None):
    """Batched targets.

    Args:
      anchors: (A, 4) float32.
      gt: (B, G, 5) float32 padded boxes ``[x1, y1, x2, y2, label]``; rows >= gt_count ignored.
      gt_count: (B,) int number of valid boxes per image.
      mask_hw: (B, 2) unpadded image (H, W) per image.
    Returns:
      state (B, A) int8, label (B, A) int32, regression (B, A, 4) float32.
    """
    B, G = gt.shape[0], gt.shape[1]
    A = anchors.shape[0]
    dev = anchors.device
    ax1, ay1, ax2, ay2 = anchors.unbind(-1)
    if G > 0:
        g = gt[..., :4]
        gx1, gy1, gx2, gy2 = [g[..., i][:, None, :] for i in range(4)]  # (B,1,G)
        iw = (torch.minimum(ax2[None, :, None], gx2) - torch.maximum(ax1[None, :, None], gx1) + 1).clamp_min(0)
        ih = (torch.minimum(ay2[None, :, None], gy2) - torch.maximum(ay1[None, :, None], gy1) + 1).clamp_min(0)
        inter = iw * ih
        area_a = ((ax2 - ax1 + 1) * (ay2 - ay1 + 1))[None, :, None]
        area_g = ((gx2 - gx1 + 1) * (gy2 - gy1 + 1))
        iou = inter / (area_a + area_g - inter)
        valid = torch.arange(G, device=dev)[None, None, :] < gt_count.to(dev)[:, None, None]
        iou = torch.where(valid, iou, torch.full_like(iou, -1.0))
        mx, arg = iou.max(dim=2)                      # first max wins, like np.argmax
        has = (gt_count.to(dev) > 0)[:, None]
        mx = torch.where(has, mx, torch.zeros_like(mx))
        state = torch.full((B, A), -1, dtype=torch.int8, device=dev)
        state = torch.where(mx < negative_overlap, torch.zeros_like(state), state)
        state = torch.where(mx >= positive_overlap, torch.ones_like(state), state)
        matched = torch.gather(gt, 1, arg[..., None].expand(B, A, 5))
        matched = torch.where(has[..., None], matched,
                              torch.cat([anchors, torch.zeros_like(anchors[:, :1])], 1)[None].expand(B, A, 5))
        label = matched[..., 4].to(torch.int32)
        mbox = matched[..., :4]
    else:
        state = torch.zeros((B, A), dtype=torch.int8, device=dev)
        label = torch.zeros((B, A), dtype=torch.int32, device=dev)
        mbox = anchors[None].expand(B, A, 4)
    if centers is None:
        centers = torch.from_numpy(centers_round_down(anchors.double().cpu().numpy())).to(dev)
    cx, cy = centers[:, 0], centers[:, 1]
    mh = mask_hw[:, 0].to(dev).to(anchors.dtype)[:, None]
    mw = mask_hw[:, 1].to(dev).to(anchors.dtype)[:, None]
    outside = (cx[None] >= mw) | (cy[None] >= mh)
    state = torch.where(outside, torch.full_like(state, -1), state)
    aw = (ax2 - ax1)[None]
    ah = (ay2 - ay1)[None]
    reg = torch.stack([(mbox[..., 0] - ax1[None]) / aw, (mbox[..., 1] - ay1[None]) / ah,
                       (mbox[..., 2] - ax2[None]) / aw, (mbox[..., 3] - ay2[None]) / ah], -1)
    reg = (reg - BOX_MEAN) / BOX_STD
    return state, label, reg
