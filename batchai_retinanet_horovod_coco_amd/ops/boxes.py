"""Box decode / clip / NMS / detection filtering (prediction graph).

Behavioural spec: keras-retinanet ``layers.RegressBoxes``, ``layers.ClipBoxes`` and
``layers.FilterDetections`` used by ``retinanet_bbox`` at ``/root/reference/train.py:95,408``
(SURVEY §2.8.8).  The torch code here is the oracle and the CPU path; on a GPU the fused HIP
kernels in ``csrc/kernels/detect.hip`` (decode+clip, bitmask NMS) are dispatched through
``ops.native``.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .anchors import BOX_MEAN, BOX_STD


def bbox_transform_inv(anchors: torch.Tensor, deltas: torch.Tensor, mean=BOX_MEAN, std=BOX_STD) -> torch.Tensor:
    """Inverse of the corner-offset encoding.  anchors (..., A, 4), deltas (..., A, 4)."""
    aw = anchors[..., 2] - anchors[..., 0]
    ah = anchors[..., 3] - anchors[..., 1]
    d = deltas * std + mean
    x1 = anchors[..., 0] + d[..., 0] * aw
    y1 = anchors[..., 1] + d[..., 1] * ah
    x2 = anchors[..., 2] + d[..., 2] * aw
    y2 = anchors[..., 3] + d[..., 3] * ah
    return torch.stack([x1, y1, x2, y2], dim=-1)


def clip_boxes(boxes: torch.Tensor, height: float, width: float) -> torch.Tensor:
    """Clamp x to [0, W] and y to [0, H] (0.4-era ClipBoxes bound, pinned by a unit test)."""
    x1 = boxes[..., 0].clamp(0, width)
    y1 = boxes[..., 1].clamp(0, height)
    x2 = boxes[..., 2].clamp(0, width)
    y2 = boxes[..., 3].clamp(0, height)
    return torch.stack([x1, y1, x2, y2], dim=-1)


def box_iou_plain(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """IoU without the +1 convention (tf.image.non_max_suppression semantics)."""
    area_a = (a[:, 2] - a[:, 0]).clamp_min(0) * (a[:, 3] - a[:, 1]).clamp_min(0)
    area_b = (b[:, 2] - b[:, 0]).clamp_min(0) * (b[:, 3] - b[:, 1]).clamp_min(0)
    lt = torch.maximum(a[:, None, :2], b[None, :, :2])
    rb = torch.minimum(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt).clamp_min(0)
    inter = wh[..., 0] * wh[..., 1]
    union = area_a[:, None] + area_b[None, :] - inter
    return torch.where(union > 0, inter / union, torch.zeros_like(inter))


def nms(boxes: torch.Tensor, scores: torch.Tensor, iou_threshold: float, max_output: int) -> torch.Tensor:
    """Greedy NMS, keeps indices in decreasing-score order (TF semantics: suppress if IoU > thr)."""
    if boxes.numel() == 0:
        return torch.zeros((0,), dtype=torch.long, device=boxes.device)
    order = torch.argsort(scores, descending=True, stable=True)
    b = boxes[order]
    iou = box_iou_plain(b, b)
    n = b.shape[0]
    suppressed = torch.zeros(n, dtype=torch.bool, device=boxes.device)
    keep = []
    iou_cpu = iou.cpu()
    sup = suppressed.cpu()
    for i in range(n):
        if sup[i]:
            continue
        keep.append(i)
        if len(keep) >= max_output:
            break
        sup |= iou_cpu[i] > iou_threshold
    return order[torch.tensor(keep, dtype=torch.long, device=boxes.device)]


def filter_detections(boxes: torch.Tensor, classification: torch.Tensor, nms_enabled: bool = True,
                      class_specific_filter: bool = True, nms_threshold: float = 0.5,
                      score_threshold: float = 0.05, max_detections: int = 300,
                      backend: Optional[str] = None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Per-image FilterDetections.  boxes (A, 4), classification (A, C) probabilities.

    Returns boxes (max_det, 4), scores (max_det,), labels (max_det,) padded with -1.
    """
    from . import native  # local import: avoids a cycle at package import
    if backend is None:
        backend = "hip" if (boxes.is_cuda and native.available()) else "torch"
    dev = boxes.device
    all_idx, all_lab = [], []
    if class_specific_filter:
        C = classification.shape[1]
        for c in range(C):
            s = classification[:, c]
            idx = torch.nonzero(s > score_threshold).flatten()
            if idx.numel() == 0:
                continue
            if nms_enabled:
                if backend == "hip":
                    k = native.nms(boxes[idx].float().contiguous(), s[idx].float().contiguous(), nms_threshold, max_detections)
                else:
                    k = nms(boxes[idx], s[idx], nms_threshold, max_detections)
                idx = idx[k]
            all_idx.append(idx)
            all_lab.append(torch.full_like(idx, c))
    else:
        s, lab = classification.max(dim=1)
        idx = torch.nonzero(s > score_threshold).flatten()
        if nms_enabled and idx.numel():
            k = nms(boxes[idx], s[idx], nms_threshold, max_detections)
            idx = idx[k]
        all_idx.append(idx)
        all_lab.append(lab[idx])
    out_b = torch.full((max_detections, 4), -1.0, device=dev)
    out_s = torch.full((max_detections,), -1.0, device=dev)
    out_l = torch.full((max_detections,), -1, dtype=torch.int32, device=dev)
    if all_idx:
        idx = torch.cat(all_idx)
        lab = torch.cat(all_lab)
        if idx.numel():
            sc = classification[idx, lab]
            k = min(max_detections, sc.numel())
            top_s, top_i = torch.topk(sc, k)
            out_b[:k] = boxes[idx[top_i]].float()
            out_s[:k] = top_s.float()
            out_l[:k] = lab[top_i].to(torch.int32)
    return out_b, out_s, out_l
