"""Flat parameter / gradient storage.

Every trainable tensor becomes a view into ONE contiguous fp32 master buffer and its
``.grad`` a view into ONE contiguous fp32 gradient buffer.  The buffers are laid out in
*backward order* (heads -> FPN -> backbone) so that gradient buckets become ready front to
back while the backward pass is still running.  This is the zero-copy replacement for
Horovod's 64 MiB fusion buffer: a bucket is just a slice.

Optionally a bf16 "compute copy" of the weights (with the frozen-BN scale folded in) is kept
in a second flat buffer; the fused Adam kernel refreshes it in the same pass that updates the
master weights, so the forward pass never re-casts weights.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

ALIGN = 64  # elements; keeps every segment 256-B aligned for vectorised kernels


@dataclass
class Segment:
    name: str
    param: nn.Parameter
    offset: int
    numel: int
    shape: Tuple[int, ...]


class FlatParams:
    """Packs ``params`` (given in backward order) into aligned flat buffers."""

    def __init__(self, named_params: Sequence[Tuple[str, nn.Parameter]], device=None):
        self.segments: List[Segment] = []
        off = 0
        for name, p in named_params:
            n = p.numel()
            self.segments.append(Segment(name, p, off, n, tuple(p.shape)))
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        self.total = off
        dev = device if device is not None else (named_params[0][1].device if named_params else "cpu")
        self.data = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=dev)
        for s in self.segments:
            self.data[s.offset:s.offset + s.numel].copy_(s.param.data.reshape(-1).float())
            s.param.data = self.data[s.offset:s.offset + s.numel].view(s.shape)
            s.param.grad = self.grad[s.offset:s.offset + s.numel].view(s.shape)
        self.by_param: Dict[int, Segment] = {id(s.param): s for s in self.segments}

    def params(self) -> List[nn.Parameter]:
        return [s.param for s in self.segments]

    def zero_grad(self) -> None:
        self.grad.zero_()
        # autograd may have replaced .grad (e.g. after set_to_none elsewhere); re-bind views
        for s in self.segments:
            g = s.param.grad
            if g is None or g.data_ptr() != self.grad[s.offset:].data_ptr():
                s.param.grad = self.grad[s.offset:s.offset + s.numel].view(s.shape)

    def rebind(self) -> None:
        """Re-point params at the flat buffer (after an external ``load_state_dict``)."""
        for s in self.segments:
            if s.param.data.data_ptr() != self.data[s.offset:].data_ptr():
                self.data[s.offset:s.offset + s.numel].copy_(s.param.data.reshape(-1))
                s.param.data = self.data[s.offset:s.offset + s.numel].view(s.shape)


def backward_order(model: nn.Module) -> List[Tuple[str, nn.Parameter]]:
    """Trainable parameters in reverse registration order (≈ order gradients become ready)."""
    named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
    return list(reversed(named))
