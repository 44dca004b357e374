"""Tensor collectives with Horovod semantics over torch.distributed (RCCL / gloo).

Reference call sites: ``hvd.DistributedOptimizer`` all-reduce-average per gradient
(``/root/reference/train.py:103-104``) and ``BroadcastGlobalVariablesCallback(0)``
(``train.py:111``) -- SURVEY §2.7 C2/C3.  Semantics kept:

(a) ``average=True`` returns ``sum / size``;
(b) every rank issues collectives in the same order (callers use a fixed bucket order, and
    ``MXR_CHECK_SIGNATURES=1`` verifies it);
(c) broadcast covers every tensor handed in;
(d) shape/dtype mismatches raise instead of hanging (signature check, and ``allgather``
    negotiates first dimensions explicitly).
"""
from __future__ import annotations

import hashlib
import os
import pickle
from typing import Any, List, Optional, Sequence

import torch
import torch.distributed as dist

from . import runtime
from . import timeline as _timeline


class Compressor:
    dtype: Optional[torch.dtype] = None

    @classmethod
    def compress(cls, t: torch.Tensor):
        if cls.dtype is not None and t.is_floating_point() and t.dtype != cls.dtype:
            return t.to(cls.dtype), t.dtype
        return t, None

    @staticmethod
    def decompress(t: torch.Tensor, ctx):
        return t if ctx is None else t.to(ctx)


class NoneCompressor(Compressor):
    dtype = None


class FP16Compressor(Compressor):
    dtype = torch.float16


class BF16Compressor(Compressor):
    dtype = torch.bfloat16


class Compression:
    """``hvd.Compression.{none, fp16, bf16}``."""
    none = NoneCompressor
    fp16 = FP16Compressor
    bf16 = BF16Compressor


class SignatureMismatch(RuntimeError):
    pass


_CHECK = os.environ.get("MXR_CHECK_SIGNATURES", "0") == "1"


def set_signature_check(enabled: bool) -> None:
    global _CHECK
    _CHECK = bool(enabled)


def check_signature(kind: str, name: Optional[str], t: torch.Tensor) -> None:
    """All-gather a hash of (kind, name, shape, dtype); raise on divergence across ranks."""
    if not runtime.distributed():
        return
    sig = "{}|{}|{}|{}".format(kind, name, tuple(t.shape), t.dtype)
    h = int(hashlib.sha1(sig.encode()).hexdigest()[:12], 16)
    dev = t.device if runtime.backend() == "nccl" else torch.device("cpu")
    mine = torch.tensor([h], dtype=torch.int64, device=dev)
    allh = [torch.zeros_like(mine) for _ in range(runtime.size())]
    dist.all_gather(allh, mine)
    vals = [int(x.item()) for x in allh]
    if len(set(vals)) != 1:
        raise SignatureMismatch("collective mismatch across ranks for {} '{}' (rank {} has {}): hashes {}".format(
            kind, name, runtime.rank(), sig, vals))


_HIER = os.environ.get("HOROVOD_HIERARCHICAL_ALLREDUCE", "0") == "1"
_GROUPS = None


def set_hierarchical(enabled: bool) -> None:
    """Two-level all-reduce (Horovod's ``HOROVOD_HIERARCHICAL_ALLREDUCE``)."""
    global _HIER
    _HIER = bool(enabled)


def _hier_groups():
    """(local group, cross group) of this rank.  ``new_group`` is collective, so every rank
    creates every node group and every cross group in the same order."""
    global _GROUPS
    if _GROUPS is None:
        ls, n = runtime.local_size(), runtime.size()
        mine_l = mine_c = None
        for node in range((n + ls - 1) // ls):
            g = dist.new_group(list(range(node * ls, min(n, (node + 1) * ls))))
            if node == runtime.cross_rank():
                mine_l = g
        for j in range(ls):
            g = dist.new_group(list(range(j, n, ls)))
            if j == runtime.local_rank():
                mine_c = g
        _GROUPS = (mine_l, mine_c)
    return _GROUPS


def _hier_allreduce_(t: torch.Tensor) -> None:
    """Sum over the world in two levels.  With RCCL: reduce-scatter inside the node (xGMI), all-reduce
    of the 1/local_size shard across nodes, all-gather inside the node -- the inter-node link only
    carries 1/local_size of the bytes.  gloo (tests) has no reduce-scatter: node all-reduce, then
    cross all-reduce."""
    lg, cg = _hier_groups()
    ls = runtime.local_size()
    if runtime.backend() == "nccl" and t.is_cuda:
        flat = t.reshape(-1)
        n = flat.numel()
        m = (n + ls - 1) // ls
        buf = flat if m * ls == n else torch.cat([flat, flat.new_zeros(m * ls - n)])
        shard = buf.new_empty(m)
        dist.reduce_scatter_tensor(shard, buf, group=lg)
        dist.all_reduce(shard, group=cg)
        dist.all_gather_into_tensor(buf, shard, group=lg)
        if buf.data_ptr() != flat.data_ptr():
            flat.copy_(buf[:n])
    else:
        dist.all_reduce(t, group=lg)
        dist.all_reduce(t, group=cg)


def _use_hier() -> bool:
    return (_HIER and runtime.distributed() and 1 < runtime.local_size() < runtime.size()
            and runtime.size() % runtime.local_size() == 0)


class Handle:
    def __init__(self, work, tensor, ctx, average, out, name):
        self.work, self.tensor, self.ctx, self.average, self.out, self.name = work, tensor, ctx, average, out, name


def _avg_div(t: torch.Tensor) -> torch.Tensor:
    if t.is_floating_point():
        return t.div_(runtime.size())
    return t.floor_divide_(runtime.size())


def allreduce_async_(tensor: torch.Tensor, average: bool = True, name: Optional[str] = None,
                     compression=Compression.none) -> Handle:
    """In-place asynchronous all-reduce; call :func:`synchronize` on the handle."""
    if _CHECK:
        check_signature("allreduce", name, tensor)
    comp, ctx = compression.compress(tensor)
    tl = _timeline.get()
    if tl.enabled:
        tl.begin(name or "allreduce", "ALLREDUCE", {"bytes": comp.numel() * comp.element_size()})
    work = None
    if _use_hier():
        _hier_allreduce_(comp)             # stream-ordered on RCCL; completes before returning on gloo
    elif runtime.distributed():
        work = dist.all_reduce(comp, op=dist.ReduceOp.SUM, async_op=True)
    return Handle(work, comp, ctx, average, tensor, name)


def synchronize(h: Handle) -> torch.Tensor:
    if h.work is not None:
        h.work.wait()
    res = h.tensor
    if h.average and runtime.size() > 1:
        _avg_div(res)
    if h.ctx is not None:
        h.out.copy_(res)
    elif res.data_ptr() != h.out.data_ptr():
        h.out.copy_(res)
    tl = _timeline.get()
    if tl.enabled:
        tl.end(h.name or "allreduce", "ALLREDUCE")
    return h.out


def poll(h: Handle) -> bool:
    return h.work is None or h.work.is_completed()


def allreduce_(tensor: torch.Tensor, average: bool = True, name: Optional[str] = None,
               compression=Compression.none) -> torch.Tensor:
    return synchronize(allreduce_async_(tensor, average, name, compression))


def allreduce(tensor: torch.Tensor, average: bool = True, name: Optional[str] = None,
              compression=Compression.none) -> torch.Tensor:
    return allreduce_(tensor.clone(), average, name, compression)


def allreduce_async(tensor: torch.Tensor, average: bool = True, name: Optional[str] = None,
                    compression=Compression.none) -> Handle:
    return allreduce_async_(tensor.clone(), average, name, compression)


def allgather(tensor: torch.Tensor, name: Optional[str] = None) -> torch.Tensor:
    """Concatenate along dim 0; first dimensions may differ between ranks (Horovod semantics)."""
    if not runtime.distributed():
        return tensor.clone()
    if _CHECK:
        check_signature("allgather", name, tensor[:0] if tensor.dim() else tensor)
    dev = tensor.device
    n = torch.tensor([tensor.shape[0] if tensor.dim() else 1], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(runtime.size())]
    dist.all_gather(ns, n)
    ns = [int(x.item()) for x in ns]
    t = tensor if tensor.dim() else tensor.reshape(1)
    mx = max(ns)
    if t.shape[0] < mx:
        pad = torch.zeros((mx - t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
        t = torch.cat([t, pad], 0)
    outs = [torch.empty_like(t) for _ in range(runtime.size())]
    dist.all_gather(outs, t.contiguous())
    return torch.cat([o[:k] for o, k in zip(outs, ns)], 0)


def broadcast_(tensor: torch.Tensor, root_rank: int = 0, name: Optional[str] = None) -> torch.Tensor:
    if runtime.distributed():
        if _CHECK:
            check_signature("broadcast", name, tensor)
        dist.broadcast(tensor, src=root_rank)
    return tensor


def broadcast(tensor: torch.Tensor, root_rank: int = 0, name: Optional[str] = None) -> torch.Tensor:
    return broadcast_(tensor.clone(), root_rank, name)


def broadcast_object(obj: Any, root_rank: int = 0) -> Any:
    if not runtime.distributed():
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=root_rank,
                               device=runtime.device() if runtime.backend() == "nccl" else None)
    return lst[0]


def allgather_object(obj: Any) -> list:
    """Every rank's ``obj``, in rank order (pickled through the default process group)."""
    if not runtime.distributed():
        return [obj]
    out = [None] * runtime.size()
    dist.all_gather_object(out, obj)
    return out


def _coalesced_broadcast(tensors: Sequence[torch.Tensor], root_rank: int) -> None:
    """One flat broadcast per dtype (instead of one per tensor)."""
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    for (dt, dev), ts in by_dtype.items():
        flat = torch.cat([t.reshape(-1) for t in ts])
        broadcast_(flat, root_rank, name="bcast_{}".format(dt))
        off = 0
        for t in ts:
            n = t.numel()
            t.copy_(flat[off:off + n].view_as(t))
            off += n


def broadcast_parameters(params, root_rank: int = 0) -> None:
    """``hvd.broadcast_parameters``: params = model.state_dict() / named_parameters / list."""
    if not runtime.distributed():
        return
    if isinstance(params, dict):
        items = sorted(params.items(), key=lambda kv: kv[0])
        tensors = [v for _, v in items]
    else:
        tensors = [p for p in params]
        tensors = [t[1] if isinstance(t, tuple) else t for t in tensors]
    with torch.no_grad():
        _coalesced_broadcast([t.data if hasattr(t, "data") else t for t in tensors], root_rank)


def broadcast_optimizer_state(optimizer, root_rank: int = 0) -> None:
    """Broadcast optimizer slots (Adam m, v) and the iteration counter."""
    if not runtime.distributed():
        return
    with torch.no_grad():
        _coalesced_broadcast(list(optimizer.state_tensors().values()), root_rank)
    it = broadcast_object(getattr(optimizer, "iterations", 0), root_rank)
    optimizer.iterations = it
    lr = broadcast_object(getattr(optimizer, "lr", None), root_rank)
    if lr is not None:
        optimizer.lr = lr


def replica_fingerprint(tensors: Sequence[torch.Tensor]) -> torch.Tensor:
    """Per tensor: (sum, sum |x|, index-weighted sum of a strided sample) in float64 -- equal on every
    rank iff the replicas hold the same values (up to coincidences these three sums cannot see)."""
    rows = []
    for t in tensors:
        x = t.detach().reshape(-1).double()
        s = x[::997]
        w = torch.arange(1, s.numel() + 1, dtype=torch.float64, device=x.device)
        rows.append(torch.stack([x.sum(), x.abs().sum(), (s * w).sum()]))
    return torch.stack(rows).reshape(-1)


def replicas_consistent(tensors: Sequence[torch.Tensor]):
    """Data-parallel replicas must stay bit-identical: every rank applies the same all-reduced gradient
    with the same deterministic optimizer.  All-gathers :func:`replica_fingerprint` and returns
    ``(consistent, ranks_that_differ_from_rank_0)`` on every rank (a collective)."""
    fp = replica_fingerprint(tensors)
    if not runtime.distributed():
        return True, []
    dev = runtime.device() if runtime.backend() == "nccl" else torch.device("cpu")
    fp = fp.to(dev)
    out = [torch.empty_like(fp) for _ in range(runtime.size())]
    dist.all_gather(out, fp)
    bad = [r for r in range(1, len(out)) if not torch.equal(out[r], out[0])]
    return not bad, bad
