"""Bucket sizing for ring all-reduce over the MI355X xGMI mesh.

Reference: Horovod fuses the 89 gradient tensors (151.7 MB fp32 for R50) into <= 64 MiB buffers
(``HOROVOD_FUSION_THRESHOLD``) before each all-reduce (``/root/reference/train.py:103-104``).

On one 8x MI355X node every GPU has 7 point-to-point xGMI links (~153 GB/s per direction each), a
fully connected mesh.  A ring uses ONE outgoing link per GPU, so ring all-reduce is per-link bound;
RCCL runs several channels (rings over different link permutations -- the complete digraph on 8
nodes splits into 7 arc-disjoint Hamiltonian cycles) to keep all 7 links busy.  A bucket of S bytes
reduced over N ranks and C channels moves S / (C N) bytes per channel per ring step; when that slice
is shorter than the protocol's pipeline chunk, the channel runs partly idle (per-step latency, not
bandwidth).  So the bucket floor for full link use is ``C * N * chunk``, and the model below prices a
bucket as latency + bytes / bus bandwidth with that under-fill penalty.

At world 8, 151.7 MB of fp32 gradients is ~0.5 ms of wire time on 7 links against a ~34 ms compute
step: the all-reduce is not the bottleneck, the exposed TAIL is (the last bucket is reduced after
the backward pass ends).  Hence the defaults: 25 MiB buckets (6 for R50: each spans >= 7 channels x
8 ranks x 256 KiB, so every link stays busy) and a small last bucket; ``--bucket-mb`` /
``HOROVOD_FUSION_THRESHOLD`` override it.  ``bench.py`` reports the model's estimate next to the
measured ``comm_ms`` / ``comm_exposed_ms``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Sequence

XGMI_LINKS = 7               # point-to-point links per GPU in an 8-GPU node
XGMI_LINK_GBS = 153.0        # GB/s per link per direction
RING_EFFICIENCY = 0.7        # achieved / wire bus bandwidth of RCCL rings (protocol + sync overheads)
LATENCY_US = 25.0            # per-collective launch + ring-startup latency, N = 8
CHUNK_BYTES = 256 * 1024     # pipeline chunk a channel needs per ring step to stay bandwidth-bound


@dataclass
class BucketEstimate:
    bytes: int
    slice_bytes: float       # bytes per channel per ring step
    fill: float              # min(1, slice / chunk): the fraction of a channel's bandwidth in use
    us: float                # modelled all-reduce time


def min_bucket_bytes(world: int, channels: int = XGMI_LINKS, chunk: int = CHUNK_BYTES) -> int:
    """Smallest bucket whose per-channel ring slice fills one pipeline chunk: channels x world x chunk."""
    return int(channels * max(world, 1) * chunk)


def estimate(bucket_bytes: int, world: int, channels: int = XGMI_LINKS, link_gbs: float = XGMI_LINK_GBS,
             efficiency: float = RING_EFFICIENCY, latency_us: float = LATENCY_US,
             chunk: int = CHUNK_BYTES) -> BucketEstimate:
    """Ring all-reduce time of one bucket: each rank sends 2 (N-1) / N of the bucket, spread over
    ``channels`` links (one ring each) at ``efficiency`` x link bandwidth, channels under-filled when
    the per-step slice is shorter than ``chunk``."""
    if world <= 1:
        return BucketEstimate(int(bucket_bytes), float(bucket_bytes), 1.0, 0.0)
    links = min(channels, XGMI_LINKS)
    slice_bytes = bucket_bytes / float(channels * world)
    fill = min(1.0, slice_bytes / chunk)
    bus = links * link_gbs * 1e9 * efficiency * fill
    wire = 2.0 * (world - 1) / world * bucket_bytes
    return BucketEstimate(int(bucket_bytes), slice_bytes, fill, latency_us + wire / bus * 1e6)


def plan(bucket_sizes: Sequence[int], world: int, **kw) -> Dict[str, object]:
    """Model of a step's bucket list (backward order): total all-reduce time, and the exposed tail (the
    last bucket, reduced after the backward pass)."""
    est: List[BucketEstimate] = [estimate(int(b), world, **kw) for b in bucket_sizes]
    return {"world": world, "total_us": round(sum(e.us for e in est), 1),
            "tail_us": round(est[-1].us, 1) if est else 0.0,
            "min_fill": round(min((e.fill for e in est), default=1.0), 3),
            "floor_mb": round(min_bucket_bytes(world, kw.get("channels", XGMI_LINKS),
                                               kw.get("chunk", CHUNK_BYTES)) / 2 ** 20, 2)}
