"""Synthetic COCO-shaped batches generated directly on the device.

Used by ``bench.py`` and by the ``synthetic`` dataset subcommand of the CLI (BASELINE.json
configs: "synthetic data / random-init weights").  Images are caffe-preprocessed-looking
float tensors (B, H, W, 3) (BGR mean already subtracted, values roughly in [-124, 152]);
boxes are random COCO-like rectangles with 1..max_boxes objects per image and labels in
[0, num_classes).  Only the boxes are needed to build anchor targets, which the trainer
computes on the device every step.
"""
from __future__ import annotations

from typing import Dict, Iterator, List, Optional

import torch

CAFFE_MEAN_BGR = (103.939, 116.779, 123.68)


def make_batch(batch_size: int, height: int, width: int, num_classes: int = 80, max_boxes: int = 20,
               device="cpu", generator: Optional[torch.Generator] = None, dtype=torch.float32) -> Dict[str, torch.Tensor]:
    g = generator
    dev = torch.device(device)
    img = torch.rand((batch_size, height, width, 3), generator=g, device=dev) * 255.0
    mean = torch.tensor(CAFFE_MEAN_BGR, device=dev)
    img = (img - mean).to(dtype)
    counts = torch.randint(1, max_boxes + 1, (batch_size,), generator=g, device=dev)
    G = max_boxes
    # box sizes log-uniform between 16 px and 60 % of the short side
    short = float(min(height, width))
    lo, hi = torch.log(torch.tensor(16.0)), torch.log(torch.tensor(0.6 * short))
    wh = torch.exp(lo + (hi - lo) * torch.rand((batch_size, G, 2), generator=g, device=dev))
    ar = torch.exp((torch.rand((batch_size, G, 1), generator=g, device=dev) - 0.5) * 1.4)
    w = (wh[..., 0:1] * ar).clamp(max=width - 2)
    h = (wh[..., 1:2] / ar).clamp(max=height - 2)
    x1 = torch.rand((batch_size, G, 1), generator=g, device=dev) * (width - 1 - w)
    y1 = torch.rand((batch_size, G, 1), generator=g, device=dev) * (height - 1 - h)
    lab = torch.randint(0, num_classes, (batch_size, G, 1), generator=g, device=dev).float()
    gt = torch.cat([x1, y1, x1 + w, y1 + h, lab], dim=-1)
    valid = torch.arange(G, device=dev)[None, :] < counts[:, None]
    gt = torch.where(valid[..., None], gt, torch.full_like(gt, -1.0))
    image_hw = torch.tensor([[height, width]] * batch_size, dtype=torch.int32, device=dev)
    return {"images": img, "gt": gt.contiguous(), "gt_count": counts.to(torch.int32), "image_hw": image_hw}


class SyntheticBatches:
    """Cycles over a small pool of pre-generated device batches (no host work per step).

    ``dtype``: image dtype of the batches -- the compute dtype, as the device preprocessing
    (data/device_preprocess.py) writes its padded batch directly in it."""

    def __init__(self, batch_size: int, height: int, width: int, num_classes: int = 80, max_boxes: int = 20,
                 pool: int = 4, device="cpu", seed: int = 0, dtype: torch.dtype = torch.float32):
        gen = torch.Generator(device=device)
        gen.manual_seed(seed)
        self.pool: List[Dict[str, torch.Tensor]] = [
            make_batch(batch_size, height, width, num_classes, max_boxes, device, gen, dtype) for _ in range(pool)]
        self.i = 0

    def __iter__(self) -> Iterator[Dict[str, torch.Tensor]]:
        return self

    def __next__(self) -> Dict[str, torch.Tensor]:
        b = self.pool[self.i % len(self.pool)]
        self.i += 1
        return b


# ----------------------------------------------------------------------------------------
# Generator-protocol synthetic dataset (CLI ``synthetic`` subcommand, CPU tests)
# ----------------------------------------------------------------------------------------
import os as _os

import numpy as _np

from .generator import Generator as _Generator


class SyntheticGenerator(_Generator):
    """Deterministic random images + boxes behind the full Generator pipeline (decode-free)."""

    def __init__(self, num_images: int = 2, height: int = 480, width: int = 640, num_classes: int = 80,
                 max_boxes: int = 8, data_seed: int = 0, cache_bytes: Optional[int] = None, **kwargs):
        self._n, self._h, self._w = int(num_images), int(height), int(width)
        if cache_bytes is None:
            # one node's ranks share the host: 4 GiB split over the local ranks (MXR_SYNTH_CACHE_MB overrides)
            env = _os.environ.get("MXR_SYNTH_CACHE_MB")
            local = int(_os.environ.get("LOCAL_WORLD_SIZE", _os.environ.get("OMPI_COMM_WORLD_LOCAL_SIZE", "1")) or 1)
            cache_bytes = int(float(env) * 2 ** 20) if env is not None else (4 << 30) // max(1, local)
        self.cache_bytes = int(cache_bytes)     # 0 = no cache
        self._nc, self._mb, self._seed = int(num_classes), int(max_boxes), int(data_seed)
        self.classes = {"class_{}".format(i): i for i in range(self._nc)}
        self.labels = {v: k for k, v in self.classes.items()}
        super().__init__(**kwargs)

    def _rng(self, i):
        return _np.random.RandomState(self._seed * 100003 + i)

    def size(self):
        return self._n

    def num_classes(self):
        return self._nc

    def name_to_label(self, name):
        return self.classes[name]

    def label_to_name(self, label):
        return self.labels[label]

    def image_aspect_ratio(self, image_index):
        return float(self._w) / float(self._h)

    # decoded images are kept up to ``cache_bytes``: drawing an 800x1333 random image holds the GIL for
    # ~6 ms, which capped a threaded host pipeline at ~150 img/s -- a cost of the synthetic source, not of
    # the pipeline (PIL's JPEG decode and the native resize / warp release the GIL).  (Round 2 moved the
    # draw from RandomState.randint to default_rng().integers: the synthetic pixels of every index changed
    # then; no stored loss or fixture depends on them.)

    def load_image(self, image_index):
        cache = self.__dict__.setdefault("_img_cache", {})
        img = cache.get(image_index)
        if img is None:
            img = _np.random.default_rng(self._seed * 100003 + image_index).integers(
                0, 256, (self._h, self._w, 3), dtype=_np.uint8)
            if (len(cache) + 1) * img.nbytes <= self.cache_bytes:
                cache[image_index] = img
        return img

    def __getstate__(self):
        st = super().__getstate__()
        st["_img_cache"] = {}          # a worker process draws (and caches) its own
        return st

    def load_annotations(self, image_index):
        r = self._rng(image_index + 7919)
        n = r.randint(1, self._mb + 1)
        w = r.uniform(16, 0.5 * self._w, n)
        h = r.uniform(16, 0.5 * self._h, n)
        x1 = r.uniform(0, self._w - w - 1)
        y1 = r.uniform(0, self._h - h - 1)
        lab = r.randint(0, self._nc, n)
        return _np.stack([x1, y1, x1 + w, y1 + h, lab], axis=1)
