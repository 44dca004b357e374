"""Data-dependent initialisation of the frozen BatchNorm statistics.

The reference always starts from ImageNet weights (``--imagenet-weights`` is its default,
``/root/reference/train.py:358-362,412-413``), whose frozen BN moving statistics keep every
backbone activation near unit scale.  Offline, a ``--no-weights`` start has identity BN
(mean 0, var 1): the Caffe-style ResNet then grows its activations ~10x per stage (C5 std
~7e4 at 800x1333) and the heads emit logits in the hundreds, so the focal loss starts at ~1e5.

``calibrate_frozen_bn`` stands in for the pretrained statistics: one forward pass over a batch
sets each frozen BN's ``moving_mean`` / ``moving_variance`` to the per-channel statistics of
its own conv output (gamma 1, beta 0), layer by layer in execution order, so each BN sees the
already-calibrated layers in front of it.  BN stays frozen afterwards (the training semantics of
SURVEY §2.8.1 are unchanged) and, because BN folds into the conv epilogues, it costs nothing at
run time.  The pass runs on the PyTorch conv backend in fp32.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..ops import conv as conv_ops


@torch.no_grad()
def calibrate_frozen_bn(model: torch.nn.Module, images: torch.Tensor, eps_floor: float = 1e-6) -> int:
    """Set frozen-BN statistics of ``model`` from ``images`` (NHWC); returns #BN layers set."""
    prev_backend = conv_ops.get_conv_backend()
    count = [0]

    def on_conv(layer, raw: torch.Tensor) -> None:
        bn = layer.bn
        flat = raw.float().reshape(-1, raw.shape[-1])
        mean = flat.mean(0)
        var = flat.var(0, unbiased=False).clamp_min(eps_floor)
        bn.gamma.fill_(1.0)
        bn.beta.zero_()
        bn.moving_mean.copy_(mean)
        bn.moving_variance.copy_(var)
        count[0] += 1

    was_training = model.training
    conv_ops.set_conv_backend("torch")
    conv_ops.set_calibration_hook(on_conv)
    try:
        model.eval()
        model(images.float())
    finally:
        conv_ops.set_calibration_hook(None)
        conv_ops.set_conv_backend(prev_backend)
        model.train(was_training)
    return count[0]


def calibrate_from_synthetic(model: torch.nn.Module, device: torch.device, batch: int = 2,
                             height: int = 512, width: int = 640, seed: Optional[int] = 0) -> int:
    """Calibrate on a synthetic COCO-shaped batch (used by bench.py / ``train.py --calibrate-bn``)."""
    from ..data.synthetic import make_batch
    if seed is not None:
        torch.manual_seed(seed)
    b = make_batch(batch, height, width, device=device)
    return calibrate_frozen_bn(model, b["images"])
