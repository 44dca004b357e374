"""One training step: targets -> forward -> focal + smooth-L1 -> backward -> reduce/clip/Adam.

This is CS3 of the survey (the hot loop of ``fit_generator`` driven from
``/root/reference/train.py:444-450``), re-planned for one MI355X per process:

* batches arrive as device tensors: images (B, H, W, 3) and padded gt boxes (B, G, 5);
  anchor targets are computed ON the device (fused HIP kernel), so only kilobytes of boxes
  cross PCIe instead of the reference's 65 MB/image one-hot labels;
* the forward runs NHWC in the compute dtype (bf16 on MI355X) against fp32 master weights;
* losses are fused sigmoid-focal / smooth-L1 kernels that also emit the logit gradients;
* gradients land in the flat fp32 buffer, get all-reduced in buckets (overlapped with the
  backward when ``clip_mode='global'``), and one fused kernel does clip + Adam.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch

from ..ops import anchors as anchor_ops
from ..ops import losses
from ..parallel import runtime
from ..parallel.distributed_optimizer import DistributedOptimizer
from .flat import FlatParams, backward_order
from .optimizer import KerasAdam


_ROCTX = os.environ.get("MXR_ROCTX", "0") == "1"


class _range:
    """roctx range (``MXR_ROCTX=1``; visible in rocprofv3 --marker-trace / sys-trace)."""

    def __init__(self, name: str):
        self.name = name

    def __enter__(self):
        if _ROCTX and torch.cuda.is_available():
            torch.cuda.nvtx.range_push(self.name)
        return self

    def __exit__(self, *a):
        if _ROCTX and torch.cuda.is_available():
            torch.cuda.nvtx.range_pop()


# MXR_PAD_FOCAL=0: hand autograd plain (B, A, C) classification / regression gradients (the final layers pad them)
_PAD_FOCAL = os.environ.get("MXR_PAD_FOCAL", "1") == "1"

class Trainer:
    def __init__(self, model, lr: float = 1e-5, clipnorm: float = 0.001, compute_dtype: torch.dtype = torch.float32,
                 clip_mode: str = "local", compression=None, bucket_bytes: Optional[int] = None,
                 device: Optional[torch.device] = None, overlap: bool = True, target_backend: str = "auto"):
        from ..parallel.collectives import Compression
        self.device = device or (runtime.device() if runtime.is_initialized() else torch.device("cpu"))
        self.model = model.to(self.device)
        self.compute_dtype = compute_dtype
        self.flat = FlatParams(backward_order(self.model), device=self.device)
        self.base_optimizer = KerasAdam(self.flat, lr=lr, clipnorm=clipnorm)
        self.optimizer = DistributedOptimizer(self.base_optimizer, compression=compression or Compression.none,
                                              clip_mode=clip_mode, bucket_bytes=bucket_bytes, overlap=overlap)
        self.anchors = anchor_ops.AnchorCache()
        self.num_classes = model.num_classes
        self.target_backend = target_backend
        self.stop_training = False
        self.shapes_callback = None
        self.last_logs: Dict[str, torch.Tensor] = {}
        self.compute_weights = None
        self._cls_pad_buf = None
        self._focal_req = None      # ops.conv_launch.FocalRequest: the classification final's fused focal loss
        self._reg_pad_buf = None
        from ..ops import native
        from ..ops import fp8 as _fp8
        _fp8.reset_state()      # process-wide fp8 delayed-scaling state (the packed features) starts per model
        if (self.device.type == "cuda" and compute_dtype == torch.bfloat16 and native.available()
                and hasattr(self.model, "convs") and os.environ.get("MXR_NO_COMPUTE_WEIGHTS") != "1"):
            # bf16 W*s compute copies maintained by the fused Adam kernel (no per-layer fold/cast)
            self.compute_weights = native.ComputeWeights(self.flat, self.model.convs())
            native.set_compute_weights(self.compute_weights)
        if self.device.type == "cuda" and native.available() and os.environ.get("MXR_NO_GRAD_SINKS") != "1":
            # conv weight/bias gradients accumulate straight into flat.grad (no autograd adds)
            native.set_grad_sinks(native.GradSinks(self.flat, self.optimizer.notify_grad_ready))

    # ---------------------------------------------------------------- targets
    def compute_targets(self, images: torch.Tensor, gt: torch.Tensor, gt_count: torch.Tensor, image_hw: torch.Tensor):
        H, W = int(images.shape[1]), int(images.shape[2])
        anchors = self.anchors.get((H, W), self.device, self.shapes_callback)
        centers = self.anchors.centers((H, W), self.device, self.shapes_callback)
        from ..ops import native
        use_hip = (self.target_backend == "hip" or
                   (self.target_backend == "auto" and anchors.is_cuda and native.available()))
        if use_hip:
            return native.anchor_targets(anchors, gt, gt_count, image_hw, centers=centers)
        state, label, reg = anchor_ops.anchor_targets_torch(anchors, gt, gt_count, image_hw, centers=centers)
        return state, label, reg, (state == 1).sum().to(torch.int32).reshape(1)

    # ---------------------------------------------------------------- step
    def _fused_losses(self) -> bool:
        from ..ops import native
        return self.device.type == "cuda" and native.available()

    def forward_backward(self, images, gt, gt_count, image_hw):
        """Targets + forward + losses + backward.  Returns (reg_loss, cls_loss) device scalars."""
        with _range("targets"):
            state, label, reg_t, npos = self.compute_targets(images, gt, gt_count, image_hw)
        x = images.to(self.compute_dtype)
        req = self._focal_request(state, label, npos)
        with _range("forward"):
            try:
                out = self.model(x)
            finally:
                if req is not None:
                    self.model.focal_request = None
        with _range("backward"):
            return self._losses_backward(out, reg_t, state, label, npos)

    def _focal_request(self, state, label, npos):
        """This step's targets for the classification final's fused focal loss (bf16 HIP heads with the padded
        focal gradient), handed to the model for its forward; None where the fusion does not apply."""
        if not (self._fused_losses() and _PAD_FOCAL and self.compute_dtype == torch.bfloat16
                and hasattr(self.model, "cls_pad_sink")):
            return None
        from ..ops.conv_launch import FocalRequest
        if self._focal_req is None:
            self._focal_req = FocalRequest()
        A = self.model.num_anchors if hasattr(self.model, "num_anchors") else 9
        self._focal_req.set(state, label, npos, A)
        self.model.focal_request = self._focal_req
        return self._focal_req

    def _losses_backward(self, out, reg_t, state, label, npos):
        if self._fused_losses():
            # fused loss kernels emit d(loss)/d(outputs) directly; backprop from the outputs
            from ..ops import native
            reg = out["regression"]
            A = self.model.num_anchors if hasattr(self.model, "num_anchors") else 9
            rsink = getattr(self.model, "reg_pad_sink", None)
            if rsink is not None and _PAD_FOCAL and reg.dtype == torch.bfloat16 and reg.shape[1] % A == 0 and \
                    (4 * A) % 64:
                # smooth-L1 writes d(loss)/d(regression) into the final layer's 64-padded rows (36 -> 64);
                # the layer's data / weight / bias gradients then read them as is (no pad, cast or slice)
                key = (reg.shape[0], reg.shape[1] // A, (4 * A + 63) // 64 * 64, reg.device)
                buf = self._reg_pad_buf
                if buf is None or buf[0] != key:
                    buf = (key, torch.zeros(key[:3], dtype=reg.dtype, device=reg.device))
                    self._reg_pad_buf = buf
                reg_loss, dpad = native.smooth_l1_fwd_bwd(reg, reg_t, state, npos, grad_out=buf[1], group=A)
                rsink["dy"] = dpad
                dreg = torch.zeros((), dtype=reg.dtype, device=reg.device).expand(reg.shape)
            else:
                reg_loss, dreg = native.smooth_l1_fwd_bwd(reg, reg_t, state, npos)
            cls = out["classification"]
            sink = getattr(self.model, "cls_pad_sink", None)
            cp = (A * cls.shape[-1] + 63) // 64 * 64
            req = self._focal_req
            if req is not None and req.loss is not None:
                # the final layer's forward fused the focal loss: its loss and the padded gradient rows (in the
                # pad sink) are already there; the logits were never written
                cls_loss = req.loss
                req.loss = None
                dcls = torch.zeros((), dtype=cls.dtype, device=cls.device).expand(cls.shape)
            elif sink is not None and _PAD_FOCAL and cls.dtype == torch.bfloat16 and cls.shape[1] % A == 0 and \
                    cls.shape[-1] % 8 == 0 and (A * cls.shape[-1]) % 64:
                # the focal kernel writes d(loss)/d(logits) straight into the final layer's zero-padded
                # data-gradient rows; autograd carries a zero-stride placeholder
                key = (cls.shape[0], cls.shape[1] // A, cp, cls.device)
                buf = self._cls_pad_buf
                if buf is None or buf[0] != key:
                    buf = (key, torch.zeros(key[:3], dtype=cls.dtype, device=cls.device))
                    self._cls_pad_buf = buf
                cls_loss, dpad = native.focal_fwd_bwd(cls, state, label, npos, grad_out=buf[1], group=A)
                sink["dy"] = dpad
                dcls = torch.zeros((), dtype=cls.dtype, device=cls.device).expand(cls.shape)
            else:
                cls_loss, dcls = native.focal_fwd_bwd(cls, state, label, npos)
            torch.autograd.backward([reg, cls], [dreg, dcls])
        else:
            reg_loss = losses.smooth_l1_loss(out["regression"], reg_t, state, backend="torch")
            cls_loss = losses.focal_loss(out["classification"], state, label, backend="torch")
            (reg_loss + cls_loss).backward()
        return reg_loss.detach(), cls_loss.detach()

    def forward_losses(self, images, gt, gt_count, image_hw):
        """Loss values only (no backward) -- used by evaluation/tests."""
        with torch.no_grad():
            state, label, reg_t, npos = self.compute_targets(images, gt, gt_count, image_hw)
            out = self.model(images.to(self.compute_dtype))
            reg_loss = losses.smooth_l1_loss(out["regression"], reg_t, state, backend="torch")
            cls_loss = losses.focal_loss(out["classification"], state, label, backend="torch")
        return reg_loss, cls_loss

    def train_on_batch(self, images: torch.Tensor, gt: torch.Tensor, gt_count: torch.Tensor,
                       image_hw: torch.Tensor) -> Dict[str, torch.Tensor]:
        """Returns device scalars {loss, regression_loss, classification_loss} (no host sync)."""
        if not self.model.training:
            # (Module.train() walks all ~150 modules: ~0.9 ms of host time, which sat in front of the
            # step's first kernels every step when called unconditionally)
            self.model.train()
        return self._train_on_batch(images, gt, gt_count, image_hw)

    def _train_on_batch(self, images, gt, gt_count, image_hw):
        self.optimizer.zero_grad()
        images = images.to(self.device, non_blocking=True)
        gt = gt.to(self.device, non_blocking=True)
        gt_count = gt_count.to(self.device, non_blocking=True)
        image_hw = image_hw.to(self.device, non_blocking=True)
        reg_loss, cls_loss = self.forward_backward(images, gt, gt_count, image_hw)
        loss = reg_loss + cls_loss
        with _range("optimizer"):
            self.optimizer.step()
        logs = {"loss": loss, "regression_loss": reg_loss, "classification_loss": cls_loss}
        self.last_logs = logs
        return logs

    def graph_step(self, images, gt, gt_count, image_hw, warmup: int = 2):
        """Capture ONE whole training step (targets, forward, losses, backward, clip, Adam, compute-
        weight refresh) in a HIP graph; returns ``replay(images, gt, gt_count, image_hw) -> logs``.

        Inputs are copied into static device buffers (same shapes as the example batch).  Every
        kernel of the step is launched by a single graph launch -- no per-kernel CPU dispatch.

        Multi-rank runs capture the native RCCL bucket engine's work too (``parallel.native_comm``): each
        bucket's readiness event, the in-order ``ncclAllReduce`` on the comm stream and the optimizer's waits on
        the done events become graph nodes, so a replay issues the all-reduces exactly where the eager step
        does, overlapped with the backward.  Every rank captures the same collective sequence and replays it in
        lockstep.  (The torch.distributed engine is not captured: gloo runs on the host.)  One graph per batch
        shape: a caller with several padded shape classes keeps one replay per class.  Not with fp8 (its
        delayed-scaling state advances on the host every step).
        """
        from ..ops import fp8 as _fp8
        if runtime.distributed() and self.optimizer.native is None:
            raise RuntimeError("graph_step across ranks needs the native RCCL bucket engine (MXR_COMM=auto/native); "
                               "the torch.distributed path runs eagerly")
        if _fp8.enabled():
            raise RuntimeError("graph_step: the fp8 delayed-scaling state advances on the host each step")
        dev = self.device
        static = {"images": images.to(dev).clone(), "gt": gt.to(dev).clone(), "gt_count": gt_count.to(dev).clone(),
                  "image_hw": image_hw.to(dev).clone()}
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self.train_on_batch(**static)
        torch.cuda.current_stream(dev).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        # thread-local capture: the comm engine's watchdog thread may still poll an earlier step's events
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            logs = self.train_on_batch(**static)
        from ..ops import native
        plan = native.adam_plan(self.flat) if native.available() else None

        def replay(images, gt, gt_count, image_hw):
            for k, v in (("images", images), ("gt", gt), ("gt_count", gt_count), ("image_hw", image_hw)):
                if v.data_ptr() != static[k].data_ptr():
                    static[k].copy_(v, non_blocking=True)
            graph.replay()
            # the captured Adam advances the device step counter; keep the host mirrors in sync
            self.base_optimizer.iterations += 1
            if plan is not None:
                plan.host_iter += 1
            return logs

        # capturing RECORDS the step without executing it, but the host-side counters advanced
        # while the Python ran -> undo that advance
        self.base_optimizer.iterations -= 1
        if plan is not None:
            plan.host_iter -= 1
        self._graph = graph
        return replay

    # ---------------------------------------------------------------- keras-ish
    @property
    def lr(self) -> float:
        return self.base_optimizer.lr

    @lr.setter
    def lr(self, v: float) -> None:
        self.base_optimizer.lr = float(v)

    def state_for_broadcast(self):
        return [self.flat.data] + [b for b in self.model.buffers()]

    def on_weights_changed(self) -> None:
        """Call after weights/optimizer state were replaced (broadcast, checkpoint restore)."""
        self.flat.rebind()
        if self.compute_weights is not None:
            self.compute_weights.build()     # BN scales may have changed too
