"""ctypes bindings + autograd wrappers for the in-tree HIP kernel library.

``_lib/libmxr_kernels.so`` is built by :mod:`batchai_retinanet_horovod_coco_amd.build` with
``hipcc --offload-arch=gfx950``.  It is loaded AFTER ``import torch`` so it binds to the HIP
runtime torch already mapped (same soname), and every launch goes onto torch's current HIP
stream (``torch.cuda.current_stream().cuda_stream``) -- so the kernels compose with torch ops,
RCCL collectives and HIP-graph capture.

On a GPU box the library is REQUIRED (``load(required=True)``); a missing or stale build raises
instead of silently falling back to PyTorch.  ``disable()`` switches every op to its PyTorch
reference path for A/B runs (``bench.py --kernels off``).
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
# MXR_KERNEL_LIB: another build of the kernel library (same-box A/B of a kernel change)
LIB_PATH = os.environ.get("MXR_KERNEL_LIB") or os.path.join(_PKG, "_lib", "libmxr_kernels.so")

_LIB: Optional[ctypes.CDLL] = None
_DISABLED = [os.environ.get("MXR_DISABLE_KERNELS", "0") == "1"]
_LOAD_ERR: List[str] = []

c_int, c_ll, c_float, c_vp = ctypes.c_int, ctypes.c_longlong, ctypes.c_float, ctypes.c_void_p

MAXLEV = 5


class ConvGeom(ctypes.Structure):
    _fields_ = [("nlev", c_int), ("H", c_int * MAXLEV), ("W", c_int * MAXLEV), ("Ho", c_int * MAXLEV),
                ("Wo", c_int * MAXLEV), ("in_off", c_int * MAXLEV), ("mstart", c_int * (MAXLEV + 1)),
                ("in_img", c_int), ("out_img", c_int), ("stride", c_int), ("pt", c_int), ("pl", c_int),
                ("kh", c_int), ("kw", c_int), ("cin", c_int), ("cout", c_int), ("M", c_ll),
                ("ostride", c_int), ("oH", c_int), ("oW", c_int), ("ooy", c_int), ("oox", c_int)]


_SIGS = {
    "mxr_focal_fwd_bwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_ll, c_int, c_float, c_float, c_float, c_float,
                          c_int, c_int, c_int, c_vp],
    "mxr_smooth_l1_fwd_bwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_ll, c_float, c_int, c_int, c_int, c_vp],
    "mxr_loss_grid": [],
    "mxr_anchor_targets": [c_vp, c_vp, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_float, c_float,
                           c_float, c_vp],
    "mxr_chunk_struct_sizes": [c_vp],
    "mxr_adam_step": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_float, c_float,
                      c_float, c_vp],
    "mxr_refresh_copy": [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp],
    "mxr_grad_norm_clip": [c_vp, c_ll, c_vp, c_float, c_float, c_float, c_vp, c_vp],
    "mxr_scale_inplace": [c_vp, c_ll, c_vp, c_vp],
    "mxr_norm_grid": [],
    "mxr_maxpool_fwd": [c_vp, c_vp, c_vp] + [c_int] * 11 + [c_int, c_int, c_vp],
    "mxr_wgrad3x3_c64": [c_vp] * 5 + [c_int] * 4 + [c_vp],
    "mxr_wgrad_halo": [c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int,
                       c_vp, c_vp, c_vp, c_int, c_vp],
    "mxr_flip_batch": [c_vp, c_vp, c_vp, c_vp, c_int, c_vp],
    "mxr_conv1x1_stream": [c_vp] * 6 + [c_int] * 12 + [c_vp],
    "mxr_conv1x1_pers_dual": [c_vp] * 9 + [c_ll, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "mxr_conv1x1_pers": [c_vp] * 8 + [c_ll, c_int, c_int, c_int, c_int, c_vp],
    "mxr_conv_wgrad_p8_f8": [c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_int, c_vp,
                             ctypes.POINTER(ConvGeom), c_int, c_vp],
    "mxr_hx8_quant_pack_batch": [c_vp, c_int, c_int, c_vp],
    "mxr_conv_wgrad_p8_f8_bias": [c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_int, c_vp,
                                  ctypes.POINTER(ConvGeom), c_int, c_vp, c_int, c_vp],
    "mxr_stem_fwd": [c_vp, c_vp, c_vp, c_vp] + [c_int] * 8 + [c_vp],
    "mxr_stem_pool_fwd": [c_vp, c_vp, c_vp, c_vp, c_vp] + [c_int] * 11 + [c_vp],
    "mxr_stem_pack": [c_vp, c_vp, c_vp, c_vp],
    "mxr_stem_wgrad": [c_vp, c_vp, c_vp, c_vp, c_vp] + [c_int] * 8 + [c_vp] + [c_int] * 4 + [c_vp],
    "mxr_maxpool_bwd": [c_vp, c_vp, c_vp] + [c_int] * 10 + [c_int, c_vp],
    "mxr_upsample_add_fwd": [c_vp, c_vp, c_vp, c_vp, c_vp] + [c_int] * 6 + [c_int, c_vp],
    "mxr_upsample_bwd": [c_vp, c_vp, c_vp, c_vp] + [c_int] * 6 + [c_int, c_vp],
    "mxr_decode_clip": [c_vp, c_vp, c_int, c_vp, c_int, c_int, c_float, c_float, c_float, c_vp],
    "mxr_nms": [c_vp, c_int, c_float, c_int, c_vp, c_vp, c_vp, c_vp],
    "mxr_filter_select": [c_vp, c_int, c_int, c_int, c_int, c_float, c_vp, c_vp, c_int, c_vp],
    "mxr_filter_nms": [c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_int, c_int, c_int, c_float, c_float,
                       c_float, c_float, c_int, c_vp, c_vp, c_vp, c_vp, c_vp],
    "mxr_conv_geom_size": [],
    "mxr_s2_stack_flip": [c_vp, c_vp, c_int, c_int, c_vp, c_vp],
    "mxr_conv_fwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(ConvGeom), c_int, c_int, c_int, c_vp],
    "mxr_conv_fwd_pipe": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(ConvGeom), c_int, c_int, c_int,
                          c_vp],
    "mxr_conv_fwd_pipe_dual": [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                               ctypes.POINTER(ConvGeom), c_int, c_int, c_vp],
    "mxr_conv_dgrad_pipe_dd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp,
                               ctypes.POINTER(ConvGeom), c_int, c_vp],
    "mxr_conv_fwd_pipe_sk": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(ConvGeom), c_int, c_int, c_int,
                             c_int, c_vp, c_vp],
    "mxr_conv_p8": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(ConvGeom), c_int, c_int, c_int, c_vp],
    "mxr_conv3x3_halo": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(ConvGeom), c_vp, c_int, c_int, c_int,
                         c_int, c_vp],
    "mxr_hx32_pack_weights": [c_vp, c_vp, c_int, c_int, c_vp],
    "mxr_hx32_pack_batch": [c_vp, c_int, c_vp, c_ll, c_vp],
    "mxr_conv3x3_hx32": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(ConvGeom), c_vp, c_int, c_int, c_int,
                         c_int, c_vp],
    "mxr_conv_wgrad_p8": [c_vp, c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_int, c_vp, ctypes.POINTER(ConvGeom), c_int,
                          c_vp],
    "mxr_conv_wgrad_p8_dual": [c_vp, c_vp, c_int, c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp,
                               ctypes.POINTER(ConvGeom), c_int, c_vp],
    "mxr_conv_wgrad_p8_bias": [c_vp, c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_int, c_vp, ctypes.POINTER(ConvGeom),
                               c_int, c_vp, c_int, c_vp],
    "mxr_conv_wgrad_pipe": [c_vp, c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_int, c_vp, ctypes.POINTER(ConvGeom), c_int,
                            c_vp],
    "mxr_flip_transpose": [c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp],
    "mxr_image_warp_normalize": [c_vp, c_int, c_int, c_vp, c_int, c_int, c_vp, c_int, c_int, c_int, c_float, c_float,
                                 c_float, c_float, c_float, c_vp],
    "mxr_image_resize_into": [c_vp, c_int, c_int, c_vp, c_int, c_int, c_ll, c_int, c_vp],
    "mxr_fp8_amax": [c_vp, c_ll, c_vp, c_vp],
    "mxr_fp8_quant": [c_vp, c_ll, c_vp, c_vp, c_vp, c_vp],
    "mxr_fp8_quant_rows": [c_vp, c_int, c_int, c_vp, c_vp, c_vp],
    "mxr_conv_fwd_f8": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(ConvGeom), c_int, c_vp, c_vp,
                        c_vp, c_int, c_float, c_int, c_vp],
    "mxr_conv_p8_f8": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(ConvGeom), c_int, c_int,
                       c_vp, c_vp, c_vp, c_int, c_float, c_int, c_vp],
    "mxr_bf8_quant": [c_vp, c_ll, c_vp, c_vp, c_vp, c_vp],
    "mxr_quant_delayed": [c_vp, c_ll, c_vp, c_vp, c_int, c_float, c_vp, c_int, c_vp],
    "mxr_hx8_pack_weights": [c_vp, c_vp, c_int, c_int, c_vp],
    "mxr_hx8_quant_pack": [c_vp, c_int, c_int, c_vp, c_vp, c_vp],
    "mxr_conv3x3_hx32_f8": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(ConvGeom), c_vp, c_int,
                            c_int, c_int, c_vp, c_vp, c_vp, c_int, c_float, c_int, c_vp],
    "mxr_conv3x3_hx32_focal": [c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(ConvGeom), c_vp, c_int, c_vp, c_vp, c_vp, c_vp,
                               c_int, c_int, c_int, c_float, c_float, c_float, c_float, c_vp, c_int, c_vp, c_vp],
    "mxr_conv3x3_hx32_focal_v": [c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(ConvGeom), c_vp, c_int, c_vp, c_vp, c_vp, c_vp,
                                 c_int, c_int, c_int, c_float, c_float, c_float, c_float, c_vp, c_int, c_vp, c_int,
                                 c_vp],
    "mxr_conv3x3_hx32_f8_focal": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(ConvGeom), c_vp, c_int, c_vp, c_vp,
                                  c_vp, c_vp, c_int, c_int, c_int, c_float, c_float, c_float, c_float, c_vp, c_int, c_vp,
                                  c_vp],
    "mxr_conv3x3_hx32_f8_focal_q": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(ConvGeom), c_vp, c_int, c_vp,
                                    c_vp, c_vp, c_vp, c_int, c_int, c_int, c_float, c_float, c_float, c_float, c_vp,
                                    c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_float, c_vp],
    "mxr_s2_shuffle": [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "mxr_s2_stack": [c_vp, c_vp, c_int, c_int, c_vp, c_vp],
    "mxr_pyr_pack": [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp],
    "mxr_pyr_pack_f8": [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_float, c_vp],
}
_OPTIONAL = {"mxr_conv_wgrad", "mxr_bias_grad", "mxr_relu_bwd"}


def load(required: bool = False, check_device: bool = True) -> bool:
    """Load the kernel library.  ``required`` raises if it is missing/invalid."""
    global _LIB
    if _LIB is not None:
        return True
    if not os.path.exists(LIB_PATH):
        msg = "HIP kernel library not built: {} (run python -m batchai_retinanet_horovod_coco_amd.build)".format(LIB_PATH)
        _LOAD_ERR.append(msg)
        if required:
            raise RuntimeError(msg)
        return False
    try:
        lib = ctypes.CDLL(LIB_PATH)
        for name, args in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = c_int
        if lib.mxr_conv_geom_size() != ctypes.sizeof(ConvGeom):
            raise RuntimeError("ConvGeom layout mismatch ({} vs {})".format(lib.mxr_conv_geom_size(),
                                                                         ctypes.sizeof(ConvGeom)))
    except Exception as e:  # noqa: BLE001
        _LOAD_ERR.append(str(e))
        if required:
            raise
        return False
    _LIB = lib
    return True


def disable() -> None:
    _DISABLED[0] = True


def enable() -> None:
    _DISABLED[0] = False


def available() -> bool:
    if _DISABLED[0] or not torch.cuda.is_available():
        return False
    return load(required=os.environ.get("MXR_REQUIRE_KERNELS", "1") == "1")


def conv_supported() -> bool:
    return available() and os.environ.get("MXR_HIP_CONV", "1") == "1"


def loaded_libraries() -> List[str]:
    return [LIB_PATH] if _LIB is not None else []


def lib() -> ctypes.CDLL:
    if _LIB is None:
        load(required=True)
    return _LIB


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_CUR_DEV = getattr(torch._C, "_cuda_getDevice", None)


def _s() -> int:
    """Raw handle of the current stream (hot: once per launch -- the torch.cuda.current_stream() wrapper
    costs several us of device-index resolution per call)."""
    if _RAW_STREAM is not None:
        return _RAW_STREAM(_CUR_DEV())
    return torch.cuda.current_stream().cuda_stream


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


_SYNC_DEBUG = os.environ.get("MXR_SYNC_DEBUG", "0") == "1"


def _chk(rc: int, name: str) -> None:
    if rc != 0:
        raise RuntimeError("{} failed with code {}".format(name, rc))
    if _SYNC_DEBUG:
        # debug mode: synchronise after every launch so an asynchronous fault is
        # reported at the kernel that caused it, not at a later unrelated sync point
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:
            raise RuntimeError("{} faulted: {}".format(name, e)) from e


def _dt(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return 1
    if t.dtype == torch.float32:
        return 0
    raise TypeError("unsupported dtype {}".format(t.dtype))


_ZERO = {}


def zero_page(device) -> torch.Tensor:
    key = str(device)
    z = _ZERO.get(key)
    if z is None:
        z = torch.zeros(256, dtype=torch.uint8, device=device)
        _ZERO[key] = z
    return z


_TRASH = {}


def trash_page(device) -> torch.Tensor:
    """A writable 256-B scratch line per device: kernels that keep a fixed count of stores per wave (counted
    vmcnt waits) send the stores of chunks outside the tensor there instead of skipping them."""
    key = str(device)
    t = _TRASH.get(key)
    if t is None:
        t = torch.empty(256, dtype=torch.uint8, device=device)
        _TRASH[key] = t
    return t


# =========================================================================================
# losses
# =========================================================================================
LOSS_GRID = 2048


def _npos(state: torch.Tensor, npos: Optional[torch.Tensor]) -> torch.Tensor:
    if npos is None:
        npos = (state == 1).sum().to(torch.int32).reshape(1)
    return npos


def focal_fwd_bwd(logits, state, label, npos=None, alpha=0.25, gamma=2.0, grad_out=None, group=0):
    """Returns (loss 0-d f32, dlogits like logits) -- dlogits already / max(1, npos).

    ``grad_out`` (with ``group`` rows per padded row): write dlogits into this [rows / group, ld] buffer
    instead (the packed head's zero-padded pixel rows, see RetinaNet.forward); it is returned."""
    from .losses import LOGIT_HI, LOGIT_LO
    logits = logits.contiguous()
    C = logits.shape[-1]
    rows = logits.numel() // C
    npos = _npos(state, npos)
    ld = 0
    if grad_out is not None:
        ld = grad_out.shape[-1]
        if not (grad_out.is_contiguous() and grad_out.dtype == logits.dtype and group > 0
                and grad_out.numel() == rows // group * ld):
            raise ValueError("focal_fwd_bwd: grad_out does not match the padded layout")
        grad = grad_out
    else:
        grad = torch.empty_like(logits)
    part = torch.empty(LOSS_GRID, dtype=torch.float32, device=logits.device)
    out = torch.empty(1, dtype=torch.float32, device=logits.device)
    _chk(lib().mxr_focal_fwd_bwd(_p(logits), _p(state.contiguous()), _p(label.contiguous()), _p(npos), _p(grad),
                                 _p(part), _p(out), rows, C, alpha, gamma, LOGIT_LO, LOGIT_HI, _dt(logits),
                                 int(group) if ld else 0, ld, _s()),
         "focal")
    return out.reshape(()), grad

def smooth_l1_fwd_bwd(reg, reg_t, state, npos=None, sigma=3.0, grad_out=None, group=0):
    """Returns (loss 0-d f32, dreg like reg).  ``grad_out`` (with ``group`` anchors per padded row): write
    dreg into this zero-padded [rows / group, ld] buffer instead (the packed regression head's 64-wide
    data-gradient rows; its padding columns are never written) and return it."""
    reg = reg.contiguous()
    rows = reg.numel() // 4
    npos = _npos(state, npos)
    ld = 0
    if grad_out is not None:
        ld = grad_out.shape[-1]
        if not (grad_out.is_contiguous() and grad_out.dtype == reg.dtype and group > 0
                and grad_out.numel() == rows // group * ld):
            raise ValueError("smooth_l1_fwd_bwd: grad_out does not match the padded layout")
        grad = grad_out
    else:
        grad = torch.empty_like(reg)
    part = torch.empty(LOSS_GRID, dtype=torch.float32, device=reg.device)
    out = torch.empty(1, dtype=torch.float32, device=reg.device)
    _chk(lib().mxr_smooth_l1_fwd_bwd(_p(reg), _p(reg_t.float().contiguous()), _p(state.contiguous()), _p(npos),
                                     _p(grad), _p(part), _p(out), rows, sigma, _dt(reg), int(group) if ld else 0,
                                     ld, _s()), "smooth_l1")
    return out.reshape(()), grad


class FocalLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, state, label, alpha, gamma, npos=None):
        loss, grad = focal_fwd_bwd(logits, state, label, npos, alpha, gamma)
        ctx.save_for_backward(grad)
        return loss

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return grad * g.to(grad.dtype), None, None, None, None, None


class SmoothL1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, reg, reg_t, state, sigma, npos=None):
        loss, grad = smooth_l1_fwd_bwd(reg, reg_t, state, npos, sigma)
        ctx.save_for_backward(grad)
        return loss

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return grad * g.to(grad.dtype), None, None, None, None


# =========================================================================================
# anchor targets
# =========================================================================================
def anchor_targets(anchors, gt, gt_count, image_hw, neg=0.4, pos=0.5, std=0.2, centers=None):
    """Returns (state int8 (B,A), label int32 (B,A), regression f32 (B,A,4), npos int32 (1,))."""
    B, G = gt.shape[0], gt.shape[1]
    A = anchors.shape[0]
    dev = anchors.device
    state = torch.empty((B, A), dtype=torch.int8, device=dev)
    label = torch.empty((B, A), dtype=torch.int32, device=dev)
    reg = torch.empty((B, A, 4), dtype=torch.float32, device=dev)
    npos = torch.empty(1, dtype=torch.int32, device=dev)
    gtc = gt.float().contiguous()
    if centers is None:
        from .anchors import centers_round_down
        centers = torch.from_numpy(centers_round_down(anchors.double().cpu().numpy())).to(dev)
    _chk(lib().mxr_anchor_targets(_p(anchors.contiguous()), _p(centers.contiguous()), A, _p(gtc), B, G, _p(gt_count.to(torch.int32).contiguous()),
                                  _p(image_hw.to(torch.int32).contiguous()), _p(state), _p(label), _p(reg), _p(npos),
                                  neg, pos, std, _s()), "anchor_targets")
    return state, label, reg, npos


# =========================================================================================
# optimizer
# =========================================================================================
class AdamPlan:
    """Device-side chunk/segment tables for the fused multi-tensor Keras-Adam kernel."""

    CHUNK = 8192

    def __init__(self, flat, scales: Optional[dict] = None, copy: bool = False):
        import numpy as np
        dev = flat.data.device
        sizes = (c_int * 2)()
        lib().mxr_chunk_struct_sizes(ctypes.addressof(sizes))
        assert sizes[0] == 16 and sizes[1] == 24, tuple(sizes)
        chunks, segs, scale_parts = [], [], []
        soff = 0
        for si, s in enumerate(flat.segments):
            sc = scales.get(id(s.param)) if scales else None
            row_len = max(1, s.numel // s.shape[0]) if len(s.shape) > 0 else 1
            if sc is not None:
                segs.append((s.offset, soff, row_len, 1 if copy else 0))
                scale_parts.append(sc.detach().float().reshape(-1))
                soff += sc.numel()
            else:
                segs.append((s.offset, -1, row_len, 1 if copy else 0))
            st = 0
            while st < s.numel:
                ln = min(self.CHUNK, s.numel - st)
                chunks.append((s.offset + st, ln, si))
                st += ln
        ch = np.zeros(len(chunks), dtype=[("start", "<i8"), ("len", "<i4"), ("seg", "<i4")])
        for i, c in enumerate(chunks):
            ch[i] = c
        sg = np.zeros(len(segs), dtype=[("offset", "<i8"), ("scale_off", "<i8"), ("row_len", "<i4"),
                                        ("has_copy", "<i4")])
        for i, s in enumerate(segs):
            sg[i] = s
        self.chunks = torch.from_numpy(ch.view(np.uint8).copy()).to(dev)
        self.segs = torch.from_numpy(sg.view(np.uint8).copy()).to(dev)
        self.nchunks = len(chunks)
        self.scales = (torch.cat(scale_parts).to(dev) if scale_parts else torch.zeros(1, device=dev))
        self.copy = torch.empty(flat.total, dtype=torch.bfloat16, device=dev) if copy else None
        self.hyper = torch.zeros(4, dtype=torch.float32, device=dev)
        self.iter = torch.zeros(1, dtype=torch.int64, device=dev)
        self.generation = 0
        self._lr = None
        self.host_iter = 0

    def set_lr(self, lr: float) -> None:
        if self._lr != lr:
            self.hyper[1] = lr
            self._lr = lr


_PLANS = {}


# fp8 head weights requantised by one batched launch per optimizer step (ComputeWeights.hx8_quant); a switch for
# same-process A/Bs (scripts/bench_switch.py), not an environment knob
HX8_BATCH = True


class ComputeWeights:
    """bf16 compute copies of the conv weights with the frozen-BN scale folded in (``W * s``).

    They live in the Adam plan's copy buffer: the fused Adam kernel rewrites them as a by-product of
    every optimizer step (no per-layer fold / cast launches in the forward), ``refresh()`` rebuilds
    them after weights are replaced (checkpoint load, broadcast).  ``_effective`` in
    :mod:`native_conv` serves layers from here while this object is active.
    """

    def __init__(self, flat, convs):
        self.flat = flat
        self.convs = [c for c in convs]
        self.build()

    def build(self):
        scales = {}
        for c in self.convs:
            if getattr(c, "bn", None) is not None:
                scales[id(c.weight)] = c.bn.scale_shift()[0]
        plan = AdamPlan(self.flat, scales=scales, copy=True)
        _PLANS[id(self.flat)] = plan
        self.plan = plan
        import weakref
        self.views = {}
        for seg in self.flat.segments:
            self.views[id(seg.param)] = (weakref.ref(seg.param),
                                         plan.copy[seg.offset:seg.offset + seg.numel].view(seg.shape))
        self._build_flips()
        self.__dict__.pop("hviews", None)    # hx32-packed copies: rebuilt lazily over the new plan
        for k in ("q8views", "q8table", "q8done", "q8served", "_fptrs"):    # fp8 copies: likewise
            self.__dict__.pop(k, None)
        self.refresh()

    def refresh(self):
        p = self.plan
        _chk(lib().mxr_refresh_copy(_p(self.flat.data), _p(p.copy), _p(p.scales), _p(p.chunks), p.nchunks,
                                    _p(p.segs), _s()), "refresh_copy")
        p.generation += 1

    # ------------------------------------------------------------------ flipped (data-gradient) weights
    def _build_flips(self):
        """Flip-transposed copies W[co][ky][kx][ci] -> Wd[ci][kh-1-ky][kw-1-kx][co] of every 4-D weight,
        rebuilt by ONE batched launch (mxr_flip_batch) the first time a data gradient asks for one after
        the compute copies changed -- instead of one flip launch per layer per step."""
        import numpy as np
        dev = self.plan.copy.device
        segs, tiles, self.fviews = [], [], {}
        self.fcopy = torch.empty_like(self.plan.copy)
        for seg in self.flat.segments:
            if len(seg.shape) != 4:
                continue
            co, kh, kw, ci = (int(v) for v in seg.shape)
            si = len(segs)
            segs.append((seg.offset, seg.offset, co, kh, kw, ci))
            self.fviews[self.plan.copy[seg.offset:].data_ptr()] = (
                self.fcopy[seg.offset:seg.offset + seg.numel].view(ci, kh, kw, co), tuple(seg.shape))
            for tap in range(kh * kw):
                for c0 in range(0, co, 32):
                    for i0 in range(0, ci, 32):
                        tiles.append((si, tap, c0, i0))
        st = np.zeros(len(segs), dtype=[("src", "<i8"), ("dst", "<i8"), ("cout", "<i4"), ("kh", "<i4"),
                                        ("kw", "<i4"), ("cin", "<i4")])
        for i, t in enumerate(segs):
            st[i] = t
        self.fsegs = torch.from_numpy(st.view(np.uint8).copy()).to(dev)
        self.ftiles = torch.tensor(tiles if tiles else [(0, 0, 0, 0)], dtype=torch.int32, device=dev)
        self.ntiles = len(tiles)
        self.fdone = -1

    def flipped(self, w: torch.Tensor) -> Optional[torch.Tensor]:
        """The flip-transposed copy of compute weight ``w`` (a view served by :meth:`get`), or None."""
        e = self.fviews.get(w.data_ptr())
        if e is None or tuple(w.shape) != e[1] or w.dtype != torch.bfloat16:
            return None
        if self.fdone != self.plan.generation:
            _chk(lib().mxr_flip_batch(_p(self.plan.copy), _p(self.fcopy), _p(self.fsegs), _p(self.ftiles),
                                      self.ntiles, _s()), "flip_batch")
            self.fdone = self.plan.generation
        return e[0]

    # ------------------------------------------------------------------ hx32-packed weights
    def _build_hx32(self):
        """conv_hx32's packed layout ([tap][cin / 32][plane][cout][16]) of every 3x3 compute weight it can
        run -- the forward copy (cin % 32 == 0) and the flipped data-gradient copy (cout % 32 == 0) --
        rebuilt by ONE batched launch (mxr_hx32_pack_batch) per optimizer step, the first time a hx32
        launch asks for one, instead of one pack launch per conv call."""
        import numpy as np
        dev = self.plan.copy.device
        segs, self.hviews, self.hflip = [], {}, False
        doff = ustart = 0
        pending = []
        for seg in self.flat.segments:
            if len(seg.shape) != 4 or tuple(seg.shape[1:3]) != (3, 3):
                continue
            co, _, _, ci = (int(v) for v in seg.shape)
            fwd = self.plan.copy[seg.offset:seg.offset + seg.numel]
            if ci % 32 == 0 and co % 8 == 0:
                pending.append((fwd, co, ci, tuple(seg.shape)))
            if co % 32 == 0 and ci % 8 == 0:
                flip = self.fcopy[seg.offset:seg.offset + seg.numel]
                pending.append((flip, ci, co, (ci, 3, 3, co)))
                self.hflip = True
        n = sum(int(t.numel()) for t, _, _, _ in pending)
        self.hbuf = torch.empty(max(n, 8), dtype=torch.bfloat16, device=dev)
        for src, co, ci, shape in pending:
            numel = int(src.numel())
            segs.append((src.data_ptr(), doff, ustart, co, ci))
            self.hviews[src.data_ptr()] = (self.hbuf[doff:doff + numel], shape)
            doff += numel
            ustart += numel // 8
        st = np.zeros(max(len(segs), 1), dtype=[("src", "<i8"), ("doff", "<i8"), ("ustart", "<i8"), ("cout", "<i4"),
                                                ("cin", "<i4")])
        for i, t in enumerate(segs):
            st[i] = t
        self.hsegs = torch.from_numpy(st.view(np.uint8).copy()).to(dev)
        self.hnseg, self.hunits, self.hdone = len(segs), ustart, -1

    def hx32_packed(self, w: torch.Tensor) -> Optional[torch.Tensor]:
        """The packed copy of compute weight ``w`` (a forward copy or a flipped copy served by this
        object), or None."""
        if not hasattr(self, "hviews"):
            self._build_hx32()
        e = self.hviews.get(w.data_ptr())
        if e is None or tuple(w.shape) != e[1] or w.dtype != torch.bfloat16:
            return None
        if self.hdone != self.plan.generation:
            if self.hflip and self.fdone != self.plan.generation:
                _chk(lib().mxr_flip_batch(_p(self.plan.copy), _p(self.fcopy), _p(self.fsegs), _p(self.ftiles),
                                          self.ntiles, _s()), "flip_batch")
                self.fdone = self.plan.generation
            _chk(lib().mxr_hx32_pack_batch(_p(self.hsegs), self.hnseg, _p(self.hbuf), self.hunits, _s()),
                 "hx32_pack_batch")
            self.hdone = self.plan.generation
        return e[0]

    def get(self, weight):
        e = self.views.get(id(weight))
        return e[1] if e is not None and e[0]() is weight else None

    # ------------------------------------------------------------------ fp8 (conv_hx32_f8) quantised weights
    def hx8_quant(self, w: torch.Tensor):
        """(packed e4m3 bytes, per-row inv scales) of compute weight ``w`` in conv_hx32_f8's layout -- a forward copy
        or a flipped data-gradient copy served by this object (3x3, cin % 64 == 0) -- or None.  A weight registers at
        its first request (quantised alone that once); from then on every registered weight is requantised by ONE
        batched launch (mxr_hx8_quant_pack_batch) per optimizer step, the first time any of them is asked for."""
        if (not HX8_BATCH or w.dtype != torch.bfloat16 or w.dim() != 4 or tuple(w.shape[1:3]) != (3, 3)
                or int(w.shape[-1]) % 64):
            return None
        if not hasattr(self, "q8views"):
            self.q8views, self.q8table, self.q8done = {}, None, -1
            self.q8served = {self.plan.copy[seg.offset:].data_ptr(): tuple(seg.shape)
                             for seg in self.flat.segments if len(seg.shape) == 4}
            self.q8served.update({v.data_ptr(): tuple(v.shape) for v, _ in self.fviews.values()})
        key = w.data_ptr()
        e = self.q8views.get(key)
        if e is None:
            if self.q8served.get(key) != tuple(w.shape) or not w.is_contiguous():
                return None
            cout, cin = int(w.shape[0]), int(w.shape[-1])
            qp = torch.empty(w.numel(), dtype=torch.uint8, device=w.device)
            inv = torch.empty(cout, dtype=torch.float32, device=w.device)
            _chk(lib().mxr_hx8_quant_pack(_p(w), cout, cin, _p(qp), _p(inv), _s()), "hx8_quant_pack")
            self.q8views[key] = (qp, inv, w)
            self.q8table = None
            return qp, inv
        if self.q8done != self.plan.generation:
            if self.fdone != self.plan.generation and any(k in self.fdone_ptrs() for k in self.q8views):
                _chk(lib().mxr_flip_batch(_p(self.plan.copy), _p(self.fcopy), _p(self.fsegs), _p(self.ftiles),
                                          self.ntiles, _s()), "flip_batch")
                self.fdone = self.plan.generation
            if self.q8table is None:
                import numpy as np
                rec = np.zeros(len(self.q8views), dtype=[("src", "<i8"), ("dst", "<i8"), ("inv", "<i8"),
                                                         ("cout", "<i4"), ("cin", "<i4"), ("row0", "<i4"),
                                                         ("pad", "<i4")])
                row0 = 0
                for i, (qp, inv, src) in enumerate(self.q8views.values()):
                    rec[i] = (src.data_ptr(), qp.data_ptr(), inv.data_ptr(), int(src.shape[0]), int(src.shape[-1]),
                              row0, 0)
                    row0 += int(src.shape[0])
                self.q8table = (torch.from_numpy(rec.view(np.uint8).copy()).to(w.device), len(rec), row0)
            t, n, rows = self.q8table
            _chk(lib().mxr_hx8_quant_pack_batch(_p(t), n, rows, _s()), "hx8_quant_pack_batch")
            self.q8done = self.plan.generation
        return e[0], e[1]

    def fdone_ptrs(self):
        """data_ptrs of the flipped copies (their batched quantisation needs this step's flip first)."""
        if not hasattr(self, "_fptrs"):
            self._fptrs = {v.data_ptr() for v, _ in self.fviews.values()}
        return self._fptrs


class GradSinks:
    """Direct delivery of conv weight/bias gradients into the flat fp32 gradient buffer.

    The wgrad / bias-grad reduction kernels ACCUMULATE straight into the parameter's slot of
    ``flat.grad`` (zeroed at the start of every step) instead of returning a temporary that autograd
    then adds in; ``notify(param)`` replaces the post-accumulate-grad hook that drives the bucketed
    all-reduce.
    """

    def __init__(self, flat, notify):
        import weakref
        self.notify = notify
        self.views = {id(s.param): (weakref.ref(s.param), flat.grad[s.offset:s.offset + s.numel].view(s.shape))
                      for s in flat.segments}

    def get(self, param):
        if param is None:
            return None
        e = self.views.get(id(param))
        return e[1] if e is not None and e[0]() is param else None


_GRAD_SINKS = [None]


def set_grad_sinks(gs: Optional[GradSinks]) -> None:
    _GRAD_SINKS[0] = gs


def grad_sinks() -> Optional[GradSinks]:
    return _GRAD_SINKS[0]


_COMPUTE_WEIGHTS = [None]


def set_compute_weights(cw: Optional[ComputeWeights]) -> None:
    _COMPUTE_WEIGHTS[0] = cw


def compute_weights() -> Optional[ComputeWeights]:
    return _COMPUTE_WEIGHTS[0]


def adam_plan(flat) -> AdamPlan:
    p = _PLANS.get(id(flat))
    if p is None:
        p = AdamPlan(flat)
        _PLANS[id(flat)] = p
    return p


def adam_step(flat, m, v, grad_scale, lr, iteration, b1, b2, eps, plan: Optional[AdamPlan] = None):
    """Fused Keras-Adam on the flat buffers.  ``lr`` is the base lr (lr_t is computed on device)."""
    plan = plan or adam_plan(flat)
    plan.set_lr(lr)
    if plan.host_iter != iteration:
        plan.iter.fill_(iteration)
    plan.host_iter = iteration + 1
    gs = grad_scale.reshape(1).float().contiguous() if torch.is_tensor(grad_scale) else \
        torch.full((1,), float(grad_scale), device=flat.data.device)
    _chk(lib().mxr_adam_step(_p(flat.data), _p(flat.grad), _p(m), _p(v), _p(plan.copy), _p(plan.scales),
                             _p(plan.chunks), plan.nchunks, _p(plan.segs), _p(gs), _p(plan.hyper), _p(plan.iter),
                             b1, b2, eps, _s()), "adam")
    plan.generation += 1     # the compute copies changed (ComputeWeights.flipped re-flips lazily)


NORM_GRID = 1024


def grad_norm_clip(g: torch.Tensor, norm_mul: float = 1.0, clipnorm: float = 0.0, scale_mul: float = 1.0) -> torch.Tensor:
    """Returns a (2,) f32 tensor: [norm * norm_mul, clip_factor * scale_mul] (all on device)."""
    part = torch.empty(NORM_GRID, dtype=torch.float32, device=g.device)
    out = torch.empty(2, dtype=torch.float32, device=g.device)
    _chk(lib().mxr_grad_norm_clip(_p(g), g.numel(), _p(part), norm_mul, clipnorm, scale_mul, _p(out), _s()), "norm")
    return out


def l2norm(g: torch.Tensor) -> torch.Tensor:
    return grad_norm_clip(g)[0]


def scale_inplace(g: torch.Tensor, s: torch.Tensor) -> None:
    _chk(lib().mxr_scale_inplace(_p(g), g.numel(), _p(s.reshape(1).float().contiguous()), _s()), "scale")


# =========================================================================================
# pooling / upsampling
# =========================================================================================
# which maxpool_fwd kernel runs for 3x3 / stride-2 bf16 pools: 1 = maxpool_fwd_k3s2 (the nine window loads
# issued together), 0 = the generic loop.  Both give identical bytes (tests/test_kernels_gpu.py).
POOL_K3S2_IMPL = 0


def maxpool_fwd_raw(x, k, s, pads, relu_in: bool = False, impl: Optional[int] = None):
    """(y, argmax) of the TF-'same' max-pool; ``relu_in``: x is a ReLU output, windows whose max is 0
    get argmax 255 so the backward also applies that ReLU's backward (nothing flows through 0)."""
    N, H, W, C = x.shape
    pt, pb, pl, pr = pads
    Ho = (H + pt + pb - k) // s + 1
    Wo = (W + pl + pr - k) // s + 1
    y = torch.empty((N, Ho, Wo, C), dtype=x.dtype, device=x.device)
    arg = torch.empty((N, Ho, Wo, C), dtype=torch.uint8, device=x.device)
    _chk(lib().mxr_maxpool_fwd(_p(x), _p(y), _p(arg), N, H, W, C, Ho, Wo, k, s, pt, pl, int(relu_in), _dt(x),
                               POOL_K3S2_IMPL if impl is None else int(impl), _s()), "maxpool")
    return y, arg


def maxpool_bwd_raw(dy, arg, x_shape, k, s, pads):
    N, H, W, C = x_shape
    Ho, Wo = dy.shape[1], dy.shape[2]
    dx = torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
    _chk(lib().mxr_maxpool_bwd(_p(dy), _p(arg), _p(dx), N, H, W, C, Ho, Wo, k, s, pads[0], pads[2], _dt(dy), _s()),
         "maxpool_bwd")
    return dx


class MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, pads):
        x = x.contiguous()
        y, arg = maxpool_fwd_raw(x, k, s, pads)
        ctx.save_for_backward(arg)
        ctx.cfg = (tuple(x.shape), k, s, pads, x.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        x_shape, k, s, pads, dt = ctx.cfg
        return maxpool_bwd_raw(dy.contiguous().to(dt), arg, x_shape, k, s, pads), None, None, None


def maxpool(x, k, s, pads):
    if x.shape[-1] % 8:
        pt, pb, pl, pr = pads
        xp = F.pad(x.permute(0, 3, 1, 2), (pl, pr, pt, pb), value=float("-inf"))
        return F.max_pool2d(xp, k, s).permute(0, 2, 3, 1).contiguous()
    return MaxPoolFn.apply(x, k, s, pads)


_UPIDX = {}


def _up_tables(h, w, H, W, device):
    key = (h, w, H, W, str(device))
    t = _UPIDX.get(key)
    if t is None:
        import numpy as np
        iy = np.minimum(np.floor(np.arange(H, dtype=np.float32) * np.float32(h / H)).astype(np.int64), h - 1)
        ix = np.minimum(np.floor(np.arange(W, dtype=np.float32) * np.float32(w / W)).astype(np.int64), w - 1)
        ys = np.searchsorted(iy, np.arange(h + 1), side="left")
        xs = np.searchsorted(ix, np.arange(w + 1), side="left")
        t = tuple(torch.from_numpy(a.astype(np.int32)).to(device) for a in (iy, ix, ys, xs))
        _UPIDX[key] = t
    return t


class UpsampleAddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, lat):
        x = x.contiguous()
        lat = lat.contiguous()
        N, h, w, C = x.shape
        H, W = lat.shape[1], lat.shape[2]
        iy, ix, ys, xs = _up_tables(h, w, H, W, x.device)
        y = torch.empty_like(lat)
        _chk(lib().mxr_upsample_add_fwd(_p(x), _p(lat), _p(y), _p(iy), _p(ix), N, h, w, H, W, C, _dt(x), _s()),
             "upsample_add")
        ctx.cfg = (N, h, w, H, W, C)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, h, w, H, W, C = ctx.cfg
        dy = dy.contiguous()
        iy, ix, ys, xs = _up_tables(h, w, H, W, dy.device)
        dx = torch.empty((N, h, w, C), dtype=dy.dtype, device=dy.device)
        _chk(lib().mxr_upsample_bwd(_p(dy), _p(dx), _p(ys), _p(xs), N, h, w, H, W, C, _dt(dy), _s()), "upsample_bwd")
        return dx, dy


def upsample_add(x, lat):
    if x.shape[-1] % 8 or x.dtype != lat.dtype:
        from .conv import upsample_like
        return lat + upsample_like(x, lat.shape[1:3])
    return UpsampleAddFn.apply(x, lat)


# =========================================================================================
# detection
# =========================================================================================
def decode_clip(anchors, deltas, H, W, std=0.2):
    B, A = deltas.shape[0], deltas.shape[1]
    boxes = torch.empty((B, A, 4), dtype=torch.float32, device=deltas.device)
    d = deltas.contiguous()
    _chk(lib().mxr_decode_clip(_p(anchors.contiguous()), _p(d), _dt(d), _p(boxes), B, A, std, float(H), float(W),
                               _s()), "decode")
    return boxes


def nms(boxes: torch.Tensor, scores: torch.Tensor, thr: float, max_out: int) -> torch.Tensor:
    """Indices kept (into ``boxes``), in decreasing score order."""
    n = boxes.shape[0]
    if n == 0:
        return torch.zeros(0, dtype=torch.long, device=boxes.device)
    order = torch.argsort(scores, descending=True, stable=True)
    b = boxes[order].float().contiguous()
    words = (n + 63) // 64
    if words * 8 > 64 * 1024:
        from .boxes import nms as nms_torch
        return nms_torch(boxes, scores, thr, max_out)
    mask = torch.empty((n, words), dtype=torch.int64, device=boxes.device)
    keep = torch.empty(min(n, max_out), dtype=torch.int32, device=boxes.device)
    nk = torch.empty(1, dtype=torch.int32, device=boxes.device)
    _chk(lib().mxr_nms(_p(b), n, thr, max_out, _p(mask), _p(keep), _p(nk), _s()), "nms")
    k = int(nk.item())
    return order[keep[:k].long()]


FILTER_CAP = 4096


def filter_detections_batched(anchors: torch.Tensor, deltas: torch.Tensor, cls_logits: torch.Tensor, H: float,
                              W: float, score_threshold: float = 0.05, nms_threshold: float = 0.5,
                              max_detections: int = 300, box_std: float = 0.2, cap: int = FILTER_CAP):
    """Class-specific FilterDetections for a whole batch on the device (csrc/kernels/filter.hip).

    anchors (A, 4) fp32, deltas (B, A, 4), cls_logits (B, A, C) bf16/fp32 LOGITS (sigmoid applied in the
    kernel).  Returns boxes (B, D, 4), scores (B, D), labels (B, D) int32 padded with -1 (D = max_detections).
    Two launches per batch (select, per-(image, class) sort + greedy NMS) and one torch.topk; the only host
    sync is the overflow check (an (image, class) with more than ``cap`` candidates is re-run exactly)."""
    B, A, C = cls_logits.shape
    dev = cls_logits.device
    D = int(max_detections)
    if C % 8 != 0:
        pad = (C + 7) // 8 * 8 - C
        cls_logits = torch.nn.functional.pad(cls_logits, (0, pad), value=-1e4)
    Cp = cls_logits.shape[-1]
    cls_logits = cls_logits.contiguous()
    deltas = deltas.contiguous()
    anchors = anchors.float().contiguous()
    cnt = torch.zeros(B * Cp, dtype=torch.int32, device=dev)
    cand = torch.empty(B * Cp * cap, dtype=torch.int64, device=dev)
    _chk(lib().mxr_filter_select(_p(cls_logits), 1 if cls_logits.dtype == torch.bfloat16 else 0, B, A, Cp,
                                 float(score_threshold), _p(cnt), _p(cand), cap, _s()), "filter_select")
    out_s = torch.full((B * Cp * D,), -1.0, dtype=torch.float32, device=dev)
    out_b = torch.full((B * Cp * D, 4), -1.0, dtype=torch.float32, device=dev)
    out_n = torch.zeros(B * Cp, dtype=torch.int32, device=dev)
    ovf = torch.zeros(B * Cp, dtype=torch.int32, device=dev)
    ddt = 1 if deltas.dtype == torch.bfloat16 else 0
    if ddt == 0 and deltas.dtype != torch.float32:
        deltas = deltas.float()
    _chk(lib().mxr_filter_nms(_p(cand), _p(cnt), cap, 0, 0, B * Cp, _p(anchors), _p(deltas), ddt, A, Cp, float(H),
                              float(W), float(box_std), float(nms_threshold), D, _p(out_s), _p(out_b), _p(out_n),
                              _p(ovf), _s()), "filter_nms")
    if bool(ovf.any()):
        # exact path for crowded (image, class) pairs: full candidate list, sorted on the device
        for seg in torch.nonzero(ovf).flatten().tolist():
            b, c = divmod(seg, Cp)
            p = torch.sigmoid(cls_logits[b, :, c].float())
            idx = torch.nonzero(p > score_threshold).flatten()
            order = torch.argsort(p[idx], descending=True, stable=True)
            idx = idx[order]
            keys = (p[idx].view(torch.int32).to(torch.int64) << 32) | (0xFFFFFFFF - idx).to(torch.int64)
            n = torch.tensor([idx.numel()], dtype=torch.int32, device=dev)
            _chk(lib().mxr_filter_nms(_p(keys.contiguous()), _p(n), 0, 1, seg, 1, _p(anchors), _p(deltas), ddt, A,
                                      Cp, float(H), float(W), float(box_std), float(nms_threshold), D, _p(out_s),
                                      _p(out_b), _p(out_n), _p(ovf), _s()), "filter_nms_exact")
    scores = out_s.view(B, Cp * D)
    k = min(D, Cp * D)
    top_s, top_i = torch.topk(scores, k, dim=1)
    boxes = out_b.view(B, Cp * D, 4).gather(1, top_i[..., None].expand(B, k, 4))
    labels = (top_i // D).to(torch.int32)
    valid = top_s >= 0
    labels = torch.where(valid, labels, torch.full_like(labels, -1))
    boxes = torch.where(valid[..., None], boxes, torch.full_like(boxes, -1.0))
    top_s = torch.where(valid, top_s, torch.full_like(top_s, -1.0))
    return boxes, top_s, labels


# =========================================================================================
# device image preprocessing (data/device_preprocess.py)
# =========================================================================================
def image_warp_normalize(src: torch.Tensor, matrix=None, out_hw=None, interp: int = 1, border: int = 1,
                         cval: float = 0.0, scale: float = 1.0, mean=(0.0, 0.0, 0.0)) -> torch.Tensor:
    """uint8 HWC(3) -> float32 HWC: ``x*scale - mean`` then (optionally) the affine warp ``matrix``."""
    assert src.dtype == torch.uint8 and src.dim() == 3 and src.shape[2] == 3 and src.is_contiguous()
    H, W = int(src.shape[0]), int(src.shape[1])
    OH, OW = (H, W) if out_hw is None else (int(out_hw[0]), int(out_hw[1]))
    dst = torch.empty((OH, OW, 3), dtype=torch.float32, device=src.device)
    m = (ctypes.c_double * 6)()
    warp = 0
    if matrix is not None:
        import numpy as np
        a = np.asarray(matrix, dtype=np.float64).reshape(-1)[:6]
        for i in range(6):
            m[i] = float(a[i])
        warp = 1
    _chk(lib().mxr_image_warp_normalize(_p(src), H, W, _p(dst), OH, OW, ctypes.cast(m, c_vp), warp, int(interp),
                                        int(border), float(cval), float(scale), float(mean[0]), float(mean[1]),
                                        float(mean[2]), _s()), "image_warp")
    return dst


def image_resize_into(src: torch.Tensor, batch: torch.Tensor, index: int, out_hw) -> None:
    """Bilinear (cv2 INTER_LINEAR) resize of float HWC ``src`` into ``batch[index, :OH, :OW]``."""
    assert src.dtype == torch.float32 and src.is_contiguous() and batch.is_contiguous() and batch.shape[3] == 3
    OH, OW = int(out_hw[0]), int(out_hw[1])
    if OH > batch.shape[1] or OW > batch.shape[2]:
        raise ValueError("resize target {} exceeds batch slot {}".format((OH, OW), tuple(batch.shape[1:3])))
    dt = {torch.float32: 0, torch.bfloat16: 1}[batch.dtype]
    _chk(lib().mxr_image_resize_into(_p(src), int(src.shape[0]), int(src.shape[1]), _p(batch[index]), OH, OW,
                                     int(batch.shape[2]) * 3, dt, _s()), "image_resize")


# =========================================================================================
# convolution (see native_conv.py)
# =========================================================================================
def __getattr__(name):
    if name.startswith("__"):
        # module protocol lookups (``from .native import X`` probes ``__path__``) must not import native_conv:
        # importing a conv module first then re-entered it half-initialised (circular import)
        raise AttributeError(name)
    from . import native_conv
    try:
        return getattr(native_conv, name)
    except AttributeError:
        raise AttributeError(name) from None
