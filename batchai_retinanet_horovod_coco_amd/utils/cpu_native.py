"""ctypes bindings to ``_lib/libmxr_cpu.so`` (host C++ runtime) with numpy fallbacks.

Functions: ``compute_overlap`` (+1 IoU, replaces the reference's Cython), ``resize_bilinear`` /
``warp_affine`` (replace cv2.resize / cv2.warpAffine, absent here), ``nms`` (TF CPU NMS
semantics), ``coco_iou`` (pycocotools bbox IoU with iscrowd), ``coco_match`` (COCOeval's greedy matching), ``crc32c`` (TensorBoard framing).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# MXR_CPU_LIB: an alternative build of the same library (the ASan/UBSan one: build.py --sanitize)
LIB_PATH = os.environ.get("MXR_CPU_LIB") or os.path.join(_PKG, "_lib", "libmxr_cpu.so")
_LIB: Optional[ctypes.CDLL] = None
_TRIED = [False]
import threading as _threading
_LOCK = _threading.Lock()

_dp = ctypes.POINTER(ctypes.c_double)
_fp = ctypes.POINTER(ctypes.c_float)
_ip = ctypes.POINTER(ctypes.c_int)
_bp = ctypes.POINTER(ctypes.c_ubyte)


def lib() -> Optional[ctypes.CDLL]:
    if _LIB is None:
        with _LOCK:
            return _load()
    return _LIB


def _load() -> Optional[ctypes.CDLL]:
    global _LIB
    if _LIB is None and not _TRIED[0]:
        _TRIED[0] = True
        if not os.path.exists(LIB_PATH):
            try:
                from .. import build
                build.build_cpu()
            except Exception:  # noqa: BLE001
                return None
        try:
            L = ctypes.CDLL(LIB_PATH)
        except OSError:
            return None
        L.mxr_cpu_compute_overlap.argtypes = [_dp, ctypes.c_longlong, _dp, ctypes.c_longlong, _dp]
        L.mxr_cpu_compute_overlap.restype = None
        L.mxr_cpu_resize_bilinear.argtypes = [_fp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _fp, ctypes.c_int,
                                              ctypes.c_int]
        L.mxr_cpu_resize_bilinear.restype = None
        L.mxr_cpu_warp_affine.argtypes = [_fp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, _fp, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float]
        L.mxr_cpu_warp_affine.restype = None
        L.mxr_cpu_nms.argtypes = [_fp, _fp, ctypes.c_int, ctypes.c_float, ctypes.c_int, _ip]
        L.mxr_cpu_nms.restype = ctypes.c_int
        L.mxr_cpu_coco_iou.argtypes = [_dp, ctypes.c_int, _dp, ctypes.c_int, _bp, _dp]
        L.mxr_cpu_coco_iou.restype = None
        L.mxr_cpu_coco_match.argtypes = [_dp, ctypes.c_int, ctypes.c_int, _ip, _bp, _bp, _dp, ctypes.c_int, _ip]
        L.mxr_cpu_coco_match.restype = None
        L.mxr_crc32c.argtypes = [ctypes.c_char_p, ctypes.c_longlong, ctypes.c_uint32]
        L.mxr_crc32c.restype = ctypes.c_uint32
        _LIB = L
    return _LIB


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def compute_overlap(boxes: np.ndarray, query: np.ndarray) -> np.ndarray:
    b, q = _c(boxes, np.float64).reshape(-1, 4), _c(query, np.float64).reshape(-1, 4)
    L = lib()
    if L is None:
        from ..ops.anchors import compute_overlap as py
        return py(b, q)
    out = np.empty((b.shape[0], q.shape[0]), dtype=np.float64)
    L.mxr_cpu_compute_overlap(b.ctypes.data_as(_dp), b.shape[0], q.ctypes.data_as(_dp), q.shape[0],
                              out.ctypes.data_as(_dp))
    return out


def resize_bilinear(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    src = _c(img, np.float32)
    squeeze = src.ndim == 2
    if squeeze:
        src = src[..., None]
    H, W, C = src.shape
    L = lib()
    if L is None:
        out = _resize_np(src, out_h, out_w)
    else:
        out = np.empty((out_h, out_w, C), dtype=np.float32)
        L.mxr_cpu_resize_bilinear(src.ctypes.data_as(_fp), H, W, C, out.ctypes.data_as(_fp), out_h, out_w)
    return out[..., 0] if squeeze else out


def _resize_np(src, oh, ow):
    H, W, _ = src.shape
    fy = np.clip((np.arange(oh) + 0.5) * H / oh - 0.5, 0, H - 1)
    fx = np.clip((np.arange(ow) + 0.5) * W / ow - 0.5, 0, W - 1)
    y0 = np.floor(fy).astype(int)
    x0 = np.floor(fx).astype(int)
    y1 = np.minimum(y0 + 1, H - 1)
    x1 = np.minimum(x0 + 1, W - 1)
    ty = (fy - y0)[:, None, None].astype(np.float32)
    tx = (fx - x0)[None, :, None].astype(np.float32)
    top = src[y0][:, x0] + (src[y0][:, x1] - src[y0][:, x0]) * tx
    bot = src[y1][:, x0] + (src[y1][:, x1] - src[y1][:, x0]) * tx
    return (top + (bot - top) * ty).astype(np.float32)


BORDER = {"constant": 0, "nearest": 1, "reflect": 2, "wrap": 3}
INTERP = {"nearest": 0, "linear": 1}


def warp_affine(img: np.ndarray, matrix: np.ndarray, out_hw=None, interpolation="linear", fill_mode="nearest",
                cval: float = 0.0) -> np.ndarray:
    src = _c(img, np.float32)
    squeeze = src.ndim == 2
    if squeeze:
        src = src[..., None]
    H, W, C = src.shape
    oh, ow = out_hw if out_hw is not None else (H, W)
    M = _c(np.asarray(matrix, dtype=np.float64)[:2, :3], np.float64)
    L = lib()
    if L is None:
        raise RuntimeError("libmxr_cpu.so not available for warp_affine")
    out = np.empty((oh, ow, C), dtype=np.float32)
    L.mxr_cpu_warp_affine(src.ctypes.data_as(_fp), H, W, C, M.ctypes.data_as(_dp), out.ctypes.data_as(_fp), oh, ow,
                          INTERP[interpolation], BORDER[fill_mode], float(cval))
    return out[..., 0] if squeeze else out


def nms(boxes: np.ndarray, scores: np.ndarray, thr: float, max_out: int) -> np.ndarray:
    b, s = _c(boxes, np.float32).reshape(-1, 4), _c(scores, np.float32).reshape(-1)
    L = lib()
    keep = np.empty(max(1, min(max_out, b.shape[0])), dtype=np.int32)
    if b.shape[0] == 0:
        return keep[:0]
    k = L.mxr_cpu_nms(b.ctypes.data_as(_fp), s.ctypes.data_as(_fp), b.shape[0], float(thr), int(max_out),
                      keep.ctypes.data_as(_ip))
    return keep[:k]


def coco_iou(dt: np.ndarray, gt: np.ndarray, iscrowd) -> np.ndarray:
    d, g = _c(dt, np.float64).reshape(-1, 4), _c(gt, np.float64).reshape(-1, 4)
    c = _c(np.asarray(iscrowd, dtype=np.uint8).reshape(-1), np.uint8)
    out = np.zeros((d.shape[0], g.shape[0]), dtype=np.float64)
    if d.shape[0] == 0 or g.shape[0] == 0:
        return out
    L = lib()
    L.mxr_cpu_coco_iou(d.ctypes.data_as(_dp), d.shape[0], g.ctypes.data_as(_dp), g.shape[0], c.ctypes.data_as(_bp),
                       out.ctypes.data_as(_dp))
    return out


def coco_match(iou: np.ndarray, order: np.ndarray, gt_ignore: np.ndarray, crowd: np.ndarray,
               thresholds: np.ndarray) -> np.ndarray:
    """COCOeval's greedy matching of one (image, category, area range) at every IoU threshold: ``iou`` (D, G) with
    the detections in score order, ``order`` the gt columns with the ignored gts last, ``gt_ignore`` in that order,
    ``crowd`` in column order.  Returns (T, D) int32: position in ``order`` of each detection's gt, or -1."""
    iou = _c(iou, np.float64)
    nd, ng = iou.shape
    thr = _c(thresholds, np.float64).reshape(-1)
    out = np.full((thr.shape[0], nd), -1, dtype=np.int32)
    if nd == 0 or ng == 0:
        return out
    o = _c(order, np.int32).reshape(-1)
    ig = _c(gt_ignore, np.uint8).reshape(-1)
    cr = _c(crowd, np.uint8).reshape(-1)
    L = lib()
    if L is not None:
        L.mxr_cpu_coco_match(iou.ctypes.data_as(_dp), nd, ng, o.ctypes.data_as(_ip), ig.ctypes.data_as(_bp),
                             cr.ctypes.data_as(_bp), thr.ctypes.data_as(_dp), thr.shape[0], out.ctypes.data_as(_ip))
        return out
    sub = iou[:, o]                                 # (same algorithm, host Python: the library is missing)
    crs = cr[o].astype(bool)
    for t, th in enumerate(thr):
        taken = np.zeros(ng, dtype=bool)
        for d in range(nd):
            best, m = min(th, 1 - 1e-10), -1
            for g in range(ng):
                if taken[g] and not crs[g]:
                    continue
                if m >= 0 and not ig[m] and ig[g]:
                    break
                if sub[d, g] >= best:
                    best, m = sub[d, g], g
            out[t, d] = m
            if m >= 0:
                taken[m] = True
    return out


_CRC_TABLE = None


def crc32c(data: bytes, crc: int = 0) -> int:
    L = lib()
    if L is not None:
        return int(L.mxr_crc32c(data, len(data), crc))
    global _CRC_TABLE
    if _CRC_TABLE is None:
        t = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (0x82F63B78 ^ (c >> 1)) if (c & 1) else (c >> 1)
            t.append(c)
        _CRC_TABLE = t
    crc ^= 0xFFFFFFFF
    for byte in data:
        crc = _CRC_TABLE[(crc ^ byte) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF
