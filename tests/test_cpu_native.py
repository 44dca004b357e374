"""Every entry point of the host C++ runtime (csrc/cpu/runtime_cpu.cpp) against numpy references.

Also the test set of the sanitizer run: scripts/run_sanitized_cpu_tests.sh loads the ASan/UBSan build of
the same library (MXR_CPU_LIB) and runs this file plus the data / IO tests."""
import os

import numpy as np
import pytest

from batchai_retinanet_horovod_coco_amd.utils import cpu_native as cn

pytestmark = pytest.mark.skipif(cn.lib() is None, reason="libmxr_cpu.so not built")


def test_library_is_the_requested_build():
    want = os.environ.get("MXR_CPU_LIB")
    if want:
        assert cn.LIB_PATH == want and cn.lib() is not None


def _overlap_ref(a, b):
    iw = np.minimum(a[:, None, 2], b[None, :, 2]) - np.maximum(a[:, None, 0], b[None, :, 0]) + 1
    ih = np.minimum(a[:, None, 3], b[None, :, 3]) - np.maximum(a[:, None, 1], b[None, :, 1]) + 1
    inter = np.clip(iw, 0, None) * np.clip(ih, 0, None)
    area_b = (b[:, 2] - b[:, 0] + 1) * (b[:, 3] - b[:, 1] + 1)
    area_a = (a[:, 2] - a[:, 0] + 1) * (a[:, 3] - a[:, 1] + 1)
    ua = area_a[:, None] + area_b[None, :] - inter
    return np.where(inter > 0, inter / ua, 0.0)


@pytest.mark.parametrize("n,k", [(0, 3), (7, 0), (1, 1), (513, 17)])
def test_compute_overlap(n, k):
    rng = np.random.default_rng(n + k)
    a = np.sort(rng.uniform(0, 300, (n, 4)).reshape(n, 2, 2), axis=1).transpose(0, 2, 1).reshape(n, 4)
    b = np.sort(rng.uniform(0, 300, (k, 4)).reshape(k, 2, 2), axis=1).transpose(0, 2, 1).reshape(k, 4)
    a = a[:, [0, 2, 1, 3]] if n else a
    b = b[:, [0, 2, 1, 3]] if k else b
    got = cn.compute_overlap(a, b)
    assert got.shape == (n, k)
    if n and k:
        np.testing.assert_allclose(got, _overlap_ref(a, b), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("shape,out", [((1, 1, 3), (5, 7)), ((17, 23, 3), (9, 40)), ((31, 5), (62, 10))])
def test_resize_bilinear(shape, out):
    img = np.random.default_rng(1).uniform(0, 255, shape).astype(np.float32)
    got = cn.resize_bilinear(img, *out)
    src = img if img.ndim == 3 else img[..., None]
    ref = cn._resize_np(src, *out)
    ref = ref if img.ndim == 3 else ref[..., 0]
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("fill", ["constant", "nearest", "reflect", "wrap"])
@pytest.mark.parametrize("interp", ["nearest", "linear"])
def test_warp_affine_identity_and_shift(fill, interp):
    img = np.random.default_rng(2).uniform(0, 255, (13, 19, 3)).astype(np.float32)
    same = cn.warp_affine(img, np.eye(3), interpolation=interp, fill_mode=fill)
    np.testing.assert_allclose(same, img, atol=1e-3)
    # integer shift by (dx, dy) = (3, 2): out(y, x) = in(y - 2, x - 3) inside, border rule outside
    M = np.array([[1, 0, 3], [0, 1, 2], [0, 0, 1]], dtype=np.float64)
    out = cn.warp_affine(img, M, interpolation=interp, fill_mode=fill, cval=7.0)
    np.testing.assert_allclose(out[2:, 3:], img[:-2, :-3], atol=1e-3)
    if fill == "constant":
        assert np.all(out[:2] == 7.0) and np.all(out[:, :3] == 7.0)
    # a large output canvas and a rotation stay inside the source bounds (the sanitizer run checks it)
    R = np.array([[0.8, -0.6, 10.0], [0.6, 0.8, -4.0], [0, 0, 1]])
    big = cn.warp_affine(img, R, out_hw=(41, 37), interpolation=interp, fill_mode=fill)
    assert big.shape == (41, 37, 3) and np.isfinite(big).all()


def _nms_ref(b, s, thr, k):
    order = np.argsort(-s, kind="stable")
    keep = []
    sup = np.zeros(len(b), bool)
    for i in order:
        if sup[i]:
            continue
        keep.append(i)
        if len(keep) == k:
            break
        xx1 = np.maximum(b[i, 0], b[:, 0]); yy1 = np.maximum(b[i, 1], b[:, 1])
        xx2 = np.minimum(b[i, 2], b[:, 2]); yy2 = np.minimum(b[i, 3], b[:, 3])
        inter = np.clip(xx2 - xx1, 0, None) * np.clip(yy2 - yy1, 0, None)
        area = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
        iou = inter / (area[i] + area - inter)
        sup |= iou > thr
    return np.array(keep)


@pytest.mark.parametrize("n,k", [(0, 5), (1, 5), (300, 300), (300, 10)])
def test_nms(n, k):
    rng = np.random.default_rng(n)
    xy = rng.uniform(0, 100, (n, 2))
    wh = rng.uniform(5, 40, (n, 2))
    b = np.concatenate([xy, xy + wh], 1).astype(np.float32)
    s = rng.uniform(0, 1, n).astype(np.float32)
    got = cn.nms(b, s, 0.5, k)
    if n == 0:
        assert got.size == 0
    else:
        np.testing.assert_array_equal(got, _nms_ref(b.astype(np.float64), s, 0.5, k))


def test_coco_iou_crowd():
    dt = np.array([[0, 0, 10, 10], [5, 5, 10, 10]], dtype=np.float64)      # xywh
    gt = np.array([[0, 0, 10, 10], [0, 0, 20, 20]], dtype=np.float64)
    got = cn.coco_iou(dt, gt, [0, 1])
    assert got.shape == (2, 2)
    assert got[0, 0] == pytest.approx(1.0) and got[1, 0] == pytest.approx(25 / 175)
    # crowd gt: IoU = intersection / area(dt)
    assert got[0, 1] == pytest.approx(1.0) and got[1, 1] == pytest.approx(1.0)
    assert cn.coco_iou(np.zeros((0, 4)), gt, [0, 0]).shape == (0, 2)


def test_crc32c_known_vectors():
    assert cn.crc32c(b"") == 0
    assert cn.crc32c(b"123456789") == 0xE3069283
    data = bytes(range(256)) * 9
    assert cn.crc32c(data[100:], cn.crc32c(data[:100])) == cn.crc32c(data)


def test_sanitized_build_runs_clean(tmp_path):
    """The ASan + UBSan build of the host runtime passes its tests (the sanitizer halts on
    the first report, so a clean exit means no memory error / UB was detected)."""
    import shutil
    import subprocess
    import sys
    if os.environ.get("MXR_CPU_LIB") or shutil.which("gcc") is None:
        pytest.skip("already inside the sanitized run / no gcc")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["bash", os.path.join(root, "scripts", "run_sanitized_cpu_tests.sh"), "-k", "not sanitized"],
                       cwd=root, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:]
    assert "passed" in r.stdout


def test_side_stream_unused_on_cpu():
    import torch
    from batchai_retinanet_horovod_coco_amd.ops.side_stream import SideStream
    s = SideStream()
    assert not s.usable(torch.ones(2))
    s.join()
    with s.covering():
        pass
    assert not s.pending


def test_kernel_library_symbols_resolve():
    """Every HIP kernel the library launches has its host stub: a load with RTLD_NOW resolves all symbols
    (a kernel whose stub hipcc dropped shows up only here on the CPU, or as an OSError on the GPU box)."""
    import ctypes
    import os
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "batchai_retinanet_horovod_coco_amd", "_lib", "libmxr_kernels.so")
    if not os.path.exists(lib):
        import pytest
        pytest.skip("kernel library not built")
    ctypes.CDLL(lib, mode=os.RTLD_NOW | os.RTLD_LOCAL)
