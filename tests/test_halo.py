"""Halo tile tables (ops/halo.py) for the 3x3 halo-staged conv kernel: coverage, limits, and a numpy
model of the kernel's addressing against a direct convolution (CPU)."""
import numpy as np
import pytest

from batchai_retinanet_horovod_coco_amd.ops import halo as HX

PYR = [(100, 167), (50, 84), (25, 42), (13, 21), (7, 11)]


@pytest.mark.parametrize("N,shapes", [(16, PYR), (2, [(200, 334)]), (3, [(10, 17), (5, 9), (3, 5), (2, 3), (1, 2)]),
                                      (1, [(1, 1)]), (2, [(300, 7)]), (2, [(3, 400)]), (4, [(25, 42)])])
def test_tiles_cover_every_pixel_once(N, shapes):
    tab = HX.build_tiles(N, shapes)
    assert tab.shape[1] == HX.TILE_INTS
    HX.check_tiles(tab, N, shapes)


def test_head_tile_waste_small():
    tab = HX.build_tiles(16, PYR)
    assert HX.waste(tab, 16, PYR) < 0.05
    assert tab[:, 2].max() <= HX.HX_HMAX


def _direct(x, w, N, shapes):
    P, cin = x.shape
    y = np.zeros((P, w.shape[0]))
    img = sum(h * wd for h, wd in shapes)
    for b in range(N):
        off = b * img
        for (h, wd) in shapes:
            xp = np.zeros((h + 2, wd + 2, cin))
            xp[1:-1, 1:-1] = x[off:off + h * wd].reshape(h, wd, cin)
            for ky in range(3):
                for kx in range(3):
                    y[off:off + h * wd] += (xp[ky:ky + h, kx:kx + wd].reshape(-1, cin) @ w[:, ky, kx, :].T)
            off += h * wd
    return y


@pytest.mark.parametrize("N,shapes", [(2, [(10, 17), (5, 9), (3, 5), (2, 3), (1, 2)]), (1, [(20, 90)]),
                                      (3, [(4, 4)])])
def test_emulated_kernel_matches_direct_conv(N, shapes):
    rng = np.random.default_rng(0)
    P = N * sum(h * w for h, w in shapes)
    x = rng.standard_normal((P, 5))
    w = rng.standard_normal((3, 3, 3, 5))
    tab = HX.build_tiles(N, shapes)
    np.testing.assert_allclose(HX.emulate(x, w, tab), _direct(x, w, N, shapes), atol=1e-9)


def test_covers_geometry():
    from batchai_retinanet_horovod_coco_amd.ops.native import ConvGeom  # noqa: F401  (ctypes only)
    from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC
    assert HX.covers(NC.geom_pyramid(16, PYR, 256, 256))
    assert HX.covers(NC.geom_single(2, 20, 30, 20, 30, 3, 1, (1, 1, 1, 1), 64, 64))
    assert not HX.covers(NC.geom_single(2, 20, 30, 10, 15, 3, 2, (1, 1, 1, 1), 64, 64))
    assert not HX.covers(NC.geom_single(2, 20, 30, 20, 30, 1, 1, (0, 0, 0, 0), 64, 64))
    assert not HX.covers(NC.geom_pyramid(16, PYR, 256, 36))      # cout % 8


def test_splitk_plan_only_for_small_grids():
    """conv_launch.splitk_splits: the split-K pipe form is offered only to grids under one chip round (FPN P6 / P7)
    and keeps >= 8 K sub-stages per split."""
    from batchai_retinanet_horovod_coco_amd.ops import conv as C
    from batchai_retinanet_horovod_coco_amd.ops import conv_launch as CL

    def g(n, H, W, cin, cout, k, s):
        pads = C.same_pads((H, W), k, s) if k > 1 else (0, 0, 0, 0)
        Ho, Wo = C.out_hw((H, W), k, s, pads)
        return CL.geom_single(n, H, W, Ho, Wo, k, s, pads, cin, cout)
    p6 = g(16, 25, 42, 2048, 256, 3, 2)
    assert CL.splitk_splits(p6, 11) == 7 and (p6.kh * p6.kw * p6.cin // 32) // 7 >= 8
    assert CL.splitk_splits(g(16, 13, 21, 256, 256, 3, 2), 12) == 9
    assert CL.splitk_splits(g(16, 100, 167, 256, 256, 3, 1), 11) == 0        # a big grid: no split-K


def test_native_dunder_probe_does_not_import_conv_modules():
    """``from .native import X`` probes ``native.__path__``; the lazy ``__getattr__`` must not import native_conv
    for it (importing conv_launch first then hit a circular import)."""
    import subprocess
    import sys
    code = ("import batchai_retinanet_horovod_coco_amd.ops.native as n, sys;"
            "hasattr(n, '__path__');"
            "assert 'batchai_retinanet_horovod_coco_amd.ops.native_conv' not in sys.modules;"
            "from batchai_retinanet_horovod_coco_amd.ops import conv_launch")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
