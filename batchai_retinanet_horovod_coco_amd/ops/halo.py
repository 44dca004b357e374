"""Tile tables for the halo-staged 3x3 convolution kernel (``csrc/kernels/conv_halo.hip``).

A 3x3 / stride-1 / pad-1 conv (the head towers and finals over the packed pyramid, the FPN
smoothing convs, the backbone 3x3 convs -- SURVEY §2.6 K1/K2) is tiled into 256-slot tiles of up to
four rectangular *boxes* of output pixels.  A box is ``R`` rows x ``C`` columns of one image and one
pyramid level; the kernel stages its halo -- ``(R + 2) x (C + 2)`` input pixels -- once per
32-channel chunk and lets all 9 taps read it, instead of re-fetching the im2col rows per tap.

Layout per tile (44 int32, ``HaloTile`` in the kernel)::

    nbox, nslot, nhalo, 0,
    4 x (sbeg, hoff, in_base, out_base, H, W, y0, x0, R, C)

``sbeg`` / ``hoff``: first output slot / first halo pixel of the box inside the tile; ``in_base`` /
``out_base``: pixel index of (0, 0) of that image and level in the input / output tensor.

:func:`emulate` runs a tile table through a numpy model of the kernel's addressing (halo fill,
per-tap shifted reads, epilogue scatter) so the table logic is tested on the CPU.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

HX_BOX = 4        # boxes per tile
HX_HMAX = 448     # halo pixels per tile (one LDS buffer = 448 x 64 B per 32-channel chunk)
HX_PB = 256       # output slots per tile
# widest box.  84: a 3-row box of 84 columns has a 5 x 86 = 430-pixel halo (1.70 halo pixels per output
# pixel); 28: a 9-row box of 28 columns has 11 x 30 = 330 (1.33) -- 22 % fewer halo bytes for every halo kernel
# (no measured difference between them: profiles/r4_colmax_ab.txt; fixed at 84)
COLMAX = 84
NFIELD = 10
TILE_INTS = 4 + HX_BOX * NFIELD


def _split(n: int, parts: int) -> List[Tuple[int, int]]:
    """``n`` into ``parts`` near-equal contiguous (start, length) pieces."""
    out, start = [], 0
    for i in range(parts):
        ln = n // parts + (1 if i < n % parts else 0)
        out.append((start, ln))
        start += ln
    return out


def level_boxes(H: int, W: int) -> List[Tuple[int, int, int, int]]:
    """Boxes (y0, R, x0, C) covering one H x W level: columns split to <= COLMAX, full row bands of
    the largest R with R * C <= 256 and a halo <= HX_HMAX, plus a remainder band."""
    cols = _split(W, -(-W // COLMAX))
    cmax = max(c for _, c in cols)
    R = max(1, min(H, HX_PB // cmax))
    while R > 1 and (R + 2) * (cmax + 2) > HX_HMAX:
        R -= 1
    boxes = []
    for y0 in range(0, H, R):
        r = min(R, H - y0)
        for x0, c in cols:
            boxes.append((y0, r, x0, c))
    return boxes


def build_tiles(N: int, shapes: Sequence[Tuple[int, int]], open_tiles: int = 4) -> np.ndarray:
    """Tile table [ntiles, 44] int32 for N images whose levels ``shapes`` are packed per image in
    level order (the ConvGeom pyramid / single-level layout).  Boxes go first-fit into the last
    ``open_tiles`` open tiles (slots <= 256, halo <= 448, <= 4 boxes), in image / level / row order,
    so consecutive tiles (one XCD, one L2) touch neighbouring rows."""
    img = sum(h * w for h, w in shapes)
    offs, o = [], 0
    for h, w in shapes:
        offs.append(o)
        o += h * w
    per_level = [level_boxes(h, w) for h, w in shapes]
    tiles: List[dict] = []
    open_idx: List[int] = []
    for b in range(N):
        for lv, (H, W) in enumerate(shapes):
            base = b * img + offs[lv]
            for (y0, R, x0, C) in per_level[lv]:
                ns, nh = R * C, (R + 2) * (C + 2)
                di = None
                for ti in open_idx:
                    t = tiles[ti]
                    if len(t["boxes"]) < HX_BOX and t["nslot"] + ns <= HX_PB and t["nhalo"] + nh <= HX_HMAX:
                        di = ti
                        break
                if di is None:
                    tiles.append({"boxes": [], "nslot": 0, "nhalo": 0})
                    di = len(tiles) - 1
                    open_idx.append(di)
                    if len(open_idx) > open_tiles:
                        open_idx.pop(0)
                t = tiles[di]
                t["boxes"].append((t["nslot"], t["nhalo"], base, base, H, W, y0, x0, R, C))
                t["nslot"] += ns
                t["nhalo"] += nh
                if (t["nslot"] > HX_PB - 16 or len(t["boxes"]) == HX_BOX) and di in open_idx:
                    open_idx.remove(di)     # full: close it
    out = np.zeros((len(tiles), TILE_INTS), dtype=np.int32)
    for i, t in enumerate(tiles):
        out[i, 0:3] = (len(t["boxes"]), t["nslot"], t["nhalo"])
        for k, bx in enumerate(t["boxes"]):
            out[i, 4 + k * NFIELD:4 + (k + 1) * NFIELD] = bx
    return out


def _boxes(row) -> List[Tuple[int, ...]]:
    return [tuple(int(v) for v in row[4 + k * NFIELD:4 + (k + 1) * NFIELD]) for k in range(int(row[0]))]


def check_tiles(tab: np.ndarray, N: int, shapes: Sequence[Tuple[int, int]]) -> None:
    """Every output pixel covered exactly once; per-tile limits respected."""
    total = N * sum(h * w for h, w in shapes)
    seen = np.zeros(total, dtype=np.int32)
    for row in tab:
        nbox, nslot, nhalo = int(row[0]), int(row[1]), int(row[2])
        assert 1 <= nbox <= HX_BOX and nslot <= HX_PB and nhalo <= HX_HMAX, row[:4]
        s = h = 0
        for (sbeg, hoff, ib, ob, H, W, y0, x0, R, C) in _boxes(row):
            assert sbeg == s and hoff == h and ib == ob
            assert 0 <= y0 and y0 + R <= H and 0 <= x0 and x0 + C <= W
            for r in range(R):
                seen[ob + (y0 + r) * W + x0:ob + (y0 + r) * W + x0 + C] += 1
            s += R * C
            h += (R + 2) * (C + 2)
        assert s == nslot and h == nhalo
    assert (seen == 1).all(), "pixels covered {} .. {} times".format(seen.min(), seen.max())


def waste(tab: np.ndarray, N: int, shapes: Sequence[Tuple[int, int]]) -> float:
    """Fraction of MFMA slots that compute nothing (tiles x 256 vs output pixels)."""
    return 1.0 - N * sum(h * w for h, w in shapes) / float(len(tab) * HX_PB)


def emulate(x: np.ndarray, w: np.ndarray, tab: np.ndarray) -> np.ndarray:
    """numpy model of the kernel's data movement: x [P, cin] (every pixel of every image / level),
    w [cout, 3, 3, cin] -> y [P, cout] (fp64, no epilogue).  Follows the kernel's index math: halo
    pixel h of a box = input (y0 - 1 + h // pw, x0 - 1 + h % pw), pw = C + 2, zero outside the level;
    slot p reads halo row ``hoff + r * pw + c + ky * pw + kx`` for tap (ky, kx); the output goes to
    ``out_base + (y0 + r) * W + x0 + c``."""
    P, cin = x.shape
    cout = w.shape[0]
    y = np.zeros((P, cout), dtype=np.float64)
    for row in tab:
        nslot, nhalo = int(row[1]), int(row[2])
        boxes = _boxes(row)
        halo = np.zeros((HX_HMAX, cin))
        for h in range(nhalo):
            k = max(i for i in range(len(boxes)) if h >= boxes[i][1])
            sbeg, hoff, ib, ob, H, W, y0, x0, R, C = boxes[k]
            hr, hc = divmod(h - hoff, C + 2)
            yy, xx = y0 - 1 + hr, x0 - 1 + hc
            if 0 <= yy < H and 0 <= xx < W:
                halo[h] = x[ib + yy * W + xx]
        for p in range(nslot):
            k = max(i for i in range(len(boxes)) if p >= boxes[i][0])
            sbeg, hoff, ib, ob, H, W, y0, x0, R, C = boxes[k]
            r, c = divmod(p - sbeg, C)
            pw = C + 2
            hb = hoff + r * pw + c
            acc = np.zeros(cout)
            for ky in range(3):
                for kx in range(3):
                    acc += w[:, ky, kx, :] @ halo[hb + ky * pw + kx]
            y[ob + (y0 + r) * W + x0 + c] = acc
    return y


_CACHE: Dict[tuple, object] = {}


def device_tiles(N: int, shapes: Sequence[Tuple[int, int]], device):
    """(int32 tile tensor on ``device``, ntiles), cached per (device, N, shapes)."""
    import torch
    key = (str(device), int(N), tuple((int(h), int(w)) for h, w in shapes), COLMAX)
    hit = _CACHE.get(key)
    if hit is None:
        tab = build_tiles(N, key[2])
        hit = (torch.from_numpy(tab).to(device), int(tab.shape[0]))
        _CACHE[key] = hit
    return hit


def geom_shapes(g) -> List[Tuple[int, int]]:
    """Level shapes of a ConvGeom (3x3 / s1 / p1: input and output levels coincide)."""
    return [(int(g.H[l]), int(g.W[l])) for l in range(int(g.nlev))]


def geom_batch(g) -> int:
    return int(g.M // max(1, g.out_img))


def covers(g) -> bool:
    """Geometry the halo kernel implements: 3x3, stride 1, pad 1, same-size output, cin % 32 == 0,
    cout % 8 == 0, 32-bit element offsets."""
    if not (g.kh == 3 and g.kw == 3 and g.stride == 1 and g.pt == 1 and g.pl == 1 and g.ostride == 1):
        return False
    if g.cin % 32 or g.cout % 8:
        return False
    if any(g.H[l] != g.Ho[l] or g.W[l] != g.Wo[l] for l in range(g.nlev)):
        return False
    if g.in_img != g.out_img:
        return False
    return (g.M + 1) * max(g.cin, g.cout) < 2 ** 31
