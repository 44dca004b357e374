"""The tuned-dispatch fast path (ops.native_conv ``only=``): for every candidate the full builders offer,
building just that one yields exactly that name -- so once a key is tuned, dispatch runs the same
candidate without constructing the others (host time per conv pass; CPU: nothing is launched)."""
import pytest
import torch

from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC

SHAPES = [
    # N, H, W, cin, cout, k, stride, pads
    (2, 50, 84, 256, 256, 3, 1, (1, 1, 1, 1)),
    (2, 50, 84, 1024, 256, 1, 1, (0, 0, 0, 0)),
    (2, 50, 84, 256, 1024, 1, 1, (0, 0, 0, 0)),
    (2, 50, 84, 64, 64, 3, 1, (1, 1, 1, 1)),
    (2, 100, 167, 64, 256, 1, 1, (0, 0, 0, 0)),
    (2, 25, 42, 512, 512, 3, 2, (1, 1, 1, 1)),
]


def _tensors(N, H, W, cin, cout, k, stride, pads):
    Ho, Wo = NC._out_hw(H, W, k, stride, pads)
    x = torch.zeros(N, H, W, cin, dtype=torch.bfloat16)
    w = torch.zeros(cout, k, k, cin, dtype=torch.bfloat16)
    dy = torch.zeros(N, Ho, Wo, cout, dtype=torch.bfloat16)
    g = NC.geom_single(N, H, W, Ho, Wo, k, stride, pads, cin, cout)
    return x, w, dy, g, (N, Ho, Wo, cout)


@pytest.mark.parametrize("shape", SHAPES)
def test_fwd_only_matches_full(shape):
    x, w, dy, g, oshape = _tensors(*shape)
    stride, pads = shape[6], shape[7]
    full = NC.fwd_candidates(x, w, None, None, g, stride, pads, True, oshape)
    assert full
    for name in full:
        one = NC.fwd_candidates(x, w, None, None, g, stride, pads, True, oshape, only=name)
        assert list(one) == [name], name
    assert NC.fwd_candidates(x, w, None, None, g, stride, pads, True, oshape, only="nope") == {}


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("form", ["plain", "mask", "out"])
def test_dgrad_only_matches_full(shape, form):
    x, w, dy, g, _ = _tensors(*shape)
    stride, pads = shape[6], shape[7]
    kw = {"mask": x} if form == "mask" else ({"out": torch.zeros_like(x)} if form == "out" else {})
    full = NC._dgrad_cands(dy, w, x, stride, pads, **kw)
    for name in full:
        one = NC._dgrad_cands(dy, w, x, stride, pads, only=name, **kw)
        assert list(one) == [name], name


@pytest.mark.parametrize("shape", SHAPES)
def test_wgrad_only_matches_full(shape):
    x, w, dy, g, _ = _tensors(*shape)
    full = NC.wgrad_candidates(x, dy, g, None)
    sink = torch.zeros(w.numel(), dtype=torch.float32)
    make = NC._wgrad_sink_cands(x, dy, g, None, lambda: None)
    full_s = make(sink)
    assert set(full) | {"miopen"} == set(full_s)
    for name in full:
        assert list(NC.wgrad_candidates(x, dy, g, None, only=name)) == [name], name
    for name in full_s:
        assert list(make(sink, name)) == [name], name
