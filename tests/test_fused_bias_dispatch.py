"""CPU: when conv_wgrad.deliver_wgrad_bias_fused takes the fused weight + bias gradient path (the tuned sink
winner is a phase-pipelined variant, both parameters have sinks, cout % 4 == 0, MXR_WGRAD_FUSED_BIAS on)
and that it falls back otherwise.  The kernel itself is covered by tests/test_kernels_gpu.py and the
in-model equality by tests/test_fused_bias_gpu.py."""
import torch

from batchai_retinanet_horovod_coco_amd.ops import conv_wgrad as CW
from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import TUNER
from batchai_retinanet_horovod_coco_amd.ops.native import ConvGeom


class _Sinks:
    def __init__(self, m):
        self.m, self.notified = m, []

    def get(self, p):
        return self.m.get(p)

    def notify(self, p):
        self.notified.append(p)


def _setup(monkeypatch, cout=256, winner="hip23", sinks=True):
    wp, bp = object(), object()
    ws, bs = torch.zeros(cout * 9 * 16), torch.zeros(cout)
    gs = _Sinks({wp: ws, bp: bs} if sinks else {})
    monkeypatch.setattr(CW._n, "grad_sinks", lambda: gs)
    calls = []
    monkeypatch.setattr(CW, "conv_wgrad", lambda *a, **kw: calls.append(kw))
    monkeypatch.delenv("MXR_CONV_FORCE", raising=False)
    monkeypatch.delenv("MXR_CONV_EXCLUDE", raising=False)
    key = "pwgrad|test|%d" % cout
    if winner is not None:
        monkeypatch.setitem(TUNER.table, key + "|s", winner)
    g = ConvGeom()
    g.cout = cout
    return key, g, wp, bp, ws, bs, gs, calls


def test_fused_path_taken(monkeypatch):
    monkeypatch.setenv("MXR_WGRAD_FUSED_BIAS", "1")
    key, g, wp, bp, ws, bs, gs, calls = _setup(monkeypatch)
    assert CW.deliver_wgrad_bias_fused(key, None, None, g, wp, bp)
    assert len(calls) == 1 and calls[0]["variant"] == 23 and calls[0]["out"] is ws
    assert calls[0]["bias_out"] is bs and calls[0]["bias_accumulate"] and calls[0]["accumulate"]
    assert gs.notified == [wp, bp]


def test_fallbacks(monkeypatch):
    for kw, env in [({"winner": "hip11"}, "1"),      # winner is not a phase-pipelined variant
                    ({"winner": "miopen"}, "1"),
                    ({"winner": None}, "1"),         # not tuned yet
                    ({"cout": 36 + 2}, "1"),         # cout % 4
                    ({"sinks": False}, "1"),         # no gradient sinks
                    ({}, "0")]:                      # disabled
        monkeypatch.setenv("MXR_WGRAD_FUSED_BIAS", env)
        key, g, wp, bp, ws, bs, gs, calls = _setup(monkeypatch, **kw)
        assert not CW.deliver_wgrad_bias_fused(key, None, None, g, wp, bp), kw
        assert not calls and not gs.notified


def test_single_geometry_needs_no_scale(monkeypatch):
    x = torch.zeros(1, 4, 4, 8)
    w = torch.zeros(8, 3, 3, 8)
    assert not CW.run_wgrad_bias_fused(x, x, w, 1, (1, 1, 1, 1), torch.ones(8), object(), object())
