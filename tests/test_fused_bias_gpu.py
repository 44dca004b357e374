"""In-model fused weight + bias gradient of the pyramid convs (conv_wgrad.deliver_wgrad_bias_fused): once the
tuned sink winner of a head wgrad is a phase-pipelined variant, the bias gradient comes out of the same
kernel instead of a separate colsum pass.  The flat gradients after one step must match the unfused step
(MXR_WGRAD_FUSED_BIAS=0) to run-to-run noise, and the fused path must actually have run."""
import pytest
import torch

from test_side_stream_gpu import _grads

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("comm", ["torch"])
def test_fused_bias_matches_unfused(cuda, monkeypatch, comm):
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.ops import conv_wgrad, native_conv
    from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import TUNER
    torch.manual_seed(0)
    state = {k: v.clone() for k, v in models.backbone("resnet18").retinanet(8).state_dict().items()}
    _grads(cuda, monkeypatch, comm, True, state)          # first sight: the tuner races every key
    for k in list(TUNER.table):
        if (k.startswith("pwgrad") or k.startswith("wgrad")) and k.endswith("|s"):
            monkeypatch.setitem(TUNER.table, k, "hip23")   # every wgrad on the phase-pipelined kernel
    hits, fpn_hits = [], []

    def counting(real, out):
        def f(*a, **kw):
            r = real(*a, **kw)
            out.append(r)
            return r
        return f

    # pyramid convs (native_conv) and single-geometry biased convs (run_wgrad_bias_fused -> conv_wgrad's)
    monkeypatch.setattr(native_conv, "deliver_wgrad_bias_fused",
                        counting(native_conv.deliver_wgrad_bias_fused, hits))
    monkeypatch.setattr(conv_wgrad, "deliver_wgrad_bias_fused",
                        counting(conv_wgrad.deliver_wgrad_bias_fused, fpn_hits))
    monkeypatch.setenv("MXR_WGRAD_FUSED_BIAS", "0")
    g_a, _, segs = _grads(cuda, monkeypatch, comm, True, state)
    g_b, _, _ = _grads(cuda, monkeypatch, comm, True, state)
    assert not any(hits) and not any(fpn_hits)
    monkeypatch.setenv("MXR_WGRAD_FUSED_BIAS", "1")
    hits.clear()
    fpn_hits.clear()
    g_c, _, _ = _grads(cuda, monkeypatch, comm, True, state)
    # tower convs (2 x 4) + the two finals (cout 8 x 9 = 72, and 36 over its zero-padded 64-wide dY rows)
    assert sum(hits) >= 10, hits
    # FPN: 3 lateral 1x1 + 3 smoothing 3x3 + P6 / P7 (every biased unscaled conv outside the heads)
    assert sum(fpn_hits) >= 8, fpn_hits

    def seg_err(a, b):
        return [float((a[o:o + n] - b[o:o + n]).abs().max() / b[o:o + n].abs().max().clamp_min(1e-12))
                for o, n in segs]

    noise, err = seg_err(g_b, g_a), seg_err(g_c, g_a)
    worst = max(range(len(err)), key=lambda i: err[i])
    assert err[worst] <= max(4 * noise[worst], 1e-2), (worst, err[worst], noise[worst])
