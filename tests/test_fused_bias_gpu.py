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


@pytest.mark.parametrize("winner", ["hip23"])
@pytest.mark.parametrize("cout,ldy", [(256, 256), (720, 768)])
def test_fused_delivery_matches_fp32(cuda, monkeypatch, winner, cout, ldy):
    """deliver_wgrad_bias_fused (the in-model path of the head convs) against an fp32 PyTorch autograd
    reference of the same conv: weight AND bias gradients accumulated into their gradient-sink slots (flat
    fp32 buffer views), on the fused kernel (conv_wgrad_p8 BIAS)."""
    import torch.nn.functional as F
    from batchai_retinanet_horovod_coco_amd.ops import conv_wgrad, native as N
    from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import TUNER
    from batchai_retinanet_horovod_coco_amd.ops.side_stream import SIDE
    torch.manual_seed(9)
    shapes = [(20, 34), (10, 17), (5, 9), (3, 5), (2, 3)]
    n, cin = 2, 256
    xs = [torch.randn(n, h, w, cin, device=cuda).bfloat16() for (h, w) in shapes]
    packed, sh = N.pyramid_pack(xs)
    dy = torch.randn(n, packed.shape[1], ldy, device=cuda).bfloat16()
    dy[..., cout:] = 0
    g = N.geom_pyramid(n, sh, cin, cout)
    wparam = torch.nn.Parameter(torch.zeros(cout, 3, 3, cin, device=cuda))
    bparam = torch.nn.Parameter(torch.zeros(cout, device=cuda))
    w0, b0 = torch.randn(cout, 3, 3, cin, device=cuda), torch.randn(cout, device=cuda)
    sinks = {id(wparam): w0.clone(), id(bparam): b0.clone()}
    notified = []

    class Sinks:
        def get(self, p):
            return sinks.get(id(p))

        def notify(self, p):
            notified.append(id(p))

    key = "pwgrad|test|%d|%d" % (cout, ldy)
    monkeypatch.setitem(TUNER.table, key + "|s", winner)
    N.set_grad_sinks(Sinks())
    try:
        assert conv_wgrad.deliver_wgrad_bias_fused(key, packed, dy, g, wparam, bparam)
        SIDE.join()
        torch.cuda.synchronize()
    finally:
        N.set_grad_sinks(None)
    assert sorted(notified) == sorted([id(wparam), id(bparam)])
    # fp32 reference: autograd of the fp32 conv per level, summed over the pyramid
    wr = torch.zeros(cout, cin, 3, 3, device=cuda, requires_grad=True)
    br = torch.zeros(cout, device=cuda, requires_grad=True)
    off = 0
    for x, (h, w) in zip(xs, sh):
        y = F.conv2d(x.float().permute(0, 3, 1, 2), wr, br, padding=1)
        y.backward(dy[:, off:off + h * w, :cout].float().reshape(n, h, w, cout).permute(0, 3, 1, 2))
        off += h * w
    dw = sinks[id(wparam)].view(cout, 3, 3, cin) - w0
    db = sinks[id(bparam)] - b0
    ref_w = wr.grad.permute(0, 2, 3, 1)
    assert float((dw - ref_w).abs().max() / ref_w.abs().max()) < 1e-2
    assert float((db - br.grad).abs().max() / br.grad.abs().max()) < 1e-4
