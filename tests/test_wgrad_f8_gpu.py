"""FP8 weight gradient of the packed head layers (csrc/kernels/conv_wgrad_p8_f8.hip: e5m2 dY x e4m3 X on the scaled
16x16x128 MFMA) vs fp32 PyTorch references: exact against the dequantised operands (fp32 accumulation), and within
fp8 precision of the unquantised gradient; every head shape class (256 / 720 / 36 outputs over the packed
pyramid), a single level, several splits, accumulation into an existing gradient."""
import pytest
import torch

from batchai_retinanet_horovod_coco_amd.ops import fp8 as F8
from batchai_retinanet_horovod_coco_amd.ops import native as N

pytestmark = pytest.mark.gpu

PYR = [(20, 34), (10, 17), (5, 9), (3, 5), (2, 3)]


def _ref_wgrad(x, dy, shapes, cout):
    """fp32 dW (cout, 3, 3, cin) of a shared 3x3 / pad-1 conv over packed levels: x (n, P, cin), dy (n, P, >= cout)."""
    n, _, cin = x.shape
    dw = torch.zeros(cout, cin, 3, 3, device=x.device)
    o = 0
    for h, w in shapes:
        xl = x[:, o:o + h * w].reshape(n, h, w, cin).permute(0, 3, 1, 2).float()
        gl = dy[:, o:o + h * w, :cout].reshape(n, h, w, cout).permute(0, 3, 1, 2).float()
        dw += torch.nn.grad.conv2d_weight(xl, (cout, cin, 3, 3), gl, padding=1)
        o += h * w
    return dw.permute(0, 2, 3, 1)


@pytest.mark.parametrize("cout,ldy", [(256, 256), (720, 768), (36, 64)])
@pytest.mark.parametrize("splits", [None, 1, 7])
def test_pyramid_wgrad_f8(cuda, cout, ldy, splits):
    torch.manual_seed(0)
    n, cin = 2, 256
    xs = [torch.relu(torch.randn(n, h, w, cin, device=cuda)).bfloat16() for (h, w) in PYR]
    packed, sh = N.pyramid_pack(xs)
    dy = (torch.randn(n, packed.shape[1], ldy, device=cuda) * 1e-3).bfloat16()
    dy[..., cout:] = 0
    g = N.geom_pyramid(n, sh, cin, cout)
    xq, ix = F8.quantize(packed)
    dq, idq = F8.quantize_bf8(dy)
    dw = F8.pyramid_wgrad(xq, ix, dq, idq, g, splits=splits)
    torch.cuda.synchronize()
    # exact kernel arithmetic: the fp32 reference on the dequantised operands
    xd = F8.dequantize(xq, ix).view_as(packed)
    dd = F8.dequantize_bf8(dq, idq).view_as(dy)
    ref_q = _ref_wgrad(xd, dd, sh, cout)
    torch.testing.assert_close(dw, ref_q, rtol=1e-4, atol=1e-4 * ref_q.abs().max().item())
    # and within fp8 precision of the unquantised gradient: with random signs the relative error of the sum is the
    # per-product one, rms ~ 2^-3/sqrt(3) (e5m2 dY) (+) 2^-4/sqrt(3) (e4m3 X) ~ 0.056
    ref = _ref_wgrad(packed, dy, sh, cout)
    rel = ((dw - ref).norm() / ref.norm()).item()
    assert rel < 0.08, rel


@pytest.mark.parametrize("cout,ldy", [(256, 256), (720, 768)])
def test_pyramid_wgrad_f8_fused_bias(cuda, cout, ldy):
    """The BIAS form: the same weight gradient, plus db = inv_dy * sum_m dq[m, :cout] accumulated into the bias
    output -- exact against the dequantised e5m2 dY, and within e5m2 precision of the bf16 column sum."""
    torch.manual_seed(4)
    n, cin = 2, 256
    xs = [torch.relu(torch.randn(n, h, w, cin, device=cuda)).bfloat16() for (h, w) in PYR]
    packed, sh = N.pyramid_pack(xs)
    dy = (torch.randn(n, packed.shape[1], ldy, device=cuda) * 1e-3 + 2e-4).bfloat16()
    dy[..., cout:] = 0
    g = N.geom_pyramid(n, sh, cin, cout)
    xq, ix = F8.quantize(packed)
    dq, idq = F8.quantize_bf8(dy)
    dw0 = F8.pyramid_wgrad(xq, ix, dq, idq, g)
    base = torch.randn(cout, device=cuda)
    db = base.clone()
    dw = F8.pyramid_wgrad(xq, ix, dq, idq, g, bias_out=db, bias_accumulate=True)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw0)                      # the bias sums leave the weight gradient untouched
    dd = F8.dequantize_bf8(dq, idq).view_as(dy)
    ref_q = dd[..., :cout].reshape(-1, cout).sum(0)
    torch.testing.assert_close(db - base, ref_q, rtol=1e-4, atol=1e-4 * ref_q.abs().max().item())
    ref = dy[..., :cout].float().reshape(-1, cout).sum(0)
    rel = ((db - base - ref).norm() / ref.norm()).item()
    assert rel < 0.05, rel
    db2 = torch.empty(cout, device=cuda)
    F8.pyramid_wgrad(xq, ix, dq, idq, g, bias_out=db2)          # plain write
    torch.cuda.synchronize()
    torch.testing.assert_close(db2, db - base, rtol=1e-6, atol=1e-6 * ref_q.abs().max().item())


def test_single_level_wgrad_f8_accumulates(cuda):
    torch.manual_seed(1)
    n, h, w, cin, cout = 2, 25, 42, 256, 256
    x = torch.relu(torch.randn(n, h * w, cin, device=cuda)).bfloat16()
    dy = (torch.randn(n, h * w, cout, device=cuda) * 1e-2).bfloat16()
    g = N.geom_pyramid(n, [(h, w)], cin, cout)
    xq, ix = F8.quantize(x)
    dq, idq = F8.quantize_bf8(dy)
    base = torch.randn(cout, 3, 3, cin, device=cuda)
    out = base.clone()
    F8.pyramid_wgrad(xq, ix, dq, idq, g, out=out, accumulate=True)
    torch.cuda.synchronize()
    ref = _ref_wgrad(F8.dequantize(xq, ix).view_as(x), F8.dequantize_bf8(dq, idq).view_as(dy), [(h, w)], cout)
    torch.testing.assert_close(out - base, ref, rtol=1e-4, atol=1e-4 * ref.abs().max().item())


def test_fp8_step_uses_fp8_wgrad(cuda, monkeypatch):
    """In an fp8 training step the packed head layers' weight gradients come from conv_wgrad_p8_f8 (into the flat
    gradient buffer) and the head gradients match the bf16-wgrad step's within fp8 precision."""
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
    from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_from_synthetic
    from batchai_retinanet_horovod_coco_amd.ops.side_stream import SIDE
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    calls = []
    real = F8.pyramid_wgrad
    monkeypatch.setattr(F8, "pyramid_wgrad", lambda *a, **k: calls.append(1) or real(*a, **k))
    grads, heads = {}, None
    for wg in (True, False):
        monkeypatch.setattr(F8, "WGRAD", wg)
        F8.set_enabled(True)
        F8.reset_state()
        try:
            torch.manual_seed(0)
            model = models.backbone("resnet50").retinanet(80)
            calibrate_from_synthetic(model, torch.device("cpu"), batch=1, height=256, width=320)
            tr = Trainer(model, compute_dtype=torch.bfloat16, clip_mode="global", device=cuda)
            b = make_batch(2, 256, 320, device=cuda, generator=torch.Generator(device=cuda).manual_seed(3))
            for _ in range(2):          # the second pass has the delayed-scaling fp8 copies
                tr.flat.zero_grad()
                tr.forward_backward(b["images"], b["gt"], b["gt_count"], b["image_hw"])
                SIDE.join()
                torch.cuda.synchronize()
            heads = [p for n, p in model.named_parameters()
                     if ("classification" in n or "regression" in n) and p.dim() == 4]
            grads[wg] = torch.cat([p.grad.flatten() for p in heads]).clone()
        finally:
            F8.set_enabled(False)
    # every head layer whose forward runs in fp8 (the 36-output regression final does not: cout % 8), both passes
    n_f8 = sum(F8.eligible(p.shape[-1], p.shape[0]) for p in heads)     # (cout, kh, kw, cin)
    assert n_f8 == len(heads) - 1
    assert len(calls) == 2 * n_f8, (len(calls), n_f8)
    rel = ((grads[True] - grads[False]).norm() / grads[False].norm()).item()
    assert rel < 0.1, rel


def test_fp8_step_bias_from_wgrad(cuda, monkeypatch):
    """In the fp8 step the head layers' bias gradients come out of the fp8 weight-gradient kernel (no bf16 column
    sums for them) and match the column-sum step's within e5m2 precision."""
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
    from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_from_synthetic
    from batchai_retinanet_horovod_coco_amd.ops import conv_wgrad as CW
    from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC
    from batchai_retinanet_horovod_coco_amd.ops.side_stream import SIDE
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    colsums = []
    real = CW.deliver_bias_grad
    monkeypatch.setattr(NC, "deliver_bias_grad", lambda *a, **k: colsums.append(1) or real(*a, **k))
    grads = {}
    for fused in (True, False):
        monkeypatch.setattr(F8, "WGRAD_BIAS", fused)
        F8.set_enabled(True)
        F8.reset_state()
        colsums.clear()
        try:
            torch.manual_seed(0)
            model = models.backbone("resnet50").retinanet(80)
            calibrate_from_synthetic(model, torch.device("cpu"), batch=1, height=256, width=320)
            tr = Trainer(model, compute_dtype=torch.bfloat16, clip_mode="global", device=cuda)
            b = make_batch(2, 256, 320, device=cuda, generator=torch.Generator(device=cuda).manual_seed(3))
            for _ in range(2):
                tr.flat.zero_grad()
                colsums.clear()
                tr.forward_backward(b["images"], b["gt"], b["gt_count"], b["image_hw"])
                SIDE.join()
                torch.cuda.synchronize()
            heads = [p for n, p in model.named_parameters()
                     if ("classification" in n or "regression" in n) and p.dim() == 1]
            grads[fused] = (torch.cat([p.grad.flatten() for p in heads]).clone(), len(colsums))
        finally:
            F8.set_enabled(False)
    # fused: the 9 fp8 head layers (all but the 36-output regression final) drop their column sums; every other
    # layer's bias path is the same in both runs (one process: the same tuned kernels)
    assert grads[False][1] - grads[True][1] == 9, (grads[True][1], grads[False][1])
    rel = ((grads[True][0] - grads[False][0]).norm() / grads[False][0].norm()).item()
    assert rel < 0.1, rel


@pytest.mark.parametrize("bf8", [True, False])
def test_quantize_delayed(cuda, bf8):
    """mxr_quant_delayed: the first call seeds the state with the exact (two-pass) quantisation; later calls use
    the previous call's amax x MARGIN as the scale (one pass) and record their own amax for the next."""
    qmax = F8.BF8_MAX if bf8 else F8.FP8_MAX
    deq = F8.dequantize_bf8 if bf8 else F8.dequantize
    key = ("test_delayed_%d" % bf8, torch.zeros(1))
    torch.manual_seed(2)
    x0 = torch.randn(3, 1000, 48, device=cuda).bfloat16()
    q0, i0 = F8.quantize_delayed(x0, key, bf8=bf8)
    qr, ir = (F8.quantize_bf8 if bf8 else F8.quantize)(x0)
    assert torch.equal(q0, qr) and torch.equal(i0, ir)
    prev = x0.float().abs().max()
    for growth in (1.5, 0.5, 1.0):
        x = (torch.randn(3, 1000, 48, device=cuda) * prev.item() * growth / 4).bfloat16()
        q, inv = F8.quantize_delayed(x, key, bf8=bf8)
        torch.cuda.synchronize()
        assert inv.item() == pytest.approx(F8.MARGIN * prev.item() / qmax, rel=1e-6)
        rel = ((deq(q, inv).view_as(x) - x.float()).norm() / x.float().norm()).item()
        assert rel < (0.1 if bf8 else 0.05), rel
        prev = x.float().abs().max()
        st = F8.amax_state(key, cuda)
        assert st.amax3[(st.phase - 1) % 3].item() == prev.item()



def test_fp8_only_tower_outputs(cuda, monkeypatch):
    """Under fp8 a tower layer whose reader is the next fp8 head layer writes only its e4m3 copy and its relu bitmask
    (no bf16 output): 7 of the 8 tower outputs go fp8-only (not the regression tower's top: the 36-output final is
    bf16), and the step's loss / gradients equal the bf16-output step's bit for bit whenever the step itself
    reproduces bit for bit (two plain runs agree); otherwise within 3x their own difference."""
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
    from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_from_synthetic
    from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC
    from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import TUNER
    from batchai_retinanet_horovod_coco_amd.ops.side_stream import SIDE
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    real = TUNER.winner
    monkeypatch.setattr(TUNER, "winner", lambda k: ("f8_20" if k.startswith("pfwd|") else "f8d_22")
                        if k.endswith("|f8") and k.startswith(("pfwd|", "pdgrad|")) else real(k))
    seen = []
    real_fwd = F8.pyramid_forward

    def spy(*a, **k):
        y = real_fwd(*a, **k)
        seen.append(bool(getattr(y, "_mxr_f8only", False)))
        return y
    monkeypatch.setattr(F8, "pyramid_forward", spy)

    def run(on):
        monkeypatch.setattr(F8, "F8_ONLY_TOWERS", on)
        F8.set_enabled(True)
        F8.reset_state()
        try:
            torch.manual_seed(0)
            model = models.backbone("resnet50").retinanet(80)
            calibrate_from_synthetic(model, torch.device("cpu"), batch=1, height=256, width=320)
            tr = Trainer(model, compute_dtype=torch.bfloat16, clip_mode="global", device=cuda)
            b = make_batch(2, 256, 320, device=cuda, generator=torch.Generator(device=cuda).manual_seed(3))
            for _ in range(3):          # tuning, delayed-scale seeding, steady pass
                seen.clear()
                tr.flat.zero_grad()
                loss = tr.forward_backward(b["images"], b["gt"], b["gt_count"], b["image_hw"])
                SIDE.join()
                torch.cuda.synchronize()
            heads = [p for n, p in model.named_parameters() if "classification" in n or "regression" in n]
            return (torch.cat([p.grad.flatten() for p in heads]).clone(), [float(v) for v in loss], list(seen))
        finally:
            F8.set_enabled(False)
            F8.reset_state()
    off1, off2, on = run(False), run(False), run(True)
    assert sum(on[2]) == 7, on[2]
    assert sum(off1[2]) == 0
    assert torch.isfinite(on[0]).all()

    def rel(a, b):
        return ((a - b).norm() / b.norm()).item()
    noise = rel(off2[0], off1[0])
    if noise == 0.0:             # the step reproduces bit for bit: so must the fp8-only form
        assert torch.equal(on[0], off1[0]) and on[1] == off1[1], (rel(on[0], off1[0]), on[1], off1[1])
    else:
        assert rel(on[0], off1[0]) <= 3 * noise + 1e-3, (rel(on[0], off1[0]), noise)


def test_fp8_only_dgrads(cuda, monkeypatch):
    """Under fp8 a data gradient whose reader is an fp8 tower layer's backward (the dX of an fp8-only tower output)
    writes only its e5m2 copy (conv_hx32_f8's masked NOY data-gradient form): 7 per step, and the step's loss /
    gradients equal the bf16-dX step's bit for bit whenever the step itself reproduces."""
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
    from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_from_synthetic
    from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import TUNER
    from batchai_retinanet_horovod_coco_amd.ops.side_stream import SIDE
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    real = TUNER.winner
    monkeypatch.setattr(TUNER, "winner", lambda k: ("f8_20" if k.startswith("pfwd|") else "f8d_22")
                        if k.endswith("|f8") and k.startswith(("pfwd|", "pdgrad|")) else real(k))
    seen = []
    real_dgrad = F8.pyramid_dgrad

    def spy(*a, **k):
        y = real_dgrad(*a, **k)
        seen.append(bool(getattr(y, "_mxr_f8only", False)))
        return y
    monkeypatch.setattr(F8, "pyramid_dgrad", spy)

    def run(on):
        monkeypatch.setattr(F8, "F8_ONLY_DGRAD", on)
        F8.set_enabled(True)
        F8.reset_state()
        try:
            torch.manual_seed(0)
            model = models.backbone("resnet50").retinanet(80)
            calibrate_from_synthetic(model, torch.device("cpu"), batch=1, height=256, width=320)
            tr = Trainer(model, compute_dtype=torch.bfloat16, clip_mode="global", device=cuda)
            b = make_batch(2, 256, 320, device=cuda, generator=torch.Generator(device=cuda).manual_seed(3))
            for _ in range(3):          # tuning, delayed-scale seeding, steady pass
                seen.clear()
                tr.flat.zero_grad()
                loss = tr.forward_backward(b["images"], b["gt"], b["gt_count"], b["image_hw"])
                SIDE.join()
                torch.cuda.synchronize()
            heads = [p for n, p in model.named_parameters() if "classification" in n or "regression" in n]
            return (torch.cat([p.grad.flatten() for p in heads]).clone(), [float(v) for v in loss], list(seen))
        finally:
            F8.set_enabled(False)
            F8.reset_state()
    off1, off2, on = run(False), run(False), run(True)
    assert sum(on[2]) == 7, on[2]
    assert sum(off1[2]) == 0
    assert torch.isfinite(on[0]).all()

    def rel(a, b):
        return ((a - b).norm() / b.norm()).item()
    noise = rel(off2[0], off1[0])
    if noise == 0.0:
        assert torch.equal(on[0], off1[0]) and on[1] == off1[1], (rel(on[0], off1[0]), on[1], off1[1])
    else:
        assert rel(on[0], off1[0]) <= 3 * noise + 1e-3, (rel(on[0], off1[0]), noise)


def test_fp8_only_dgrad_refuses_bf16_reads(cuda):
    """A layer whose backward would read the bf16 values of an fp8-only data gradient raises (no silent garbage)."""
    from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC
    shapes = ((6, 10), (3, 5))
    x = torch.randn(1, 75, 256, device=cuda).bfloat16().requires_grad_()
    w = torch.randn(256, 3, 3, 256, device=cuda, requires_grad=True)
    y = NC.PyramidConvFn.apply(x, w, None, shapes, False, False, False)
    g = torch.randn_like(y)
    g._mxr_f8only = True
    with pytest.raises(RuntimeError, match="fp8-only"):
        torch.autograd.backward([y], [g])


def test_hx8_weight_quant_batched(cuda):
    """ComputeWeights.hx8_quant: the fp8 head layers' forward and flipped data-gradient weights are requantised by ONE
    batched launch per optimizer step, bit-identical to the per-weight kernel on the current compute weights."""
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
    from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_from_synthetic
    from batchai_retinanet_horovod_coco_amd.ops.side_stream import SIDE
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    F8.set_enabled(True)
    F8.reset_state()
    try:
        torch.manual_seed(0)
        model = models.backbone("resnet50").retinanet(80)
        calibrate_from_synthetic(model, torch.device("cpu"), batch=1, height=256, width=320)
        tr = Trainer(model, lr=1e-3, compute_dtype=torch.bfloat16, clip_mode="global", device=cuda)
        b = make_batch(2, 256, 320, device=cuda, generator=torch.Generator(device=cuda).manual_seed(3))
        for _ in range(3):
            tr.train_on_batch(b["images"], b["gt"], b["gt_count"], b["image_hw"])
        SIDE.join()
        torch.cuda.synchronize()
        cw = N.compute_weights()
        assert cw is not None and len(cw.q8views) >= 9, len(getattr(cw, "q8views", {}))
        src0 = next(iter(cw.q8views.values()))[2]
        cw.hx8_quant(src0)                      # the batch for the current weights (the last step moved them)
        torch.cuda.synchronize()
        assert cw.q8done == cw.plan.generation
        for qp, inv, src in cw.q8views.values():
            rq, ri = F8.quantize_rows_hx8(src.clone())      # not a served weight: the per-weight kernel
            assert torch.equal(qp, rq) and torch.equal(inv, ri)
    finally:
        F8.set_enabled(False)
        F8.reset_state()


def test_fp8_only_output_refuses_bf16_reads(cuda):
    from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC
    from batchai_retinanet_horovod_coco_amd.ops.conv_launch import BitMask
    shapes = ((6, 10), (3, 5))
    x = torch.randn(1, 75, 256, device=cuda).bfloat16()
    x._mxr_f8only = True
    x._mxr_bits = BitMask(x)
    w = torch.randn(256, 3, 3, 256, device=cuda, requires_grad=True)
    with pytest.raises(RuntimeError, match="fp8-only"):
        NC.PyramidConvFn.apply(x, w, None, shapes, True, True, True)      # fp8 off: a bf16 layer would read x


def test_fp8_only_chain_exact(cuda, monkeypatch):
    """Three packed head layers (relu, relu, final) under fp8 with the hx8 kernels pinned: with the tower outputs
    fp8-only (e4m3 copy + bitmask, no bf16 store, out_f8) every gradient is bit-identical to the bf16-output run."""
    from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC
    from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import TUNER
    real = TUNER.winner
    monkeypatch.setattr(TUNER, "winner", lambda k: ("f8_20" if k.startswith("pfwd|") else "f8d_22")
                        if k.endswith("|f8") and k.startswith(("pfwd|", "pdgrad|")) else real(k))
    shapes = ((20, 34), (10, 17), (5, 9), (3, 5), (2, 3))
    n, c = 2, 256
    P = sum(h * w for h, w in shapes)
    torch.manual_seed(4)
    ws = [(torch.randn(c, 3, 3, c, device=cuda) / 48).requires_grad_() for _ in range(3)]
    bs = [(torch.randn(c, device=cuda) * 0.1).requires_grad_() for _ in range(3)]
    x0 = torch.randn(n, P, c, device=cuda).bfloat16()
    gy = (torch.randn(n, P, c, device=cuda) * 1e-2).bfloat16()
    flags = []

    def run(on):
        monkeypatch.setattr(F8, "F8_ONLY_TOWERS", on)
        flags.clear()
        x = x0.clone().requires_grad_()
        h = x
        for i in range(3):
            h = NC.PyramidConvFn.apply(h, ws[i], bs[i], shapes, i < 2, i > 0, i < 2, None, None, i < 2)
            flags.append(bool(getattr(h, "_mxr_f8only", False)))
        h.backward(gy)
        torch.cuda.synchronize()
        out = [x.grad.clone()] + [t.grad.clone() for t in ws + bs]
        for t in ws + bs:
            t.grad = None
        return out
    F8.set_enabled(True)
    F8.reset_state()
    try:
        for _ in range(3):          # tuning, delayed-scale seeding, steady
            ref = run(False)
        F8.reset_state()
        for _ in range(3):
            got = run(True)
    finally:
        F8.set_enabled(False)
        F8.reset_state()
    assert flags == [True, True, False], flags
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
