"""The classification final with the sigmoid-focal loss fused into its forward epilogue (conv_hx32.hip FOC form,
ops.conv_launch.FocalRequest): against the same step with the logits written and the loss kernel run
(losses.hip), the padded gradient rows and every parameter gradient are bit-identical (the epilogue runs the
loss kernel's per-element code, focal_common.h) and the loss agrees to float-summation order."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant", ["hx32_0", "hx32_10"])
def test_focal_fused_step_matches(cuda, monkeypatch, variant):
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
    from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_from_synthetic
    from batchai_retinanet_horovod_coco_amd.ops import conv_launch as CL
    from batchai_retinanet_horovod_coco_amd.ops import native
    from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import TUNER
    from batchai_retinanet_horovod_coco_amd.ops.side_stream import SIDE
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    real = TUNER.winner
    # the classification final's forward on conv_hx32 variant 0 or its 16x16x32 form 10 (the tuned winners)
    monkeypatch.setattr(TUNER, "winner", lambda k: variant if (k.startswith("pfwd|") and k.endswith("|720|0"))
                        else real(k))
    calls = []
    real_launch = CL.launch_hx32_focal
    monkeypatch.setattr(CL, "launch_hx32_focal", lambda *a, **k: calls.append(1) or real_launch(*a, **k))

    def run(fused):
        monkeypatch.setattr(CL, "FOCAL_FUSED", fused)
        torch.manual_seed(0)
        model = models.backbone("resnet50").retinanet(80)
        calibrate_from_synthetic(model, torch.device("cpu"), batch=1, height=256, width=320)
        tr = Trainer(model, compute_dtype=torch.bfloat16, clip_mode="global", device=cuda)
        b = make_batch(2, 256, 320, device=cuda, generator=torch.Generator(device=cuda).manual_seed(3))
        for _ in range(2):
            tr.flat.zero_grad()
            loss = tr.forward_backward(b["images"], b["gt"], b["gt_count"], b["image_hw"])
            SIDE.join()
            torch.cuda.synchronize()
        g = torch.cat([p.grad.flatten() for p in model.parameters() if p.grad is not None]).clone()
        return g, [float(v) for v in loss]
    off1, off2 = run(False), run(False)
    n0 = len(calls)
    on = run(True)
    assert n0 == 0 and len(calls) >= 1, (n0, len(calls))
    assert on[1][0] == off1[1][0]                                   # the regression loss is untouched
    assert abs(on[1][1] - off1[1][1]) <= 1e-5 * abs(off1[1][1]), (on[1], off1[1])
    assert torch.isfinite(on[0]).all()
    if torch.equal(off1[0], off2[0]):      # the step reproduces bit for bit: so must the fused form
        assert torch.equal(on[0], off1[0])
    else:
        assert ((on[0] - off1[0]).norm() / off1[0].norm()).item() <= 3 * ((off2[0] - off1[0]).norm()
                                                                          / off1[0].norm()).item() + 1e-6
    assert native.available()


@pytest.mark.parametrize("variant", [0, 10])
def test_focal_fused_kernel_matches_loss_kernel(cuda, variant):
    """Kernel level: the fused form's padded gradient rows equal the loss kernel's on the logits the plain
    forward of the same tiles writes (variant 0, or 10 on the 16x16x32 MFMA), and the loss agrees."""
    from batchai_retinanet_horovod_coco_amd.ops import conv_launch as CL
    from batchai_retinanet_horovod_coco_amd.ops import native as N
    torch.manual_seed(1)
    shapes = ((20, 34), (10, 17), (5, 9), (3, 5), (2, 3))
    n, cin, A, C = 2, 256, 9, 80
    P = sum(h * w for h, w in shapes)
    x = torch.relu(torch.randn(n, P, cin, device=cuda)).bfloat16()
    w = (torch.randn(A * C, 3, 3, cin, device=cuda) / 48).bfloat16()
    b = torch.full((A * C,), -4.595, device=cuda)          # the prior-probability bias of the final
    g = N.geom_pyramid(n, shapes, cin, A * C)
    rows = n * P * A
    state = torch.randint(-1, 2, (rows,), device=cuda, dtype=torch.int8)
    label = torch.randint(0, C, (rows,), device=cuda, dtype=torch.int32)
    npos = (state == 1).sum().to(torch.int32).reshape(1)
    y = torch.empty(n, P, A * C, device=cuda, dtype=torch.bfloat16)
    N.launch_fwd(x, w, b, None, y, g, False, variant="hx32_%d" % variant)
    ref_loss, ref_pad = N.focal_fwd_bwd(y.view(n, P * A, C), state, label, npos,
                                        grad_out=torch.zeros(n, P, 768, device=cuda, dtype=torch.bfloat16), group=A)
    req = CL.FocalRequest()
    req.set(state, label, npos, A)
    dpad = CL.launch_hx32_focal(x, w, b, g, req, 768, variant=variant)
    torch.cuda.synchronize()
    assert torch.equal(dpad, ref_pad)
    assert abs(req.loss.item() - ref_loss.item()) <= 1e-5 * abs(ref_loss.item())


def test_focal_fused_fp8_step_matches(cuda, monkeypatch):
    """fp8 heads: the classification final on conv_hx32_f8's FOCAL form against the same fp8 step with its logits
    written and the loss kernel run."""
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
    from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_from_synthetic
    from batchai_retinanet_horovod_coco_amd.ops import conv_launch as CL
    from batchai_retinanet_horovod_coco_amd.ops import fp8 as F8
    from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import TUNER
    from batchai_retinanet_horovod_coco_amd.ops.side_stream import SIDE
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    real = TUNER.winner
    monkeypatch.setattr(TUNER, "winner", lambda k: ("f8_20" if k.startswith("pfwd|") else "f8d_22")
                        if k.endswith("|f8") and k.startswith(("pfwd|", "pdgrad|")) else real(k))
    calls = []
    real_ff = F8._focal_forward
    monkeypatch.setattr(F8, "_focal_forward", lambda *a, **k: calls.append(1) or real_ff(*a, **k))

    monkeypatch.setattr(F8, "FOCAL_DQ", False)      # bf16 rows: the bit-identical comparison (test_focal_dq_fp8_step)

    def run(fused):
        monkeypatch.setattr(CL, "FOCAL_FUSED", fused)
        F8.set_enabled(True)
        F8.reset_state()
        try:
            torch.manual_seed(0)
            model = models.backbone("resnet50").retinanet(80)
            calibrate_from_synthetic(model, torch.device("cpu"), batch=1, height=256, width=320)
            tr = Trainer(model, compute_dtype=torch.bfloat16, clip_mode="global", device=cuda)
            b = make_batch(2, 256, 320, device=cuda, generator=torch.Generator(device=cuda).manual_seed(3))
            for _ in range(3):
                tr.flat.zero_grad()
                loss = tr.forward_backward(b["images"], b["gt"], b["gt_count"], b["image_hw"])
                SIDE.join()
                torch.cuda.synchronize()
            g = torch.cat([p.grad.flatten() for p in model.parameters() if p.grad is not None]).clone()
            return g, [float(v) for v in loss]
        finally:
            F8.set_enabled(False)
            F8.reset_state()
    off1, off2 = run(False), run(False)
    n0 = len(calls)
    on = run(True)
    assert n0 == 0 and len(calls) >= 1, (n0, len(calls))
    assert torch.isfinite(on[0]).all()
    assert abs(on[1][1] - off1[1][1]) <= 1e-5 * abs(off1[1][1]) + 3 * abs(off2[1][1] - off1[1][1]), (on[1], off1[1])
    if torch.equal(off1[0], off2[0]):
        assert torch.equal(on[0], off1[0])
    else:
        assert ((on[0] - off1[0]).norm() / off1[0].norm()).item() <= 3 * ((off2[0] - off1[0]).norm()
                                                                          / off1[0].norm()).item() + 1e-6


def test_focal_dq_fp8_step(cuda, monkeypatch):
    """fp8 heads: the FOCAL form writing the gradient rows as their e5m2 copy only (FOCAL_DQ; delayed scale shared with
    the backward's quantisation state) against the bf16 rows + quantisation pass: the same loss, head gradients within
    the double-rounding difference, and the copy path taken after the first pass.  (fp32 -> e5m2 directly vs
    fp32 -> bf16 -> e5m2: ~2^-9 / 2^-3 = 1/64 of the values land one e5m2 step (25 %) apart, an rms of ~3 % that
    sums with random signs keep -- the same order as the e5m2 error itself, test_wgrad_f8_gpu.py.)"""
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
    from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_from_synthetic
    from batchai_retinanet_horovod_coco_amd.ops import fp8 as F8
    from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import TUNER
    from batchai_retinanet_horovod_coco_amd.ops.side_stream import SIDE
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    real = TUNER.winner
    monkeypatch.setattr(TUNER, "winner", lambda k: ("f8_20" if k.startswith("pfwd|") else "f8d_22")
                        if k.endswith("|f8") and k.startswith(("pfwd|", "pdgrad|")) else real(k))
    seen = []
    real_ff = F8._focal_forward

    def spy(*a, **k):
        y = real_ff(*a, **k)
        seen.append(bool(getattr(y._mxr_focal_dpad, "_mxr_f8only", False)))
        return y
    monkeypatch.setattr(F8, "_focal_forward", spy)

    def run(dq):
        monkeypatch.setattr(F8, "FOCAL_DQ", dq)
        F8.set_enabled(True)
        F8.reset_state()
        seen.clear()
        try:
            torch.manual_seed(0)
            model = models.backbone("resnet50").retinanet(80)
            calibrate_from_synthetic(model, torch.device("cpu"), batch=1, height=256, width=320)
            tr = Trainer(model, compute_dtype=torch.bfloat16, clip_mode="global", device=cuda)
            b = make_batch(2, 256, 320, device=cuda, generator=torch.Generator(device=cuda).manual_seed(3))
            for _ in range(3):
                tr.flat.zero_grad()
                loss = tr.forward_backward(b["images"], b["gt"], b["gt_count"], b["image_hw"])
                SIDE.join()
                torch.cuda.synchronize()
            heads = [p for n, p in model.named_parameters() if "classification" in n]
            return torch.cat([p.grad.flatten() for p in heads]).clone(), [float(v) for v in loss], list(seen)
        finally:
            F8.set_enabled(False)
            F8.reset_state()
    off, on = run(False), run(True)
    assert on[2] == [False, True, True] and not any(off[2]), (on[2], off[2])
    assert on[1] == off[1], (on[1], off[1])
    assert torch.isfinite(on[0]).all()
    rel = ((on[0] - off[0]).norm() / off[0].norm()).item()
    assert rel < 0.06, rel
