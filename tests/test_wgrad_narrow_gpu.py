"""64-channel 3x3 weight-gradient kernel (csrc/kernels/wgrad_narrow.hip) vs the fp32 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(2, 37, 150), (1, 4, 64), (3, 9, 70)])
def test_wgrad3x3_c64(cuda, shape):
    n, h, w = shape
    torch.manual_seed(0)
    x = torch.randn(n, h, w, 64, device=cuda).to(torch.bfloat16)
    dy = torch.randn(n, h, w, 64, device=cuda).to(torch.bfloat16)
    scale = torch.rand(64, device=cuda) + 0.5
    dw = NC.wgrad3x3_c64(x, dy, scale)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (64, 64, 3, 3), dy.float().permute(0, 3, 1, 2),
                                      padding=1)
    ref = ref.permute(0, 2, 3, 1) * scale.view(-1, 1, 1, 1)
    rel = (dw - ref).norm() / ref.norm()
    assert rel < 1e-3, rel.item()
    acc = NC.wgrad3x3_c64(x, dy, scale, out=dw.clone(), accumulate=True)
    torch.testing.assert_close(acc, 2 * dw, rtol=1e-5, atol=1e-4)
    g = NC.geom_single(n, h, w, h, w, 3, 1, (1, 1, 1, 1), 64, 64)
    assert NC.w64_covers(g) and "w64" in NC.wgrad_candidates(x, dy, g, scale)
