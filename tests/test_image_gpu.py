"""Device image preprocessing (csrc/kernels/image.hip) vs the host C++ path (csrc/cpu/runtime_cpu.cpp)."""
import numpy as np
import pytest
import torch

from batchai_retinanet_horovod_coco_amd.data import image as I
from batchai_retinanet_horovod_coco_amd.ops import native as N
from batchai_retinanet_horovod_coco_amd.utils import cpu_native

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fill_mode", ["constant", "nearest", "reflect", "wrap"])
@pytest.mark.parametrize("interpolation", ["linear", "nearest"])
def test_warp_normalize_matches_host(cuda, fill_mode, interpolation):
    rng = np.random.RandomState(0)
    img = rng.randint(0, 256, (37, 53, 3)).astype(np.uint8)
    th = np.deg2rad(7.0)
    M = np.array([[1.1 * np.cos(th), -np.sin(th), 3.5], [np.sin(th), 0.9 * np.cos(th), -2.25], [0, 0, 1]])
    params = I.TransformParameters(fill_mode=fill_mode, interpolation=interpolation, cval=-5.0)
    ref = I.apply_transform(M, I.preprocess_image(img), params)
    got = N.image_warp_normalize(torch.from_numpy(img).to(cuda), M, None, cpu_native.INTERP[interpolation],
                                 cpu_native.BORDER[fill_mode], -5.0, 1.0, I.CAFFE_MEAN_BGR)
    torch.testing.assert_close(got.cpu(), torch.from_numpy(ref), atol=1e-3, rtol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_resize_into_matches_host(cuda, dtype):
    rng = np.random.RandomState(1)
    src = (rng.rand(31, 47, 3) * 200 - 100).astype(np.float32)
    ref = cpu_native.resize_bilinear(src, 64, 97)
    batch = torch.zeros((2, 70, 100, 3), dtype=dtype, device=cuda)
    N.image_resize_into(torch.from_numpy(src).to(cuda), batch, 1, (64, 97))
    got = batch[1, :64, :97].float().cpu()
    tol = dict(atol=1e-3, rtol=1e-5) if dtype == torch.float32 else dict(atol=0.5, rtol=1e-2)
    torch.testing.assert_close(got, torch.from_numpy(ref), **tol)
    assert float(batch[0].abs().max()) == 0.0 and float(batch[1, 64:].abs().max()) == 0.0
    assert float(batch[1, :, 97:].abs().max()) == 0.0


def test_generator_device_path_matches_host(cuda):
    from batchai_retinanet_horovod_coco_amd.data.synthetic import SyntheticGenerator
    from batchai_retinanet_horovod_coco_amd.data.transform import random_transform_generator

    def make():
        tg = random_transform_generator(min_rotation=-0.1, max_rotation=0.1, min_translation=(-0.1, -0.1),
                                        max_translation=(0.1, 0.1), min_scaling=(0.9, 0.9), max_scaling=(1.1, 1.1),
                                        flip_x_chance=0.5, prng=np.random.RandomState(3))
        return SyntheticGenerator(num_images=3, height=120, width=90, num_classes=4, max_boxes=3, data_seed=5,
                                  transform_generator=tg, batch_size=2, image_min_side=96, image_max_side=160,
                                  shuffle_groups=False)

    host, dev = make(), make()
    assert dev.enable_device_preprocess(cuda)
    for _ in range(2):
        a, b = host.next(), dev.next()
        assert b["images"].is_cuda
        torch.testing.assert_close(b["images"].cpu(), a["images"], atol=2e-3, rtol=1e-5)
        for k in ("gt", "gt_count", "image_hw"):
            assert torch.equal(a[k], b[k]), k
