"""GPU preprocess kernels against their host oracles (ops/ref.py).

* mode 1 (eval transform, ``evaluation_pipeline.py:89,116-122``): the PIL-exact fixed-point
  kernels must give the bf16 rounding of the float32 oracle EXACTLY (the oracle itself is
  bit-exact with PIL, tests/test_pil_parity_cpu.py), uniform and mixed-size batches;
* mode 0 (train transform, ``main.py:62-65``) with per-image extents: a padded slot of
  images of different sizes, one launch, each image resized from its own extent."""
import numpy as np
import pytest
import torch

from mpi_pytorch_amd.ops import functional as Fn
from mpi_pytorch_amd.ops import ref

pytestmark = pytest.mark.gpu
MEAN, STD = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)


@pytest.mark.parametrize("src,dst", [((256, 256), (128, 128)), ((677, 1000), (128, 128)),
                                     ((100, 80), (128, 128)), ((300, 301), (299, 299)),
                                     ((64, 64), (64, 64)), ((50, 400), (37, 91))])
@pytest.mark.parametrize("cpad,pad", [(3, None), (8, None), (4, (3, 3, 3, 3))])
def test_pil_kernel_bitwise(gpu, src, dst, cpad, pad):
    g = torch.Generator().manual_seed(src[0] + dst[1])
    img = torch.randint(0, 256, (3, src[0], src[1], 3), generator=g, dtype=torch.uint8)
    out = Fn.preprocess(img.to(gpu), dst, MEAN, STD, 1, cpad, pad=pad)
    exp = ref.preprocess(img, dst[0], dst[1], MEAN, STD, 1, cpad, torch.float32, pad)
    assert out.dtype == torch.bfloat16 and out.shape == exp.shape
    assert torch.equal(out.cpu(), exp.to(torch.bfloat16))


def test_pil_kernel_mixed_extents(gpu):
    rng = np.random.default_rng(0)
    ext = np.array([[300, 200], [256, 256], [97, 311], [320, 320], [8, 9]])
    slot = rng.integers(0, 256, (5, 320, 320, 3), dtype=np.uint8)  # garbage outside extents
    img = torch.from_numpy(slot)
    out = Fn.preprocess(img.to(gpu), (64, 64), MEAN, STD, 1, 4, extents=ext)
    exp = ref.preprocess(img, 64, 64, MEAN, STD, 1, 4, torch.float32, extents=ext)
    assert torch.equal(out.cpu(), exp.to(torch.bfloat16))


def test_bilinear_mixed_extents(gpu):
    rng = np.random.default_rng(1)
    ext = np.array([[224, 224], [180, 300], [97, 311], [320, 320]])
    slot = rng.integers(0, 256, (4, 320, 320, 3), dtype=np.uint8)
    img = torch.from_numpy(slot)
    out = Fn.preprocess(img.to(gpu), (128, 128), MEAN, STD, 0, 8, extents=ext)
    exp = ref.preprocess(img, 128, 128, MEAN, STD, 0, 8, torch.float32, extents=ext)
    assert out.shape == exp.shape
    assert float((out.float().cpu() - exp).abs().max()) < 0.05
    # each image depends on its own pixels only: changing outside the extents changes nothing
    slot2 = slot.copy()
    for b, (h, w) in enumerate(ext):
        slot2[b, h:] = 0
        slot2[b, :, w:] = 0
    out2 = Fn.preprocess(torch.from_numpy(slot2).to(gpu), (128, 128), MEAN, STD, 0, 8,
                         extents=ext)
    assert torch.equal(out, out2)


def test_extents_outside_pitch_rejected(gpu):
    img = torch.zeros(2, 32, 32, 3, dtype=torch.uint8, device=gpu)
    with pytest.raises(ValueError):
        Fn.preprocess(img, (16, 16), MEAN, STD, 1, 3, extents=[[32, 32], [33, 10]])
    with pytest.raises(ValueError):
        Fn.preprocess(img, (16, 16), MEAN, STD, 0, 3, extents=[[32, 32]])
