"""The evaluation transform against PIL itself (PIL is importable offline).

Reference: ``evaluation_pipeline.py:89`` resizes the uint8 PIL image with
``Image.resize((WIDTH, HEIGHT))`` (BICUBIC, antialiased), then ``ToTensor`` and
``Normalize`` (``:116-122``).  ``data/pil_resize.py`` must reproduce PIL's uint8 output bit
for bit, and preprocess mode 1 (the host oracle of the GPU kernels) must equal
PIL -> ToTensor -> Normalize exactly in float32."""
import numpy as np
import pytest
import torch
from PIL import Image

from mpi_pytorch_amd.data import pil_resize
from mpi_pytorch_amd.ops import ref

MEAN, STD = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
SIZES = [((256, 256), (128, 128)), ((677, 1000), (128, 128)), ((100, 80), (128, 128)),
         ((300, 301), (299, 299)), ((64, 64), (64, 64)), ((999, 523), (224, 224)),
         ((50, 400), (37, 91)), ((7, 5), (128, 128)), ((128, 700), (128, 128)),
         ((1000, 664), (299, 299))]


def _pil(img, out_hw):
    return np.asarray(Image.fromarray(img).resize((out_hw[1], out_hw[0]), Image.BICUBIC))


@pytest.mark.parametrize("src,dst", SIZES)
def test_resize_u8_bit_exact(src, dst):
    rng = np.random.default_rng(src[0] * 7 + dst[1])
    img = rng.integers(0, 256, (src[0], src[1], 3), dtype=np.uint8)
    assert np.array_equal(pil_resize.resize_u8(img, dst), _pil(img, dst))


def test_resize_u8_smooth_image_bit_exact():
    """Natural-image-like content (gradients + edges), where rounding ties are common."""
    y, x = np.mgrid[0:480, 0:640]
    img = np.stack([(x * 255 // 639), (y * 255 // 479), ((x // 40 + y // 40) % 2) * 255],
                   -1).astype(np.uint8)
    for dst in ((128, 128), (224, 224), (299, 299), (500, 700)):
        assert np.array_equal(pil_resize.resize_u8(img, dst), _pil(img, dst))


def _torchvision_eval(img_u8, dst):
    """PIL resize -> ToTensor (u8 / 255) -> Normalize (sub mean, div std), float32."""
    t = torch.from_numpy(_pil(img_u8, dst).copy()).float().div(255)
    m = torch.tensor(MEAN, dtype=torch.float32)
    s = torch.tensor(STD, dtype=torch.float32)
    return t.sub(m).div(s)


@pytest.mark.parametrize("src,dst", SIZES[:6])
def test_eval_transform_matches_pil_pipeline(src, dst):
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (2, src[0], src[1], 3), dtype=np.uint8)
    got = ref.preprocess(torch.from_numpy(img), dst[0], dst[1], MEAN, STD, 1, 3, torch.float32)
    exp = torch.stack([_torchvision_eval(img[b], dst) for b in range(2)])
    assert torch.equal(got, exp)


def test_eval_transform_with_extents():
    """Images of different sizes in one padded slot: each is resized from its own extent."""
    rng = np.random.default_rng(2)
    ext = np.array([[300, 200], [256, 256], [97, 311]])
    slot = np.zeros((3, 320, 320, 3), dtype=np.uint8)
    imgs = []
    for b, (h, w) in enumerate(ext):
        im = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        slot[b, :h, :w] = im
        imgs.append(im)
    got = ref.preprocess(torch.from_numpy(slot), 64, 64, MEAN, STD, 1, 3, torch.float32,
                         extents=ext)
    exp = torch.stack([_torchvision_eval(im, (64, 64)) for im in imgs])
    assert torch.equal(got, exp)


def test_float_bicubic_is_not_pil():
    """Why mode 1 is the fixed-point path: the float antialiased bicubic (torch
    F.interpolate, the round-2 mode 1, now mode 2) differs from PIL's uint8 result."""
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (1, 256, 256, 3), dtype=np.uint8)
    pil = ref.preprocess(torch.from_numpy(img), 128, 128, MEAN, STD, 1, 3, torch.float32)
    flt = ref.preprocess(torch.from_numpy(img), 128, 128, MEAN, STD, 2, 3, torch.float32)
    # every value differs (u8 quantisation of the PIL result), by up to ~4/255 of intensity
    # on noise: same filter, different arithmetic
    assert float((pil != flt).float().mean()) > 0.5
    assert float((pil - flt).abs().max()) < 0.1
