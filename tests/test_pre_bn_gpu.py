"""BN in the operand path (``Fn.BNLink.want_pre``): a ResNet block's bn1 + ReLU applied by
conv2's halo forward and weight-gradient kernels while they stage conv1's raw output z1, so
y1 = relu(bn1(z1)) is never written (reference: the torchvision BasicBlock reached from
``/root/reference/models.py:33``).

* kernel level: conv_fwd / conv_wgrad with ``pre`` == the same op on the materialized
  operand ``affine_act(z, pre)``, BITWISE (the staged operand is the same bf16 values, the
  MFMA order unchanged), including image borders (padding must stay zero, not relu(shift));
  shapes the halo kernels cannot take fall back to materializing, also bitwise;
* against the fp32 oracle (``ops/ref.py``);
* block level: ResNet-18 blocks with the operand BN on == off, bitwise, in deterministic
  mode (forward output, input and parameter gradients; running stats to 1 ulp).
"""
import math

import pytest
import torch

from mpi_pytorch_amd.ops import ref

pytestmark = pytest.mark.gpu


def C():
    from mpi_pytorch_amd.ops import _ext
    return _ext.ext()


def rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).abs().max() / (b.abs().max() + 1e-6))


def _operands(N, H, W, Cc, K, gpu, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    z = (torch.randn(N, H, W, Cc, generator=g) * 1.5).to(gpu, torch.bfloat16)
    sc = (torch.rand(Cc, generator=g) + 0.5)
    # half the channels with a large positive shift: relu(0 * sc + sh) = sh != 0, so a
    # transformed padding pixel would show at every border output
    sh = torch.where(torch.arange(Cc) % 2 == 0, torch.rand(Cc, generator=g) + 0.5,
                     torch.randn(Cc, generator=g) * 0.3)
    aff = torch.stack([sc, sh]).to(gpu).contiguous()
    w = (torch.randn(K, 3, 3, Cc, generator=g) / math.sqrt(9 * Cc)).to(gpu, torch.bfloat16)
    dy = torch.randn(N, H, W, K, generator=g).to(gpu, torch.bfloat16)
    return z, aff, w, dy


PRE_CASES = [
    # N, H, W, C, K (3x3 / stride 1 / pad 1)
    (2, 56, 56, 64, 64),     # layer1: resident weights
    (25, 56, 56, 64, 64),    # layer1, many tiles per block
    (3, 28, 28, 128, 128),   # layer2: streamed weights, two column tiles
    (5, 14, 14, 256, 256),   # layer3: tiles across image borders
    (7, 7, 7, 512, 512),     # layer4: separator slots
    (3, 9, 11, 96, 128),     # odd W, three channel chunks, partial last tile
    (2, 35, 35, 64, 128),    # wgrad pitch 48
    (2, 12, 12, 64, 32),     # N = 32: forward falls back to materializing
    (2, 17, 17, 32, 64),     # 32-channel wgrad partition (second chunk empty)
    (2, 40, 70, 32, 64),     # ONECH wgrad; forward on strip tiles -> materialized
]


@pytest.mark.parametrize("case", PRE_CASES)
def test_conv_fwd_pre_bitwise(gpu, case):
    N, H, W, Cc, K = case
    z, aff, w, _ = _operands(N, H, W, Cc, K, gpu, 31)
    e = torch.empty(0, device=gpu)
    shift = torch.randn(K, device=gpu) * 0.1
    x = C().affine_act(z, aff, True)
    assert rel(x, ref.affine_act(z, aff, True)) < 1e-2  # (native: one fma, RNE rounding)
    st = torch.zeros(2, K, device=gpu)
    y = C().conv_fwd(z, w, e, 1, 1, 1, 1, False, st, shift, pre=aff)
    st0 = torch.zeros(2, K, device=gpu)
    y0 = C().conv_fwd(x, w, e, 1, 1, 1, 1, False, st0, shift)
    torch.cuda.synchronize()
    assert torch.equal(y, y0), rel(y, y0)
    assert torch.equal(st, st0)
    str_ = torch.zeros(2, K, device=gpu)
    yr = ref.conv_fwd(z, w, e, 1, 1, 1, 1, False, str_, shift, pre=aff)
    assert rel(y, yr) < 2e-2 and rel(st, str_) < 2e-2


@pytest.mark.parametrize("case", PRE_CASES)
def test_conv_wgrad_pre_bitwise(gpu, case):
    N, H, W, Cc, K = case
    z, aff, w, dy = _operands(N, H, W, Cc, K, gpu, 32)
    x = C().affine_act(z, aff, True)
    dw = torch.zeros(K, 3, 3, Cc, device=gpu)
    C().conv_wgrad(dy, z, dw, 1, 1, 1, 1, overwrite=True, pre=aff)
    dw0 = torch.zeros_like(dw)
    C().conv_wgrad(dy, x, dw0, 1, 1, 1, 1, overwrite=True)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw0), rel(dw, dw0)
    dwr = torch.zeros_like(dw)
    ref.conv_wgrad(dy, z, dwr, 1, 1, 1, 1, overwrite=True, pre=aff)
    assert rel(dw, dwr) < 2e-2


@pytest.mark.parametrize("case", [c for c in PRE_CASES if c[3] % 32 == 0])
def test_halo_wgrad_producer_waves_bitwise(gpu, case):
    """The 8-wave producer form of the halo weight gradient == the 4-wave form, bitwise
    (same tiles, same MFMA order per block)."""
    N, H, W, Cc, K = case
    _z, _aff, _w, dy = _operands(N, H, W, Cc, K, gpu, 33)
    x = torch.randn(N, H, W, Cc, device=gpu).to(torch.bfloat16)
    out = []
    try:
        for prod in (1, 0):
            C().igemm_set_halo_wprod(prod)
            dw = torch.zeros(K, 3, 3, Cc, device=gpu)
            C().conv_wgrad(dy, x, dw, 1, 1, 1, 1, overwrite=True)
            out.append(dw)
    finally:
        C().igemm_set_halo_wprod(1)  # (the default)
    torch.cuda.synchronize()
    assert torch.equal(out[0], out[1])


def test_strided_conv_pre_falls_back(gpu):
    """A consumer the halo kernels cannot take (3x3 / stride 2) materializes the operand:
    same result as running on affine_act(z)."""
    z, aff, w, _ = _operands(2, 28, 28, 64, 128, gpu, 34)
    e = torch.empty(0, device=gpu)
    y = C().conv_fwd(z, w, e, 2, 2, 1, 1, False, e, e, pre=aff)
    y0 = C().conv_fwd(C().affine_act(z, aff, True), w, e, 2, 2, 1, 1, False, e, e)
    torch.cuda.synchronize()
    assert torch.equal(y, y0)


@pytest.mark.parametrize("block", ["layer1.0", "layer2.0", "layer3.1", "layer4.1"])
def test_resnet_block_pre_bitwise(gpu, block, monkeypatch):
    """A ResNet-18 BasicBlock with bn1 applied in conv2's operand path == the block that
    writes y1, bitwise in deterministic mode: output, bn running stats, input gradient and
    every parameter gradient."""
    import mpi_pytorch_amd.models.resnet as R
    from mpi_pytorch_amd.engine import build_training
    from mpi_pytorch_amd.parallel import World
    C().set_deterministic(1)
    try:
        torch.manual_seed(0)
        model = build_training("resnet18", 10, gpu, World(device=gpu), 1e-3)[0]
        a = model._mpa_arena
        blk = model.get_submodule(block)
        cin = blk.conv1.weight.shape[3]
        hw = {"layer1.0": 56, "layer2.0": 56, "layer3.1": 14, "layer4.1": 7}[block]
        g = torch.Generator(device="cpu").manual_seed(5)
        x0 = torch.randn(8, hw, hw, cin, generator=g).to(gpu, torch.bfloat16)
        sd = {k: v.clone() for k, v in blk.state_dict().items()}
        res = []
        for pre in (True, False):
            monkeypatch.setattr(R, "_PRE", pre)
            blk.load_state_dict(sd)
            a.zero_grad()
            x = x0.clone().requires_grad_(True)
            y = blk(x)
            wgt = torch.linspace(-1, 1, y.numel(), device=gpu).view_as(y)
            (y.float() * wgt).sum().backward()
            torch.cuda.synchronize()
            grads = torch.cat([a.grad[slice(*a.slice_of(p))] for p in blk.parameters()])
            res.append((y.detach().clone(), x.grad.clone(), grads.clone(),
                        [v.clone() for k, v in blk.state_dict().items() if "running" in k]))
        (y1, dx1, g1, r1), (y2, dx2, g2, r2) = res
        assert torch.equal(y1, y2)
        # (running statistics: bn_stats_affine and bn_fwd_train update them with the same
        # formula, but the compiler may contract it into fma differently: 1 ulp)
        assert all(torch.allclose(u, v, rtol=1e-6, atol=0) for u, v in zip(r1, r2))
        assert torch.equal(dx1, dx2)
        assert torch.equal(g1, g2)
    finally:
        C().set_deterministic(0)
