"""GPU checks of the zoo models' structural fusions against their plain module form, block
by block with identical inputs (bf16 kernels on both sides):

* Inception: the 1x1 branch heads as ONE grouped GEMM (``Fn.conv1x1_group``: flat arena
  weights, per-branch BN on channel windows of z, one wgrad / dgrad) vs the separate
  BasicConv2d modules (``/root/reference/models.py:83-95`` -> torchvision InceptionA/C/D/E);
* DenseNet: a dense block on one feature buffer (``_DenseBlockGrad``: norm1 on the channel
  prefix from per-feature statistics, input gradients added in fp32 by the BN-backward apply)
  vs per-layer concat + plain autograd (``models.py:74-81`` -> torchvision _DenseBlock).
"""
import pytest
import torch

from mpi_pytorch_amd.engine import build_training
from mpi_pytorch_amd.parallel import World
from mpi_pytorch_amd.ops import functional as Fn

pytestmark = pytest.mark.gpu


def _cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float(a @ b / (a.norm() * b.norm() + 1e-30))


def _rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).abs().max() / (b.abs().max() + 1e-6))


def _param_grads(arena, mods):
    out = []
    for m in mods:
        for p in m.parameters():
            o, e = arena.slice_of(p)
            out.append(arena.grad[o:e].clone())
    return torch.cat(out)


@pytest.mark.parametrize("block,hw", [("Mixed_5b", 35), ("Mixed_6c", 17), ("Mixed_7a", 17),
                                      ("Mixed_7c", 8)])
def test_inception_grouped_heads_match_separate_convs(gpu, block, hw):
    torch.manual_seed(0)
    model, _o, _s, _ = build_training("inception", 100, gpu, World(device=gpu), 1e-3)
    a = model._mpa_arena
    blk = getattr(model, block)
    heads = blk.heads()
    C = heads[0].conv.weight.shape[-1]
    assert Fn.conv1x1_group_ok(torch.empty(1, device=gpu), heads)
    g = torch.Generator(device="cpu").manual_seed(1)
    x0 = torch.randn(16, hw, hw, C, generator=g).to(gpu, torch.bfloat16)
    res = []
    for grouped in (True, False):
        a.zero_grad()
        x = x0.clone().requires_grad_(True)
        outs = Fn.conv1x1_group(x, heads, None) if grouped else [h(x) for h in heads]
        loss = sum((o.float() * torch.linspace(-1, 1, o.numel(), device=gpu).view_as(o)).sum()
                   for o in outs)
        loss.backward()
        torch.cuda.synchronize()
        res.append(([o.detach() for o in outs], x.grad.clone(), _param_grads(a, heads)))
    (o1, dx1, g1), (o2, dx2, g2) = res
    for u, v in zip(o1, o2):
        assert u.shape == v.shape and _rel(u, v) < 2e-2
    assert _cos(dx1, dx2) > 0.999 and _rel(dx1, dx2) < 3e-2
    assert _cos(g1, g2) > 0.999 and abs(float(g1.norm() / g2.norm()) - 1) < 1e-2


def test_densenet_feature_buffer_block_matches_plain(gpu):
    torch.manual_seed(0)
    model, _o, _s, _ = build_training("densenet", 100, gpu, World(device=gpu), 1e-3)
    a = model._mpa_arena
    blk = model.features.denseblock1
    g = torch.Generator(device="cpu").manual_seed(2)
    x0 = torch.randn(16, 28, 28, 64, generator=g).to(gpu, torch.bfloat16)
    sd = {k: v.clone() for k, v in blk.state_dict().items()}
    res = []
    for fused in (True, False):
        blk.load_state_dict(sd)
        a.zero_grad()
        x = x0.clone().requires_grad_(True)
        out, stats = blk(x, fused)
        assert (stats is not None) == fused
        w = torch.linspace(-1, 1, out.numel(), device=gpu).view_as(out)
        (out.float() * w).sum().backward()
        torch.cuda.synchronize()
        res.append((out.detach(), x.grad.clone(), _param_grads(a, [blk]),
                    [v.clone() for k, v in blk.state_dict().items() if "running" in k], stats))
    (o1, dx1, g1, r1, st), (o2, dx2, g2, r2, _) = res
    assert o1.shape == o2.shape and _rel(o1, o2) < 2e-2
    # the block statistics table holds every output channel's batch mean / variance
    of = o2.float().reshape(-1, o2.shape[-1])
    assert _rel(st[0], of.mean(0)) < 1e-2 and _rel(st[1], of.var(0, unbiased=False)) < 2e-2
    assert all(_rel(u, v) < 1e-2 for u, v in zip(r1, r2))
    # the plain path sums each feature's gradient contributions in bf16 (autograd's adds of
    # the concat's split), the buffer path in fp32: elementwise they differ by the bf16
    # rounding of up to six partial sums (max |diff| ~7 % of max |dx| at the cancelling
    # entries), in direction and norm they agree
    assert _cos(dx1, dx2) > 0.999 and abs(float(dx1.float().norm() / dx2.float().norm()) - 1) < 1e-2
    assert _cos(g1, g2) > 0.999 and abs(float(g1.norm() / g2.norm()) - 1) < 1e-2


@pytest.mark.parametrize("name,cin,hw", [("denseblock1", 64, 28), ("denseblock3", 256, 14)])
def test_densenet_bf16_block_gradient_accumulator(gpu, name, cin, hw, monkeypatch):
    """The dense block's gradient accumulator G in bf16 (the default: each contribution
    added in fp32 and rounded once) vs in fp32 (MPA_DENSE_GRAD_BF16=0), one whole
    DenseNet-121 block (6 / 24 layers), same inputs and output gradient: the block-input
    gradient and every parameter gradient agree in direction (cosine >= 0.999), in norm
    and elementwise to a bounded relative error.  Reference model: torchvision
    densenet121 reached from /root/reference/models.py:77."""
    import mpi_pytorch_amd.models.densenet as D
    torch.manual_seed(0)
    model, _o, _s, _ = build_training("densenet", 100, gpu, World(device=gpu), 1e-3)
    a = model._mpa_arena
    blk = getattr(model.features, name)
    g = torch.Generator(device="cpu").manual_seed(3)
    x0 = torch.randn(16, hw, hw, cin, generator=g).to(gpu, torch.bfloat16)
    sd = {k: v.clone() for k, v in blk.state_dict().items()}
    res = []
    for bf16 in (True, False):
        monkeypatch.setattr(D, "_GRAD_BF16", bf16)
        blk.load_state_dict(sd)
        a.zero_grad()
        x = x0.clone().requires_grad_(True)
        out, _stats = blk(x, True)
        w = torch.linspace(-1, 1, out.numel(), device=gpu).view_as(out)
        (out.float() * w).sum().backward()
        torch.cuda.synchronize()
        res.append((x.grad.float().clone(), _param_grads(a, [blk])))
    (dx_b, g_b), (dx_f, g_f) = res
    assert float(dx_f.abs().max()) > 0 and float(g_f.abs().max()) > 0
    assert _cos(dx_b, dx_f) > 0.999 and abs(float(dx_b.norm() / dx_f.norm()) - 1) < 5e-3
    assert _cos(g_b, g_f) > 0.999 and abs(float(g_b.norm() / g_f.norm()) - 1) < 5e-3
    assert _rel(dx_b, dx_f) < 3e-2, _rel(dx_b, dx_f)
    assert _rel(g_b, g_f) < 3e-2, _rel(g_b, g_f)
