"""Unit-level (teacher-forced) gradient parity of a native GPU model against the fp32 CPU
path.

Why not compare whole-model gradients: deep CNNs at initialisation have *shattered*
gradients - the weight gradient decorrelates under tiny input perturbations.  On the CPU,
in fp32, merely rounding the input image to bf16 moves the gradient direction to cosine
0.39 (Inception-v3), 0.90 (DenseNet-121) and 0.94 (ResNet-34), with BN in train or eval mode
(docs/NOTES.md "Numerics"); a bf16 GPU path rounds every activation, so a whole-model
direction check cannot be tight, and cannot catch a wrong branch gradient.

Instead every *unit* (a ResNet block, an Inception block, a DenseNet layer, a Fire module,
a classifier Linear, ...) is checked on its own with the GPU's actual inputs:

1. one GPU forward + backward of the whole model, where each unit's inputs and output pass
   through identity taps that record the values and the gradients (the gradient into a
   unit's input tap is that unit's own input gradient, even when the input feeds other
   units too; the output tap sees the full gradient the unit's backward received);
2. per unit, the CPU fp32 copy of the unit runs forward on the recorded GPU input (upcast)
   and backward on the recorded GPU output gradient (upcast);
3. output, input gradient and parameter gradients (the GPU's come from the flat arena)
   are compared.  Within one unit a few bf16 roundings cannot shatter the gradient, so a
   wrong dgrad / wgrad / concat offset / branch sum shows up as a low cosine.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch
import torch.nn as nn


class _Tap(torch.autograd.Function):
    """Identity whose backward records the incoming gradient into ``box``."""

    @staticmethod
    def forward(ctx, x, box):
        ctx.box = box
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        ctx.box.append(g.detach().clone())
        return g, None


def unit_modules(model: nn.Module) -> List[Tuple[str, nn.Module]]:
    """The units of a zoo model: modules called through ``Module.__call__`` (so hooks fire)
    that own parameters and take one tensor (or a list of tensors) in."""
    from ..models.resnet import BasicBlock
    from ..models import inception as I
    from ..models.densenet import _DenseLayer, _Transition
    from ..models.squeezenet import Fire
    from ..models.layers import Linear, FusedSequential
    kinds = (BasicBlock, I.InceptionA, I.InceptionB, I.InceptionC, I.InceptionD,
             I.InceptionE, I.InceptionAux, I.BasicConv2d, _DenseLayer, _Transition, Fire)
    out, taken = [], set()
    for name, m in model.named_modules():
        if any(name.startswith(t + ".") for t in taken):
            continue
        if isinstance(m, kinds):
            out.append((name, m))
            taken.add(name)
    for name, m in model.named_modules():  # classifiers called as modules
        if any(name == t or name.startswith(t + ".") for t in taken):
            continue
        if isinstance(m, Linear) and "." not in name:
            out.append((name, m))
            taken.add(name)
        elif isinstance(m, FusedSequential) and name in ("features", "classifier") and \
                not any(isinstance(c, kinds) for c in m.children()):
            out.append((name, m))  # VGG / AlexNet stacks: executed fused, hooked whole
            taken.add(name)
    return out


def _tapped_groups(name: str, fs, rec: Dict):
    """An instance-level ``run_group`` for a FusedSequential that records every group with
    parameters as unit ``name[first:end]`` (input / output values and gradients)."""
    cls_run = type(fs).run_group
    mods = list(fs._modules.values())

    def run_group(g, x, link_in=None, link_out=None):
        # (unit_parity runs the stacks unlinked: no hand-offs between groups)
        i0, i1, kind = g
        if not any(p.requires_grad for mm in mods[i0:i1] for p in mm.parameters()):
            return cls_run(fs, g, x, link_in=link_in, link_out=link_out)
        key = "%s[%d:%d]" % (name, i0, i1)
        r = rec.setdefault(key, {"calls": 0, "group": g, "fs": name, "fs_mod": fs,
                                 "kind": kind})
        r["calls"] += 1
        bx, by = [], []
        r["x"], r["gx"] = x.detach().clone(), bx
        out = cls_run(fs, g, _Tap.apply(x, bx), link_in=link_in, link_out=link_out)
        r["y"], r["gy"] = out.detach().clone(), by
        return _Tap.apply(out, by)

    return run_group


def _cos(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.double().flatten(), b.double().flatten()
    na, nb = float(a.norm()), float(b.norm())
    if na == 0.0 and nb == 0.0:
        return 1.0
    if na == 0.0 or nb == 0.0:
        return 0.0
    return float((a @ b) / (na * nb))


def _ratio(a: torch.Tensor, b: torch.Tensor) -> float:
    nb = float(b.double().norm())
    return float(a.double().norm()) / nb if nb > 0 else (1.0 if float(a.norm()) == 0 else 0.0)


def unit_parity(model_gpu: nn.Module, model_cpu: nn.Module, x: torch.Tensor, y: torch.Tensor,
                loss_fn) -> List[Dict]:
    """Run the teacher-forced comparison; returns one record per unit with the cosines
    and norm ratios of output, input gradient and parameter gradients (GPU vs CPU)."""
    units = unit_modules(model_gpu)
    cpu_mods = dict(model_cpu.named_modules())
    rec: Dict[str, Dict] = {}
    hooks = []

    def pre(name):
        def fn(mod, args):
            r = rec.setdefault(name, {"calls": 0})
            r["calls"] += 1
            a0 = args[0]
            if isinstance(a0, (list, tuple)):
                boxes = [[] for _ in a0]
                r["x"] = [t.detach().clone() for t in a0]
                r["gx"] = boxes
                return ([_Tap.apply(t, b) for t, b in zip(a0, boxes)],) + tuple(args[1:])
            box = []
            r["x"] = a0.detach().clone()
            r["gx"] = box
            return (_Tap.apply(a0, box),) + tuple(args[1:])
        return fn

    def post(name):
        def fn(mod, args, out):
            r = rec[name]
            box = []
            r["y"] = out.detach().clone()
            r["gy"] = box
            return _Tap.apply(out, box)
        return fn

    from ..models.layers import FusedSequential
    patched = []
    for name, m in units:
        if isinstance(m, FusedSequential):
            # a fused stack (VGG / AlexNet): every fused group with parameters is a unit
            patched.append(m)
            m.run_group = _tapped_groups(name, m, rec)
            continue
        hooks.append(m.register_forward_pre_hook(pre(name)))
        hooks.append(m.register_forward_hook(post(name)))
    # a GradJoin spanning two units would hand one unit the other's input gradient
    cross = getattr(model_gpu, "cross_join", None)
    if cross is not None:
        model_gpu.cross_join = False
    # DenseNet's fused blocks run each layer's norm1 inside the block, not through the
    # _DenseLayer module: the plain per-layer path makes every layer a hooked unit
    fused = getattr(model_gpu, "fused_blocks", None)
    if fused is not None:
        model_gpu.fused_blocks = False
    pools = getattr(model_gpu, "fuse_stem_pools", None)
    if pools is not None:
        model_gpu.fuse_stem_pools = False
    # Inception's grouped 1x1 branch heads: one GEMM, not the BasicConv2d units
    grouped = [m for m in model_gpu.modules() if hasattr(m, "heads")]
    for m in grouped:
        m.merge_1x1 = False
    # backward hand-offs BETWEEN units (conv -> ReLU -> conv / pool links of the VGG / AlexNet
    # stacks, Inception's chained BasicConv2d links): the consumer's dgrad would apply the
    # producer's ReLU mask, so its recorded input gradient is not the unit's own dx.  Units
    # run unlinked here; the links have tests of their own (test_models_cpu.py
    # test_feature_stack_links_match_unlinked, the model parity / learning tests).
    from ..models import layers as _L, inception as _I
    links = (_L._LINK, _I._LINK)
    _L._LINK = _I._LINK = False
    try:
        arena = model_gpu._mpa_arena
        arena.zero_grad()
        loss = loss_fn(model_gpu(x), y)
        loss.backward()
        if x.is_cuda:
            torch.cuda.synchronize()
    finally:
        for h in hooks:
            h.remove()
        for m in patched:
            del m.run_group
        if cross is not None:
            model_gpu.cross_join = cross
        if fused is not None:
            model_gpu.fused_blocks = fused
        if pools is not None:
            model_gpu.fuse_stem_pools = pools
        for m in grouped:
            m.__dict__.pop("merge_1x1", None)
        _L._LINK, _I._LINK = links
    g_gpu = arena.grad.detach().cpu()
    out = []
    plain = {name: m for name, m in units}
    for name in list(rec.keys()):
        r = rec[name]
        if r["calls"] != 1 or not r.get("gy"):
            continue  # not reached (e.g. aux head in eval) or reused
        ac = model_cpu._mpa_arena
        ac.zero_grad()
        if "group" in r:  # a fused group of a FusedSequential stack
            fs_g, fs_c = r["fs_mod"], cpu_mods[r["fs"]]
            i0, i1, _k = r["group"]
            m = nn.ModuleList(list(fs_g._modules.values())[i0:i1])
            mc = nn.ModuleList(list(fs_c._modules.values())[i0:i1])
            xc = r["x"].float().cpu().requires_grad_(True)
            yc = fs_c.run_group(r["group"], xc)
            gx_gpu = r["gx"][0].float().cpu() if r["gx"] else None
        else:
            m = plain[name]
            mc = cpu_mods[name]
            if isinstance(r["x"], list):
                xc = torch.cat([t.float().cpu() for t in r["x"]], -1).requires_grad_(True)
                yc = mc([xc])
                gx_gpu = torch.cat([b[0].float().cpu() if b else
                                    torch.zeros_like(t.float().cpu())
                                    for b, t in zip(r["gx"], r["x"])], -1)
            else:
                xc = r["x"].float().cpu().requires_grad_(True)
                yc = mc(xc)
                gx_gpu = r["gx"][0].float().cpu() if r["gx"] else None
        yg = r["y"].float().cpu()
        if yc.shape != yg.shape:  # padded head columns etc.: compare the common slice
            yg = yg[..., :yc.shape[-1]]
        gy = r["gy"][0].float().cpu()
        if gy.shape != yc.shape:
            gy = gy[..., :yc.shape[-1]]
        yc.backward(gy)
        g_cpu = ac.grad.detach()
        pg, pc = [], []
        for p_g, p_c in zip(m.parameters(), mc.parameters()):
            if not p_g.requires_grad:
                continue
            o, e = arena.slice_of(p_g)
            oc, ec = ac.slice_of(p_c)
            pg.append(g_gpu[o:e])
            pc.append(g_cpu[oc:ec])
        row = {"unit": name, "type": r.get("kind", type(m).__name__),
               "y_cos": _cos(yg, yc.detach()), "y_ratio": _ratio(yg, yc.detach())}
        if gx_gpu is not None and xc.grad is not None and r["x"] is not None and \
                getattr(r["x"] if not isinstance(r["x"], list) else r["x"][0], "dtype",
                        None) != torch.long:
            row["dx_cos"] = _cos(gx_gpu, xc.grad)
            row["dx_ratio"] = _ratio(gx_gpu, xc.grad)
        if pg:
            a, b = torch.cat(pg), torch.cat(pc)
            row["dw_cos"] = _cos(a, b)
            row["dw_ratio"] = _ratio(a, b)
            row["n_params"] = int(a.numel())
        out.append(row)
    return out
