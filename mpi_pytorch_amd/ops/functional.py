"""Autograd functions over the kernel API (NHWC activations, fused epilogues).

Each function dispatches on the activation's device: CUDA/HIP tensors go to the native
gfx950 kernels (``mpi_pytorch_amd._C``; missing extension => loud error), CPU tensors to
``ops/ref.py``.  The ops the reference reaches through ATen map to:

* ``conv_bn_act``   conv (implicit-GEMM MFMA, BN batch statistics accumulated in the conv
                    epilogue) -> BN apply (+ residual add) (+ ReLU)  [K1-K5, K8]
* ``conv_act``      conv + bias (+ ReLU) epilogue                     [K1, K5]
* ``bn_act``        standalone BN (+ReLU) for pre-activation nets (DenseNet)  [K4]
* ``linear_act``    Linear + bias (+ ReLU) on the same MFMA engine   [K9]
* ``max_pool2d``, ``avg_pool2d``, ``adaptive_avg_pool2d``            [K6, K7]
* ``dropout``                                                        [K14]
* ``cross_entropy`` fused log-softmax + NLL (mean), grad recomputed from saved LSE  [K10]

Parameter gradients never travel through autograd: backward kernels accumulate them in
fp32 directly into the flat gradient arena (``p.grad``) and then signal the DP bucketer
(``grad_done``), which may start that bucket's all-reduce immediately.  Parameters are
still autograd *inputs* so that backward reaches the first layer even though the image
tensor does not require grad.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import numpy as np
import torch

from . import ref
from . import _ext
from ..parallel.arena import weight_of, weight_t_of, grad_sink, grad_done

_EMPTY = {}
_NO_SHIFT = os.environ.get("MPA_NO_STATS_SHIFT", "0") == "1"  # diagnostics only


def K(t: torch.Tensor):
    """Kernel namespace for a tensor's device."""
    if t.is_cuda:
        return _ext.ext()
    return ref


def _empty(t: torch.Tensor) -> torch.Tensor:
    key = (t.device, torch.float32)
    e = _EMPTY.get(key)
    if e is None:
        e = torch.empty(0, device=t.device, dtype=torch.float32)
        _EMPTY[key] = e
    return e


def _or_empty(x: Optional[torch.Tensor], like: torch.Tensor) -> torch.Tensor:
    return x if x is not None else _empty(like)


def _sink(p: Optional[torch.nn.Parameter], like: torch.Tensor) -> torch.Tensor:
    if p is None:
        return _empty(like)
    s = grad_sink(p)
    return s if s is not None else _empty(like)


def _fresh(p: torch.nn.Parameter) -> bool:
    """Whether ``p``'s arena gradient is untouched since zero_grad (consumed by the call)."""
    a = getattr(p, "_mpa_arena", None)
    return a.take_fresh(p) if a is not None else False


def _done(*ps) -> None:
    for p in ps:
        if p is not None:
            grad_done(p)


# ================================================================ weight-gradient stream
# Inside TrainStep's eager backward (single GPU; MPA_WGRAD_STREAM=0 turns it off), the conv
# weight gradients run on a second HIP stream (+4 % ResNet-18, +2.7 % VGG-16 measured,
# profiles/ab_r4.txt).  A weight gradient reads only its op's dz and x and
# writes only the gradient arena, so it need not sit between the dgrad / BN-backward
# launches of the main chain: the memory-bound BN passes (no LDS, or 8 KiB) can run on the
# CUs beside a persistent MFMA-bound wgrad grid.  The step joins the stream before the
# optimizer (join_wgrad_stream); x / dz are record_stream'ed so the caching allocator does
# not hand their memory out while the side stream still reads it.
_WGRAD_STREAM = os.environ.get("MPA_WGRAD_STREAM", "1") == "1"
# (Linear weight gradients stay on the compute stream: on the side stream AlexNet lost
# 4.7 %, its three large FC weight gradients contending with the FC dgrads; round-4 A/B,
# profiles/ab_r4.txt call 21.)
_SIDE = {"stream": None, "on": False, "used": False}


def _capture_blocks_streams() -> bool:
    """A HIP-graph capture keeps one stream: replaying a multi-stream graph measured slower
    than the one-stream graph, and both slower than eager with streams (DenseNet-121 8.93k /
    9.07k / 9.53k img/s, profiles/ab_r4.txt call 15)."""
    return torch.cuda.is_current_stream_capturing()


# Halo weight-gradient form per step (unless MPA_HALO_WPROD pins it): the 4-wave kernel
# while the weight gradients run on the side stream, the producer-wave kernel when they
# share the compute stream (data parallelism).  Same-box round-5 A/B, ResNet-18 b1024:
# side stream 51.9k (4-wave) vs 51.0k (producer waves) img/s, one stream 50.4k vs 50.7k
# (profiles/halo_sched_r5.txt).
_WPROD_PINNED = "MPA_HALO_WPROD" in os.environ


def _halo_wgrad_form(side_on: bool) -> None:
    if not _WPROD_PINNED:
        _ext.ext().igemm_set_halo_wprod(0 if side_on else 1)


def wgrad_stream_begin(enabled: bool = True) -> None:
    """Route the following conv weight gradients to the side stream (TrainStep backward)."""
    _SIDE["on"] = bool(enabled and _WGRAD_STREAM)
    if torch.cuda.is_available():
        _halo_wgrad_form(_SIDE["on"])
        if _SIDE["on"]:
            _SIDE["main"] = torch.cuda.current_stream()


def wgrad_streams():
    """(compute stream, side stream) while side-stream weight gradients are routed and the
    side stream exists, else None: a gradient bucket launched then must wait for both
    (parallel/ddp.py GradBucketer._launch)."""
    if _SIDE["on"] and _SIDE["stream"] is not None and _SIDE.get("main") is not None:
        return _SIDE["main"], _SIDE["stream"]
    return None


def join_wgrad_stream() -> None:
    """Make the current stream wait for every side-stream weight gradient; route off."""
    _SIDE["on"] = False
    if _SIDE["used"]:
        torch.cuda.current_stream().wait_stream(_SIDE["stream"])
        _SIDE["used"] = False


def _run_wgrad(fn, *tensors) -> None:
    """Run ``fn`` (a weight-gradient launch and its arena notifications) on the side stream
    when routing is on, else in place."""
    t0 = tensors[0]
    if not (_SIDE["on"] and t0.is_cuda) or _capture_blocks_streams():
        fn()
        return
    main = torch.cuda.current_stream()
    side = _SIDE["stream"]
    if side is None or side.device != t0.device:
        side = _SIDE["stream"] = torch.cuda.Stream(t0.device)
    side.wait_stream(main)
    # (set_stream / restore instead of the torch.cuda.stream context: ~20 us less host
    # time per weight gradient, which the host-bound small-batch step feels)
    torch.cuda.set_stream(side)
    try:
        fn()
    finally:
        torch.cuda.set_stream(main)
    for t in tensors:
        t.record_stream(side)
    _SIDE["used"] = True


# ================================================================== branch stream (Inception)
# Inside TrainStep's step (single GPU, eager), an Inception block's longest branch chain is
# enqueued on a second stream and the block's other branches on the compute stream, joined
# before the block output is used (models/inception.py SideBranch).  Autograd runs each
# node's backward on the stream of its forward, so the chains' backwards overlap too.
# Every tensor that crosses between the streams is record_stream'ed on its consumer (the
# chain input and block buffer at the fork, the block-output gradient in
# _ChannelBuffer.backward, the chain-input gradient in _ConvGroupBNAct.backward), so the
# caching allocator never hands out memory the other stream still reads.
_BRANCH_STREAM = os.environ.get("MPA_BRANCH_STREAM", "1") == "1"
_BR = {"stream": None, "on": False, "used": False}


def branch_streams(enabled: bool) -> None:
    """Allow (TrainStep forward + backward) or stop side-branch streams."""
    _BR["on"] = bool(enabled and _BRANCH_STREAM)


def branch_stream(x: torch.Tensor):
    """The stream a side branch reading ``x`` runs on, or None (off, CPU, no grad, or a
    HIP-graph capture)."""
    if not (_BR["on"] and x.is_cuda and torch.is_grad_enabled()):
        return None
    if _capture_blocks_streams():
        return None
    s = _BR["stream"]
    if s is None or s.device != x.device:
        s = _BR["stream"] = torch.cuda.Stream(x.device)
    _BR["used"] = True
    return s


def join_branch_stream() -> None:
    """The compute stream waits for everything enqueued on the branch stream."""
    s = _BR["stream"]
    if s is not None and _BR["used"]:
        torch.cuda.current_stream(s.device).wait_stream(s)
    _BR["used"] = False


def _branch_use(*ts) -> None:
    """Mark tensors that may come from the other stream as used by the current one."""
    if _BR["on"] and _BR["stream"] is not None:
        cur = torch.cuda.current_stream(_BR["stream"].device)
        for t in ts:
            if t is not None and t.is_cuda:
                t.record_stream(cur)


# =============================================================================== conv+BN
class BNLink:
    """Backward hand-off between two fused conv+BN ops when the first op's output feeds ONLY
    the second (ResNet BasicBlock: conv1 -> bn1 -> relu -> conv2).  The consumer's dgrad
    epilogue then performs the producer's BN-backward reduction - it applies the ReLU
    mask and sums (g, g * x_hat) while the gradient is still in registers - and the
    producer's backward runs only the BN apply pass (no reduce pass, no re-read of dy/y).

    (Round 5 also built the producer's BN + ReLU into the consumer's operand staging; it
    measured 3.9 % slower - profiles/wprod_pre_ab_r5.txt - and was removed in round 6.)"""

    __slots__ = ("z", "y", "mean", "rstd", "gamma", "beta", "sums", "gacc")

    def __init__(self):
        self.z = self.y = self.mean = self.rstd = self.gamma = self.beta = self.sums = None
        # gacc: a DenseNet block gradient.  The consumer's (1x1) dgrad then ADDS gamma*rstd *
        # g into its first Ci channels instead of returning dx, and the producer side
        # (_DenseBlockGrad) finishes the BN backward with deferred per-channel corrections
        self.gacc = None


class BNDefer:
    """A train-mode BN whose apply pass runs in its one consumer (ResNet's downsample BN,
    read as bn2's residual): the producing op computes only the statistics half
    (``bn_stats_affine``: mean, rstd, running stats) and returns the raw conv output; ``aff``
    ([2, C] scale | shift) is what the consumer's ``bn_fwd_train(res_affine=)`` applies while
    reading it.  The tensor then stands for the BN output in autograd: the consumer hands
    back d/d(BN output), which the producer's backward turns into its own BN backward."""

    __slots__ = ("aff", "z", "mean", "rstd", "gamma", "beta", "done")

    def __init__(self):
        self.aff = None
        # the producer's BN inputs, for the consumer's fused backward (bn_bwd_pair): the
        # consumer then hands back d/dz directly and sets `done`
        self.z = self.mean = self.rstd = self.gamma = self.beta = None
        self.done = False


# MPA_BN_PAIR=0: the consumer of a deferred BN (ResNet bn2) writes g = dy * mask and the
# downsample op runs its own BN backward (reduce + apply) on it
_BN_PAIR = os.environ.get("MPA_BN_PAIR", "1") == "1"


class GradJoin:
    """Several gradient contributions to ONE activation, summed without separate add passes.

    A residual block's input x feeds two ops (conv1 and the shortcut: identity or the
    downsample conv); an Inception block's input feeds three or four branches (1x1 convs
    and a pool).  Autograd would sum those bf16 gradients with elementwise adds - a full
    extra read/read/write sweep of the activation per extra consumer.  Instead all
    consumers hold the same join, created with ``expected`` = their number.  Each backward
    that runs hands its contribution to the join and returns None for x, except the LAST
    one, which returns the sum: a computed tensor (a pool or BN gradient) becomes the
    running partial, a dgrad is parked as the deferred launch itself and later either
    writes fresh or accumulates into the partial in its GEMM epilogue
    (``conv_dgrad(..., accum=)``: fp32 add, one rounding per contribution).  A fresh write is
    given to a dgrad that covers every pixel, so a 1x1/s2 downsample (three of four stride
    phases without taps) never needs a zero fill.  Independent of autograd's execution
    order (autograd runs x's producer only after every consumer's backward)."""

    __slots__ = ("partial", "expected", "arrived")

    def __init__(self, expected: int = 2):
        self.partial = None
        self.expected = int(expected)
        self.arrived = 0

    def take(self):
        p, self.partial = self.partial, None
        return p

    def arrive(self) -> bool:
        """Count one contribution; True when it is the last."""
        self.arrived += 1
        return self.arrived >= self.expected


class _Deferred:
    """A parked dgrad: ``run(accum)`` launches it (fresh when accum is None); ``args`` =
    (dz, w, wt, conv) lets the next contribution merge it into its own launch."""

    __slots__ = ("run", "full", "args")

    def __init__(self, run, full: bool, args=None):
        self.run = run
        self.full = full
        self.args = args


# MPA_DGRAD_PAIR=0: a residual stage's conv1 (3x3/s2) and 1x1/s2 shortcut dgrads run as two
# launches (the second accumulating into the first's dx) instead of one merged launch
_PAIR = os.environ.get("MPA_DGRAD_PAIR", "1") == "1"


def _dgrad_pair(k, a, b, in_hw):
    """Both parked/current dgrads of one activation in one launch (``conv_dgrad_pair``):
    a = (dz, w, wt, conv) of a conv whose taps cover every pixel, b = the other."""
    dz, w, wt, conv = a
    dz2, w2, wt2, conv2 = b
    sh, sw, ph, pw = conv.kgeom
    sh2, sw2, ph2, pw2 = conv2.kgeom
    if (sh, sw) != (sh2, sw2) or (dz.is_cuda and (wt is None or wt2 is None)):
        return None
    if tuple(dz.shape) != tuple(dz2.shape) or w.shape[3] != w2.shape[3]:
        return None
    if not hasattr(k, "conv_dgrad_pair"):
        return None
    return k.conv_dgrad_pair(dz, w, wt, in_hw[0], in_hw[1], sh, sw, ph, pw, dz2, w2, wt2,
                             ph2, pw2)


class _MaskedRes:
    """A residual block's shortcut gradient dy * (y > 0) not yet written: the block input's
    other consumer (conv1's stride-1 dgrad) adds it in its epilogue (``conv_dgrad_res``), or
    it is materialised when that is not available."""

    __slots__ = ("dy", "mask")

    def __init__(self, dy, mask):
        self.dy = dy
        self.mask = mask

    def materialize(self, k):
        if not self.dy.is_cuda:
            return (self.dy.float() * ref.bitmask_unpack(self.mask, self.dy.shape)).to(
                self.dy.dtype)
        bits = (self.mask.unsqueeze(-1) >> torch.arange(8, device=self.mask.device,
                                                         dtype=torch.uint8)) & 1
        return self.dy * bits.reshape(self.dy.shape).to(self.dy.dtype)


# MPA_RES_MASK=0: a residual block writes its shortcut gradient dy * mask for conv1's dgrad to
# accumulate, instead of conv1's dgrad epilogue reading dy and the bit mask itself
_RES_MASK = os.environ.get("MPA_RES_MASK", "1") == "1"


def _join_grad(join: Optional[GradJoin], t):
    """Offer a computed contribution ``t`` (a tensor or a _MaskedRes) to ``join``; returns
    what the op hands back to autograd (the sum if it is the last contribution, else None)."""
    if join is None or t is None:
        return t
    last = join.arrive()
    prev = join.take()
    if isinstance(t, _MaskedRes) and (last or prev is not None):
        t = t.materialize(None)
    if isinstance(prev, _MaskedRes):
        prev = prev.materialize(None)
    if prev is None:
        acc = t
    elif isinstance(prev, _Deferred):
        acc = prev.run(t)  # the parked dgrad accumulates into t
    else:  # two computed tensors (Inception's Mixed_7a maxpool + aux-head avg-pool)
        acc = prev.contiguous()
        K(acc).add_bf16_(acc, t.contiguous())
    if last:
        return acc
    join.partial = acc
    return None


def _dgrad_full(conv, in_hw) -> bool:
    """Every pixel of dx receives taps (no tap-less stride phase)."""
    sh, sw = conv.kgeom[:2]
    R, S = conv.weight.shape[1:3]
    return sh <= R and sw <= S


def _dgrad_joined(k, join: Optional[GradJoin], dz, w, in_hw, conv, wt):
    """conv dgrad, summed with the join's other contributions (see GradJoin)."""
    sh, sw, ph, pw = conv.kgeom

    def run(acc):
        return k.conv_dgrad(dz, w, in_hw[0], in_hw[1], sh, sw, ph, pw, wt, acc)

    if join is None:
        return run(None)
    last = join.arrive()
    prev = join.take()
    full = _dgrad_full(conv, in_hw)
    args = (dz, w, wt, conv)
    if isinstance(prev, _MaskedRes):
        acc = None
        sh, sw, ph, pw = conv.kgeom
        if sh == 1 and sw == 1 and hasattr(k, "conv_dgrad_res") and (wt is not None
                                                                    or not dz.is_cuda):
            acc = k.conv_dgrad_res(dz, w, wt, in_hw[0], in_hw[1], ph, pw, prev.dy, prev.mask)
        if acc is None:
            acc = run(prev.materialize(k))
        if last:
            return acc
        join.partial = acc
        return None
    if prev is None:
        if last:
            return run(None)
        join.partial = _Deferred(run, full, args)
        return None
    if isinstance(prev, _Deferred):
        acc = None
        if _PAIR and prev.args is not None and full != prev.full:
            acc = (_dgrad_pair(k, args, prev.args, in_hw) if full
                   else _dgrad_pair(k, prev.args, args, in_hw))
        if acc is not None:
            pass
        elif full or not prev.full:
            acc = prev.run(run(None))
        else:
            acc = run(prev.run(None))
    else:
        acc = run(prev)
    if last:
        return acc
    join.partial = acc
    return None


class _ConvBNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, w, b, gamma, beta, conv, bn, relu, link_in=None, link_out=None,
                join_x=None, join_res=None, defer=None, res_defer=None, out=None):
        k = K(x)
        sh, sw, ph, pw = conv.kgeom
        C = w.shape[0]
        stats = torch.empty(2, C, device=x.device, dtype=torch.float32)
        # BN statistics come out of the conv epilogue, shifted by the running mean
        z = k.conv_fwd(x, weight_of(w), _or_empty(b, x), sh, sw, ph, pw, False, stats,
                       _empty(x) if _NO_SHIFT else bn.running_mean)
        # relu(bn(z) + residual): the backward's ReLU mask as one bit per element, written by
        # the forward, so neither backward pass reads y (two activation-sized reads less)
        ymask = None
        if relu and residual is not None:
            ymask = torch.empty(z.numel() // 8, device=z.device, dtype=torch.uint8)
        if defer is not None:  # statistics only; the consumer applies this BN (BNDefer)
            mean, rstd, defer.aff = k.bn_stats_affine(z, stats, gamma, beta, bn.running_mean,
                                                      bn.running_var, bn.momentum_value(),
                                                      bn.eps, bn.num_batches_tracked)
            defer.z, defer.mean, defer.rstd, defer.gamma, defer.beta = z, mean, rstd, gamma, beta
            defer.done = False
            y = z
        else:
            y, mean, rstd = k.bn_fwd_train(z, stats, gamma, beta, bn.running_mean,
                                           bn.running_var, bn.momentum_value(), bn.eps,
                                           _or_empty(residual, x), relu,
                                           bn.num_batches_tracked, mask=ymask,
                                           res_affine=(res_defer.aff if res_defer is not None
                                                       else None), out=out)
        ctx.conv = conv
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.bias = b
        ctx.params = (w, gamma, beta)
        ctx.in_hw = (x.shape[1], x.shape[2])
        # (relu(bn(z)) without a residual recomputes its mask from z: y is not kept)
        keep_y = relu and ymask is None and not (residual is None and beta is not None)
        ctx.save_for_backward(x, z, y if keep_y else None, mean, rstd, ymask)
        ctx.link_in = link_in
        ctx.link_out = link_out
        ctx.join_x = join_x
        ctx.join_res = join_res
        ctx.defer = defer
        ctx.res_defer = res_defer if (ymask is not None and relu and _BN_PAIR) else None
        if link_out is not None:
            link_out.z, link_out.mean, link_out.rstd = z, mean, rstd
            # ReLU without a residual: the consumer's halo dgrad recomputes the mask from z
            # (as the forward rounded y) when the BN is affine and never reads y (the
            # implicit-GEMM fallback does)
            zmask = relu and residual is None and gamma is not None and beta is not None
            link_out.y = y if relu else None
            link_out.gamma, link_out.beta = (gamma, beta) if zmask else (None, None)
            link_out.sums = None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, z, y, mean, rstd, ymask = ctx.saved_tensors
        w, gamma, beta = ctx.params
        conv = ctx.conv
        k = K(dy)
        dy = _rows(dy)
        want_g = bool(ctx.has_res and ctx.needs_input_grad[1])
        lo = ctx.link_out
        rd = ctx.res_defer
        dres_pair = None
        if ctx.defer is not None and ctx.defer.done:
            # the consumer's bn_bwd_pair already ran this BN's backward: dy IS d/dz, and the
            # affine gradients are in place
            dz = dy
            ctx.defer.done = False
        elif (rd is not None and rd.z is not None and ctx.needs_input_grad[1]
                and ctx.join_res is None and hasattr(k, "bn_bwd_pair")):
            g2, b2 = rd.gamma, rd.beta
            dz, dres_pair = k.bn_bwd_pair(dy, z, ymask, mean, rstd, gamma, _sink(gamma, dy),
                                          _sink(beta, dy), rd.z, rd.mean, rd.rstd, g2,
                                          _sink(g2, dy), _sink(b2, dy))
            _done(g2, b2)
            rd.done = True
            rd.z = None
        elif lo is not None and lo.sums is not None:
            # the consumer's dgrad already masked dy and reduced (sum g, sum g*xhat)
            dz, g = k.bn_bwd_apply(dy, z, _empty(dy), mean, rstd, gamma, _sink(gamma, dy),
                                   _sink(beta, dy), lo.sums, True, want_g)
            lo.sums = None
        elif ctx.relu and not ctx.has_res and beta is not None:
            # relu(bn(z)) without a residual: the mask is recomputed from z, y is not read
            dz, g = k.bn_bwd(dy, z, _empty(dy), mean, rstd, gamma, _sink(gamma, dy),
                             _sink(beta, dy), True, want_g, beta)
        else:
            # identity shortcut: conv1's dgrad adds dy * mask in its epilogue (_MaskedRes), so
            # g is not written here
            mres = (want_g and _RES_MASK and ymask is not None and ctx.join_res is not None
                    and ctx.join_res.arrived == 0 and ctx.join_res.partial is None)
            dz, g = k.bn_bwd(dy, z, _or_empty(y, dy), mean, rstd, gamma, _sink(gamma, dy),
                             _sink(beta, dy), True, want_g and not mres, ymask=ymask)
            if mres:
                g = _MaskedRes(dy, ymask)
        if ctx.defer is None or dz is not dy:
            _done(gamma, beta)
        sh, sw, ph, pw = conv.kgeom
        if w.requires_grad:
            def wgrad():
                k.conv_wgrad(dz, x, w.grad, sh, sw, ph, pw, overwrite=_fresh(w))
                conv.fix_grad(w.grad)
                _done(w)
            _run_wgrad(wgrad, dz, x)
        _done(ctx.bias)
        if dres_pair is not None:
            dres = dres_pair  # d/dz of the deferred BN's producer (see BNDefer.done)
        else:
            dres = g if (ctx.has_res and ctx.needs_input_grad[1]) else None
            dres = _join_grad(ctx.join_res, dres)
        dx = None
        if ctx.needs_input_grad[0]:
            li = ctx.link_in
            wt = weight_t_of(w)
            if (li is not None and li.gacc is not None and (wt is not None or not dz.is_cuda)
                    and k.conv_bnred_ok(w.shape[0], w.shape[3])):
                li.sums = k.conv_dgrad_bnred_gacc(dz, weight_of(w), wt, li.z, li.mean, li.rstd,
                                                  li.gamma, li.beta, li.gacc)
                dx = None
            elif (li is not None and li.z is not None and (wt is not None or not dz.is_cuda)
                    and k.conv_bnred_ok(w.shape[0], w.shape[3])):
                dx, li.sums = k.conv_dgrad_bnred(dz, weight_of(w), ctx.in_hw[0], ctx.in_hw[1],
                                                 sh, sw, ph, pw, wt, li.z,
                                                 _or_empty(li.y, dz), li.mean, li.rstd,
                                                 gamma=li.gamma, beta=li.beta)
                dx = _join_grad(ctx.join_x, dx)
            else:
                dx = _dgrad_joined(k, ctx.join_x, dz, weight_of(w), ctx.in_hw, conv, wt)
        return (dx, dres, None, None, None, None, None, None, None, None, None, None, None, None,
                None, None)


def _rows(t: torch.Tensor) -> torch.Tensor:
    """``t`` if its rows are uniformly strided with contiguous channels (a channel window
    of a wider NHWC buffer, which the BN kernels read in place), else a contiguous copy."""
    if t.is_contiguous():
        return t
    if t.dim() >= 2 and t.stride(-1) == 1:
        ld, expect = t.stride(-2), t.stride(-2) * t.shape[-2]
        ok = ld >= t.shape[-1] and ld % 8 == 0
        for d in range(t.dim() - 3, -1, -1):
            ok = ok and (t.shape[d] == 1 or t.stride(d) == expect)
            expect *= t.shape[d]
        if ok:
            return t
    return t.contiguous()


def conv_bn_act(x, conv, bn, relu: bool = True, residual: Optional[torch.Tensor] = None,
                link_in: Optional[BNLink] = None, link_out: Optional[BNLink] = None,
                join_x: Optional[GradJoin] = None, join_res: Optional[GradJoin] = None,
                defer: Optional[BNDefer] = None, res_defer: Optional[BNDefer] = None,
                out: Optional[torch.Tensor] = None):
    """relu(bn(conv(x)) [+ residual]); BN in train or eval mode per ``bn.training``.
    ``out`` (train mode, no residual): a channel window of a wider NHWC buffer the result
    is written into (see ``channel_buffer``).

    A conv bias in front of a train-mode BN (VGG11_bn) is added before the statistics, so
    forward and running stats are exact; its gradient is exactly zero in exact arithmetic
    (BN removes any per-channel constant) and is left at zero instead of accumulating
    rounding noise."""
    x = conv.fit_input(x)
    if bn.training:
        # (defer: bn(conv(x)) without ReLU or residual, a train-mode affine BN)
        if defer is not None and (relu or residual is not None or bn.weight is None
                                  or bn.bias is None):
            defer = None
        if out is not None and (residual is not None or defer is not None or link_out is not None):
            out = None
        return _ConvBNAct.apply(x, residual, conv.weight, conv.bias, bn.weight, bn.bias, conv,
                                bn, relu, link_in, link_out, join_x, join_res, defer, res_defer,
                                out)
    k = K(x)
    sh, sw, ph, pw = conv.kgeom
    z = k.conv_fwd(x, weight_of(conv.weight), _or_empty(conv.bias, x), sh, sw, ph, pw, False,
                   _empty(x), _empty(x))
    return k.bn_fwd_eval(z, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps,
                         _or_empty(residual, x), relu)


class _ConvGroupBNAct(torch.autograd.Function):
    """relu(bn_b(conv_b(x))) for several 1x1 convs that read the same x (Inception's branch
    heads), as ONE GEMM over their joint output rows.

    The weights sit back to back in the arena (``_mpa_param_groups``), so the joint weight,
    its bf16 shadow and its gradient are flat views - no copies.  Forward: one conv over
    N = sum N_b columns with BN statistics from its epilogue, then each branch's BN+ReLU
    reads its channel window of z (strided rows).  A member with ``pool_after`` (Inception's
    pool branch: 1x1 conv and 3x3 average pool commute) average-pools its window first and
    takes its BN statistics from the pooled values.  Backward: each branch's BN (and pool)
    backward writes its window of ONE dz, then one wgrad (x read once, not once per branch)
    and ONE dgrad (one write of dx instead of a write plus an accumulate pass per extra
    branch).
    Reference: InceptionA/C/D/E branch heads of torchvision inception_v3, reached from
    ``/root/reference/models.py:83-95``."""

    @staticmethod
    def forward(ctx, x, W, mods, join, outs, *params):
        k = K(x)
        ntot = W.shape[0]
        stats = torch.empty(2, ntot, device=x.device, dtype=torch.float32)
        z = k.conv_fwd(x, W, _empty(x), 1, 1, 0, 0, False, stats, _empty(x))
        res, saved, o = [], [], 0
        for m in mods:
            bn, n = m.bn, m.conv.weight.shape[0]
            pool = getattr(m, "pool_after", None)
            if pool is not None:  # avg-pool the window, BN statistics of the pooled values
                zin = k.avgpool_fwd(z[..., o:o + n], *pool)
                st = _empty(x)
            else:
                zin, st = z[..., o:o + n], stats[:, o:o + n]
            dst = outs[len(res)] if outs is not None else None
            y, mean, rstd = k.bn_fwd_train(zin, st, bn.weight, bn.bias, bn.running_mean,
                                           bn.running_var, bn.momentum_value(), bn.eps,
                                           _empty(x), True, bn.num_batches_tracked, out=dst)
            res.append(y)
            saved.append((mean, rstd, o, n, zin if pool is not None else None, pool))
            o += n
        ctx.mods, ctx.join, ctx.saved, ctx.W = mods, join, saved, W
        ctx.in_hw = (x.shape[1], x.shape[2])
        ctx.nparams = len(params)
        ctx.save_for_backward(x, z)
        return tuple(res)

    @staticmethod
    def backward(ctx, *dys):
        x, z = ctx.saved_tensors
        _branch_use(*dys)  # (a member's gradient may come from a side-branch chain)
        k = K(z)
        dz = torch.empty_like(z)
        for m, (mean, rstd, o, n, zp, pool), dy in zip(ctx.mods, ctx.saved, dys):
            gamma, beta = m.bn.weight, m.bn.bias
            if pool is not None:
                dzp, _g = k.bn_bwd(_rows(dy), zp, _empty(dy), mean, rstd, gamma,
                                   _sink(gamma, dy), _sink(beta, dy), True, False, beta)
                k.avgpool_bwd(dzp, z.shape[1], z.shape[2], *pool, dx_out=dz[..., o:o + n])
            else:
                k.bn_bwd(_rows(dy), z[..., o:o + n], _empty(dy), mean, rstd, gamma,
                         _sink(gamma, dy), _sink(beta, dy), True, False, beta,
                         dx_out=dz[..., o:o + n])
            _done(gamma, beta)
        ws = [m.conv.weight for m in ctx.mods]
        if ws[0].requires_grad:
            def wgrad():
                fresh = [_fresh(w) for w in ws]  # (every flag consumed)
                G = ws[0]._mpa_arena.flat_view(ws, "grad").view(ctx.W.shape)
                k.conv_wgrad(dz, x, G, 1, 1, 0, 0, overwrite=all(fresh))
                _done(*ws)
            _run_wgrad(wgrad, dz, x)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _dgrad_joined(k, ctx.join, dz, ctx.W, ctx.in_hw, ctx.mods[0].conv, None)
        ctx.W = None
        return (dx, None, None, None, None) + (None,) * ctx.nparams


def conv1x1_group_ok(x, mods) -> bool:
    """Whether ``conv1x1_group`` can run ``mods`` (train-mode 1x1/s1 BasicConv2d's whose
    weights are one flat arena range)."""
    ws = [m.conv.weight for m in mods]
    a = getattr(ws[0], "_mpa_arena", None)
    if a is None or not torch.is_grad_enabled() or not all(m.bn.training for m in mods):
        return False
    if any(m.conv.kgeom != (1, 1, 0, 0) or m.conv.weight.shape[1:3] != (1, 1) or
           m.conv.bias is not None or not w.requires_grad for m, w in zip(mods, ws)):
        return False
    if any(getattr(m, "pool_after", None) is not None and
           tuple(m.pool_after[2:6]) != (1, 1, (m.pool_after[0] - 1) // 2,
                                        (m.pool_after[1] - 1) // 2) for m in mods):
        return False  # (a pooled window must keep z's spatial size)
    return a.flat_view(ws, "master") is not None


def conv1x1_group(x, mods, join: Optional[GradJoin] = None, outs=None):
    """[relu(bn(conv(x))) for each BasicConv2d in mods] as one GEMM (see _ConvGroupBNAct);
    ``join``: x's gradient is summed with its other consumers' (one contribution here);
    ``outs``: per member, a channel window to write its output into, or None."""
    ws = [m.conv.weight for m in mods]
    a = ws[0]._mpa_arena
    W = a.flat_view(ws, "shadow" if a.shadow is not None else "master")
    ntot = sum(w.shape[0] for w in ws)
    W = W.view(ntot, 1, 1, ws[0].shape[-1])
    params = [p for m in mods for p in (m.conv.weight, m.bn.weight, m.bn.bias) if p is not None]
    return _ConvGroupBNAct.apply(x, W, list(mods), join, outs, *params)


def _pool_out(n: int, k: int, s: int, p: int, ceil: bool) -> int:
    """Pooled extent, ATen's rule (a ceil-mode window must start inside the padded input)."""
    o = (n + 2 * p - k + (s - 1 if ceil else 0)) // s + 1
    if ceil and (o - 1) * s >= n + p:
        o -= 1
    return o


class _ConvBNReLUPool(torch.autograd.Function):
    """maxpool(relu(bn(conv(x)))) -- the ResNet / DenseNet stem -- with BN, ReLU and the
    pool fused into one pass over the conv output z (forward) and the pool's gradient
    gathered straight into the BN backward (backward): the full-size BN output and its
    gradient never exist.  Reference: torchvision stems reached from ``models.py:24-30``
    (resnet) and ``models.py:74-80`` (densenet)."""

    @staticmethod
    def forward(ctx, x, w, b, gamma, beta, conv, bn, cfg):
        k = K(x)
        sh, sw, ph, pw = conv.kgeom
        C = w.shape[0]
        stats = torch.empty(2, C, device=x.device, dtype=torch.float32)
        shift = _empty(x) if _NO_SHIFT else bn.running_mean
        r = None
        if (_STEM_POOL_FWD and x.is_cuda and b is None and tuple(cfg) == (3, 3, 2, 2, 1, 1, False)
                and gamma is not None and beta is not None):
            # the pool taken inside the stem conv kernel, BN + ReLU on the pooled extremes
            r = k.conv_stem_pool_fwd(x, weight_of(w), sh, sw, ph, pw, stats, shift, gamma, beta,
                                     bn.running_mean, bn.running_var, bn.momentum_value(),
                                     bn.eps, bn.num_batches_tracked)
        if r is not None:
            y, idx, mean, rstd, z, zsel = r
        else:
            z = k.conv_fwd(x, weight_of(w), _or_empty(b, x), sh, sw, ph, pw, False, stats, shift)
            # zsel: raw z at each window's argmax, so the backward's reduction pass reads only
            # pooled-size tensors (maxpool_bn_bwd_sel_reduce_kernel)
            N, H, W, C_ = z.shape
            zsel = torch.empty(N, _pool_out(H, cfg[0], cfg[2], cfg[4], cfg[6]),
                               _pool_out(W, cfg[1], cfg[3], cfg[5], cfg[6]), C_,
                               device=z.device, dtype=z.dtype)
            y, idx, mean, rstd = k.bn_relu_maxpool_fwd(z, stats, gamma, beta, bn.running_mean,
                                                       bn.running_var, bn.momentum_value(),
                                                       bn.eps, *cfg, bn.num_batches_tracked,
                                                       zsel_out=zsel)
        ctx.conv = conv
        ctx.cfg = cfg
        ctx.bias = b
        ctx.params = (w, gamma, beta)
        ctx.in_hw = (x.shape[1], x.shape[2])
        ctx.save_for_backward(x, z, idx, mean, rstd, zsel)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, z, idx, mean, rstd, zsel = ctx.saved_tensors
        w, gamma, beta = ctx.params
        conv = ctx.conv
        k = K(dy)
        sh, sw, ph, pw = conv.kgeom
        dy = dy.contiguous()
        if (_STEM_POOL_WGRAD and w.requires_grad and not ctx.needs_input_grad[0]
                and ctx.bias is None and tuple(ctx.cfg) == (3, 3, 2, 2, 1, 1, False)
                and k.stem_pool_wgrad_ok(dy, idx, z, x, w.grad, sh, sw, ph, pw)):
            # image stem: the BN / pool backward's dz pass runs inside the weight
            # gradient's operand staging, so no full-resolution dz exists
            sums = k.maxpool_bn_bwd_sums(dy, zsel, mean, rstd, gamma, beta, _sink(gamma, dy),
                                         _sink(beta, dy))
            _done(gamma, beta)

            def wgrad():
                k.stem_pool_wgrad(dy, idx, z, mean, rstd, gamma, beta, sums, x, w.grad,
                                  sh, sw, ph, pw, _fresh(w))
                conv.fix_grad(w.grad)
                _done(w)
            _run_wgrad(wgrad, dy, idx, z, x, mean, rstd, sums)
            return None, None, None, None, None, None, None, None
        dz = k.maxpool_bn_bwd(dy, idx, z, mean, rstd, gamma, beta, _sink(gamma, dy),
                              _sink(beta, dy), *ctx.cfg[:6], zsel=zsel)
        _done(gamma, beta)
        if w.requires_grad:
            def wgrad():
                k.conv_wgrad(dz, x, w.grad, sh, sw, ph, pw, overwrite=_fresh(w))
                conv.fix_grad(w.grad)
                _done(w)
            _run_wgrad(wgrad, dz, x)
        _done(ctx.bias)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = k.conv_dgrad(dz, weight_of(w), ctx.in_hw[0], ctx.in_hw[1], sh, sw, ph, pw,
                              weight_t_of(w))
        return dx, None, None, None, None, None, None, None


# (A/B switches) the stem's pool backward inside its weight gradient (on: 1.06 ms vs 1.63 ms
# two-pass at batch 1024), and its pool forward inside the stem conv kernel (conv_stem.hip;
# off: the 114 KB z image in LDS leaves one 4-wave block per CU, 1.64 ms vs 1.17 ms for
# conv + bn_relu_maxpool_fwd - profiles/stem_pool_r6.txt)
_STEM_POOL_WGRAD = os.environ.get("MPA_STEM_POOL_WGRAD", "1") == "1"
_STEM_POOL_FWD = os.environ.get("MPA_STEM_POOL_FWD", "0") == "1"


def conv_bn_relu_maxpool(x, conv, bn, pool):
    """``pool(relu(bn(conv(x))))`` for a MaxPool2d ``pool``; fused in train mode."""
    cfg = (pool.kernel_size[0], pool.kernel_size[1], pool.stride[0], pool.stride[1],
           pool.padding[0], pool.padding[1], bool(pool.ceil_mode))
    if bn.training and cfg[0] * cfg[1] <= 256:
        x = conv.fit_input(x)
        return _ConvBNReLUPool.apply(x, conv.weight, conv.bias, bn.weight, bn.bias, conv, bn,
                                     cfg)
    return pool(conv_bn_act(x, conv, bn, relu=True))


# ============================================================================ conv + bias
_UNIT = {}


def _unit_affine(C: int, device):
    """(mean 0, rstd 1, gamma 1, beta 0) of length C: the identity 'BN' through which a
    plain ReLU's mask and bias-gradient reduction ride the fused BN-backward-reduction
    dgrad (bn(y) = y, so the mask is y > 0 and sum g is the bias gradient)."""
    key = (C, device)
    t = _UNIT.get(key)
    if t is None:
        z, o = torch.zeros(C, device=device), torch.ones(C, device=device)
        t = _UNIT[key] = (z, o, o, z)
    return t


class _ConvAct(torch.autograd.Function):
    """act(conv(x) + b).  ``link_out`` (BNLink): this op's ReLU output feeds ONLY the next
    conv, whose dgrad applies the ReLU mask (y > 0) and reduces the bias gradient in its
    epilogue (the BN-backward-reduction flavour with an identity affine), so this op's
    backward runs no act_bwd pass (VGG / AlexNet conv -> ReLU -> conv chains,
    ``/root/reference/models.py:50,59``); ``link_in``: the BNLink of this op's input."""

    @staticmethod
    def forward(ctx, x, w, b, conv, relu, join=None, stats=None, shift=None, out=None,
                link_in=None, link_out=None):
        k = K(x)
        sh, sw, ph, pw = conv.kgeom
        if out is not None:  # written straight into a channel window of a wider buffer
            k.conv_fwd_into(x, weight_of(w), _or_empty(b, x), sh, sw, ph, pw, relu,
                            _or_empty(stats, x), _or_empty(shift, x), out)
            y = out
        else:
            y = k.conv_fwd(x, weight_of(w), _or_empty(b, x), sh, sw, ph, pw, relu,
                           _or_empty(stats, x), _or_empty(shift, x))
        ctx.conv = conv
        ctx.relu = relu
        ctx.params = (w, b)
        ctx.in_hw = (x.shape[1], x.shape[2])
        ctx.join = join
        ctx.link_in = link_in
        ctx.link_out = link_out
        if link_out is not None and relu and out is None:
            C = y.shape[-1]
            link_out.z = link_out.y = y
            link_out.mean, link_out.rstd, link_out.gamma, link_out.beta = \
                _unit_affine(C, y.device)
            link_out.sums = None
        ctx.save_for_backward(x, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y = ctx.saved_tensors
        w, b = ctx.params
        conv = ctx.conv
        k = K(dy)
        dy = dy.contiguous()
        lo = ctx.link_out
        if lo is not None and lo.sums is not None:
            # the consumer's dgrad already applied the mask; its sum g is the bias gradient
            g = dy
            bs = _sink(b, dy)
            if bs.numel():
                k.add_f32_(bs, lo.sums[:bs.numel()])
            lo.sums = None
        else:
            g = k.act_bwd(dy, _or_empty(y, dy), _sink(b, dy))
        _done(b)
        sh, sw, ph, pw = conv.kgeom
        if w.requires_grad:
            def wgrad():
                k.conv_wgrad(g, x, w.grad, sh, sw, ph, pw, overwrite=_fresh(w))
                conv.fix_grad(w.grad)
                _done(w)
            _run_wgrad(wgrad, g, x)
        dx = None
        if ctx.needs_input_grad[0]:
            li = ctx.link_in
            wt = weight_t_of(w)
            if (li is not None and li.z is not None and ctx.join is None
                    and (wt is not None or not g.is_cuda)
                    and k.conv_bnred_ok(w.shape[0], w.shape[3])):
                dx, li.sums = k.conv_dgrad_bnred(g, weight_of(w), ctx.in_hw[0], ctx.in_hw[1],
                                                 sh, sw, ph, pw, wt, li.z, _or_empty(li.y, g),
                                                 li.mean, li.rstd, gamma=li.gamma, beta=li.beta)
            else:
                dx = _dgrad_joined(k, ctx.join, g, weight_of(w), ctx.in_hw, conv, wt)
        return dx, None, None, None, None, None, None, None, None, None, None


def conv_act(x, conv, relu: bool = False, join: Optional[GradJoin] = None,
             stats: Optional[torch.Tensor] = None, shift: Optional[torch.Tensor] = None,
             out: Optional[torch.Tensor] = None, link_in: Optional[BNLink] = None,
             link_out: Optional[BNLink] = None):
    """act(conv(x) + b); ``join``: x's gradient is summed with its other consumers' (see
    GradJoin); ``stats`` ([2, N] fp32, training): receives the output's per-channel
    [mean | var] from the GEMM epilogue (sums shifted by ``shift`` for precision); ``out``
    (training): a channel window of a wider NHWC buffer the output is written into (the
    result is that window; ``stats`` may then be a [2, N] window of a wider table)."""
    x = conv.fit_input(x)
    if torch.is_grad_enabled() and (conv.weight.requires_grad or x.requires_grad):
        return _ConvAct.apply(x, conv.weight, conv.bias, conv, relu, join, stats, shift, out,
                              link_in, link_out)
    k = K(x)
    sh, sw, ph, pw = conv.kgeom
    return k.conv_fwd(x, weight_of(conv.weight), _or_empty(conv.bias, x), sh, sw, ph, pw, relu,
                      _empty(x), _empty(x))


# =========================================================================== standalone BN
class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, bn, relu, stats=None, out=None):
        k = K(x)
        y, mean, rstd = k.bn_fwd_train(x, _or_empty(stats, x), gamma, beta, bn.running_mean,
                                       bn.running_var, bn.momentum_value(), bn.eps, _empty(x),
                                       relu, bn.num_batches_tracked, out=out)
        ctx.params = (gamma, beta)
        # relu(bn(x)) with an affine BN recomputes its mask from x: y is not kept
        zmask = relu and beta is not None and gamma is not None
        ctx.zmask = zmask
        ctx.save_for_backward(x, y if (relu and not zmask) else None, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mean, rstd = ctx.saved_tensors
        gamma, beta = ctx.params
        k = K(dy)
        dy = _rows(dy)
        dx, _g = k.bn_bwd(dy, x, _or_empty(y, dy), mean, rstd, gamma, _sink(gamma, dy),
                          _sink(beta, dy), bool(ctx.needs_input_grad[0]), False,
                          beta if ctx.zmask else None)
        _done(gamma, beta)
        return dx, None, None, None, None, None, None


def bn_act(x, bn, relu: bool = True, stats: Optional[torch.Tensor] = None,
           out: Optional[torch.Tensor] = None):
    """relu?(bn(x)); ``stats`` (train mode): x's [mean | var] [2, C] when already known
    (a DenseNet block's per-feature statistics), saving the statistics pass; ``out`` (train
    mode): a channel window of a wider buffer to write the result into."""
    if bn.training:
        return _BNAct.apply(x, bn.weight, bn.bias, bn, relu, stats, out)
    return K(x).bn_fwd_eval(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps,
                            _empty(x), relu)


class _BNReluAvgPool2(torch.autograd.Function):
    """avg_pool2d(relu(bn(x)), 2, 2), train mode, the BN output never written: the
    statistics half (bn_stats_affine) then one pass that applies BN + ReLU while pooling.
    Backward: avgpool_bwd, then the BN backward with the mask recomputed from x."""

    @staticmethod
    def forward(ctx, x, gamma, beta, bn, stats=None):
        k = K(x)
        if stats is None:
            stats = k.bn_stats(x, bn.running_mean)
        mean, rstd, aff = k.bn_stats_affine(x, stats, gamma, beta, bn.running_mean,
                                            bn.running_var, bn.momentum_value(), bn.eps,
                                            bn.num_batches_tracked)
        ctx.params = (gamma, beta)
        ctx.hw = (x.shape[1], x.shape[2])
        ctx.save_for_backward(x, mean, rstd)
        return k.bn_relu_avgpool2_fwd(x, aff)

    @staticmethod
    def backward(ctx, dp):
        x, mean, rstd = ctx.saved_tensors
        gamma, beta = ctx.params
        k = K(dp)
        dy = k.avgpool_bwd(dp.contiguous(), ctx.hw[0], ctx.hw[1], 2, 2, 2, 2, 0, 0, False, True)
        dx, _g = k.bn_bwd(dy, x, _empty(dy), mean, rstd, gamma, _sink(gamma, dy),
                          _sink(beta, dy), bool(ctx.needs_input_grad[0]), False, beta)
        _done(gamma, beta)
        return dx, None, None, None, None


def bn_relu_avgpool2(x, bn, stats: Optional[torch.Tensor] = None):
    """avg_pool2d(relu(bn(x)), 2, 2) (DenseNet transitions with the pool ahead of the conv);
    train mode with an affine BN, even H and W; other cases compose the two ops."""
    if (bn.training and bn.weight is not None and bn.bias is not None and x.shape[1] % 2 == 0
            and x.shape[2] % 2 == 0 and x.shape[3] % 8 == 0):
        return _BNReluAvgPool2.apply(x, bn.weight, bn.bias, bn, stats)
    return avg_pool2d(bn_act(x, bn, True, stats), (2, 2), (2, 2))


# ================================================================================ linear
class _LinearAct(torch.autograd.Function):
    """y = act(x W^T + b) over the layer's padded output width; returns the first
    ``nout`` columns (a view) when the layer stores padded rows (layers.Linear)."""

    @staticmethod
    def forward(ctx, x, w, b, relu, nout):
        k = K(x)
        y = k.linear_fwd(x, weight_of(w), _or_empty(b, x), relu)
        ctx.relu = relu
        ctx.params = (w, b)
        ctx.nout = nout
        ctx.save_for_backward(x, y if relu else None)
        return y if nout == y.shape[1] else y[:, :nout]

    @staticmethod
    def backward(ctx, dy):
        x, y = ctx.saved_tensors
        w, b = ctx.params
        k = K(dy)
        dy = _padded_grad(dy, w.shape[0])
        g = k.act_bwd(dy, _or_empty(y, dy), _sink(b, dy))
        # dgrad before the weight gradient's notify: once every gradient of a classifier is
        # final, its optimizer update may start on a side stream (TrainStep's early head
        # update) - nothing may read the old bf16 weight after that point
        dx = (k.linear_dgrad(g, weight_of(w), weight_t_of(w)) if ctx.needs_input_grad[0]
              else None)
        _done(b)
        if w.requires_grad:
            k.linear_wgrad(g, x, w.grad, overwrite=_fresh(w))
            _done(w)
        return dx, None, None, None, None


def _padded_grad(dy, width: int):
    """Gradient of a padded layer's output view as a contiguous [B, width] tensor.  The
    cross-entropy backward already returns a view of a [B, width] buffer with zero padding
    columns - use that buffer (ce_bwd wrote its zeros:
    tests/test_kernels_gpu.py::test_cross_entropy_padded_rows); anything else is
    zero-padded by a copy."""
    if dy.shape[1] == width:
        return dy.contiguous()
    base = dy._base
    if (base is not None and base.dim() == 2 and tuple(base.shape) == (dy.shape[0], width)
            and base.is_contiguous() and dy.data_ptr() == base.data_ptr()
            and dy.stride() == base.stride()):
        return base  # (ce_bwd wrote zeros into the padding columns)
    return torch.nn.functional.pad(dy, (0, width - dy.shape[1])).contiguous()


def linear_act(x, lin, relu: bool = False):
    nout = getattr(lin, "out_features", lin.weight.shape[0])
    if torch.is_grad_enabled() and (lin.weight.requires_grad or x.requires_grad):
        return _LinearAct.apply(x, lin.weight, lin.bias, relu, nout)
    y = K(x).linear_fwd(x, weight_of(lin.weight), _or_empty(lin.bias, x), relu)
    return y if nout == y.shape[1] else y[:, :nout]


# ================================================================================= pools
class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cfg, join=None, link_in=None):
        y, idx = K(x).maxpool_fwd(x, *cfg)
        ctx.cfg = cfg
        ctx.join = join
        ctx.link_in = link_in
        ctx.hw = (x.shape[1], x.shape[2])
        ctx.save_for_backward(idx, y if link_in is not None else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        idx, y = ctx.saved_tensors
        k = K(dy)
        dy = dy.contiguous()
        li = ctx.link_in
        if li is not None and ctx.join is None and hasattr(k, "maxpool_bwd_relu"):
            # the input is a ReLU output whose producer handed its backward over (BNLink):
            # route only where the pooled value is > 0 and return the producer's bias sums
            r = k.maxpool_bwd_relu(dy, idx, y, ctx.hw[0], ctx.hw[1], *ctx.cfg[:6])
            if r is not None:
                li.sums = r[1]
                return r[0], None, None, None
        dx = k.maxpool_bwd(dy, idx, ctx.hw[0], ctx.hw[1], *ctx.cfg)
        return _join_grad(ctx.join, dx), None, None, None


def max_pool2d(x, kernel, stride, padding=(0, 0), ceil_mode=False,
               join: Optional[GradJoin] = None, link_in: Optional[BNLink] = None):
    """``join``: the input's other consumers share it (see GradJoin); ``link_in``: the input
    is a conv -> ReLU output that feeds only this pool, and the pool's backward applies the
    ReLU mask and reduces the conv's bias gradient (Fn.BNLink; 2x2/s2 pools)."""
    cfg = (kernel[0], kernel[1], stride[0], stride[1], padding[0], padding[1], bool(ceil_mode))
    if torch.is_grad_enabled() and x.requires_grad:
        return _MaxPool.apply(x, cfg, join, link_in)
    return K(x).maxpool_fwd(x, *cfg)[0]


class _AvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cfg, join=None):
        ctx.cfg = cfg
        ctx.join = join
        ctx.hw = (x.shape[1], x.shape[2])
        return K(x).avgpool_fwd(x, *cfg)

    @staticmethod
    def backward(ctx, dy):
        dx = K(dy).avgpool_bwd(dy.contiguous(), ctx.hw[0], ctx.hw[1], *ctx.cfg)
        return _join_grad(ctx.join, dx), None, None


def avg_pool2d(x, kernel, stride, padding=(0, 0), ceil_mode=False, count_include_pad=True,
               join: Optional[GradJoin] = None):
    cfg = (kernel[0], kernel[1], stride[0], stride[1], padding[0], padding[1], bool(ceil_mode),
           bool(count_include_pad))
    if torch.is_grad_enabled() and x.requires_grad:
        return _AvgPool.apply(x, cfg, join)
    return K(x).avgpool_fwd(x, *cfg)


class _AdaptiveAvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, oh, ow):
        ctx.hw = (x.shape[1], x.shape[2])
        return K(x).adaptive_avgpool_fwd(x, oh, ow)

    @staticmethod
    def backward(ctx, dy):
        return K(dy).adaptive_avgpool_bwd(dy.contiguous(), ctx.hw[0], ctx.hw[1]), None, None


def adaptive_avg_pool2d(x, out_hw):
    oh, ow = out_hw
    if torch.is_grad_enabled() and x.requires_grad:
        return _AdaptiveAvgPool.apply(x, oh, ow)
    return K(x).adaptive_avgpool_fwd(x, oh, ow)


# ============================================================ concat at channel offsets
class _ChannelBuffer(torch.autograd.Function):
    """The channel concat of ``parts`` that their producers already wrote into their
    windows of ``buf`` (``out=`` of conv_bn_act / bn_act / conv1x1_group): forward returns
    the buffer (a part NOT at its window is copied in), backward hands each part its
    window of the gradient - a row-strided view, which the BN backward kernels read in
    place.  SURVEY K13: torchvision's ``torch.cat`` of Inception branch outputs
    (``/root/reference/models.py:83-95``) without the copy kernels."""

    @staticmethod
    def forward(ctx, buf, *parts):
        k = K(buf)
        o = 0
        ctx.sizes = []
        for t in parts:
            n = t.shape[-1]
            win = buf[..., o:o + n]
            if t.data_ptr() != win.data_ptr() or t.stride() != win.stride():
                k.chan_insert(buf, o, t.contiguous())
            ctx.sizes.append(n)
            o += n
        return buf.view(buf.shape)

    @staticmethod
    def backward(ctx, dy):
        s = _BR["stream"] if _BR["on"] else None
        if s is not None and dy.is_cuda:
            dy.record_stream(s)  # (a window may be read by a side-branch chain)
        outs, o = [], 0
        for n in ctx.sizes:
            outs.append(dy[..., o:o + n])
            o += n
        return (None,) + tuple(outs)


class ChannelBuffer:
    """An NHWC block output [N, H, W, sum(widths)] whose branches write their results at
    their channel offsets: ``window(i)`` is branch i's destination (pass it as ``out=``),
    ``gather(parts)`` the concat (no copy for parts already in place)."""

    def __init__(self, like: torch.Tensor, hw, widths):
        self.widths = list(widths)
        self.offs = [sum(self.widths[:i]) for i in range(len(self.widths))]
        self.buf = torch.empty((like.shape[0], hw[0], hw[1], sum(self.widths)),
                               device=like.device, dtype=like.dtype)

    def window(self, i: int) -> torch.Tensor:
        o = self.offs[i]
        return self.buf[..., o:o + self.widths[i]]

    def gather(self, parts):
        if torch.is_grad_enabled() and any(t.requires_grad for t in parts):
            return _ChannelBuffer.apply(self.buf, *parts)
        k = K(self.buf)
        for i, t in enumerate(parts):
            w = self.window(i)
            if t.data_ptr() != w.data_ptr():
                k.chan_insert(self.buf, self.offs[i], t.contiguous())
        return self.buf


# ======================================================================== channel concat
class _Concat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *xs):
        ctx.sizes = [x.shape[-1] for x in xs]
        return K(xs[0]).concat_channels(list(xs))

    @staticmethod
    def backward(ctx, dy):
        return tuple(K(dy).split_channels(dy.contiguous(), ctx.sizes))


def cat_channels(xs):
    """NHWC channel concat (torchvision's ``torch.cat(dim=1)`` on NCHW) [K13]: one native
    strided-copy kernel forward, the matching split kernel backward."""
    xs = [x.contiguous() for x in xs]
    if len(xs) == 1:
        return xs[0]
    if torch.is_grad_enabled() and any(x.requires_grad for x in xs):
        return _Concat.apply(*xs)
    return K(xs[0]).concat_channels(xs)


# =============================================================================== dropout
class DropoutRNG:
    """Stream position of the dropout masks, so every call draws a fresh mask.

    GPU: a device int32 counter per device, read by the dropout kernel as its offset and
    advanced on the stream after every call.  A HIP graph replays both, so each replay of a
    captured step draws new masks (a host-side offset would be frozen into the graph at
    capture, and every replay would reuse one mask).  CPU: a host counter.  The seed is a
    host constant.  ``state()`` / ``set_state()`` snapshot both (TrainStep.capture)."""
    seed = 0
    offset = 0
    _counters = {}

    @classmethod
    def counter(cls, device: torch.device) -> torch.Tensor:
        c = cls._counters.get(device)
        if c is None:
            c = cls._counters[device] = torch.zeros(1, dtype=torch.int32, device=device)
        return c

    @classmethod
    def state(cls):
        # (the current GPU's counter is created here if no dropout ran yet: a snapshot taken
        # before the first dropout call must still pin the position that call will start
        # from - otherwise set_state() cannot rewind it, e.g. TrainStep.capture's warm-up
        # steps in a process whose first dropout they are)
        if torch.cuda.is_available():
            cls.counter(torch.device("cuda", torch.cuda.current_device()))
        return cls.offset, {d: c.clone() for d, c in cls._counters.items()}

    @classmethod
    def set_state(cls, st) -> None:
        cls.offset = st[0]
        for d, c in st[1].items():
            cls.counter(d).copy_(c)


def _dropout_fwd(x, p):
    if x.is_cuda:  # offset = the device counter (advanced by the kernel launch pair)
        return K(x).dropout_fwd(x, p, DropoutRNG.seed, 0, DropoutRNG.counter(x.device))
    DropoutRNG.offset += 1
    return K(x).dropout_fwd(x, p, DropoutRNG.seed, DropoutRNG.offset)


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p):
        y, mask = _dropout_fwd(x, p)
        ctx.p = p
        ctx.save_for_backward(mask)
        return y

    @staticmethod
    def backward(ctx, dy):
        (mask,) = ctx.saved_tensors
        return K(dy).dropout_bwd(dy.contiguous(), mask, ctx.p), None


def dropout(x, p: float, training: bool):
    if not training or p == 0.0:
        return x
    if torch.is_grad_enabled() and x.requires_grad:
        return _Dropout.apply(x, p)
    return _dropout_fwd(x, p)[0]


# ========================================================================= cross-entropy
class _CrossEntropy(torch.autograd.Function):
    """sum_h weight_h * CE(logits_h, labels) as ONE native op: each head's fused
    log-softmax + NLL kernel adds its weighted mean into the loss scalar (and into the
    trainer's running loss sum ``acc``), the backward scales each head's softmax gradient
    by its weight - no elementwise ATen ops for Inception's ``loss + 0.4 * aux_loss``."""

    @staticmethod
    def forward(ctx, labels, weights, acc, *logits):
        k = K(logits[0])
        out = torch.empty(1, device=logits[0].device, dtype=torch.float32)
        lses = [k.ce_fwd_weighted(lg, labels, out, _or_empty(acc, lg), float(w), i > 0)
                for i, (lg, w) in enumerate(zip(logits, weights))]
        ctx.weights = weights
        ctx.save_for_backward(labels, *logits, *lses)
        return out.reshape(())

    @staticmethod
    def backward(ctx, go):
        saved = ctx.saved_tensors
        labels, n = saved[0], len(ctx.weights)
        logits, lses = saved[1:1 + n], saved[1 + n:]
        go = go.reshape(1).float().contiguous()
        gs = [K(lg).ce_bwd(lg, labels, lse, go, float(w))
              for lg, lse, w in zip(logits, lses, ctx.weights)]
        return (None, None, None) + tuple(gs)


def cross_entropy(logits, labels, weight: float = 1.0, acc: Optional[torch.Tensor] = None,
                  heads=None):
    """Mean softmax cross-entropy (``nn.CrossEntropyLoss()`` at main.py:134,150).

    ``heads``: extra (logits, weight) terms summed into the same loss (Inception aux);
    ``acc``: a float32 device scalar the loss is also added to (no host sync)."""
    lg = [logits] + [h[0] for h in (heads or [])]
    ws = (float(weight),) + tuple(float(h[1]) for h in (heads or []))
    if torch.is_grad_enabled() and any(t.requires_grad for t in lg):
        return _CrossEntropy.apply(labels, ws, acc, *lg)
    k = K(logits)
    out = torch.empty(1, device=logits.device, dtype=torch.float32)
    for i, (t, w) in enumerate(zip(lg, ws)):
        k.ce_fwd_weighted(t, labels, out, _or_empty(acc, t), w, i > 0)
    return out.reshape(())


def count_correct(logits, labels, count: torch.Tensor) -> None:
    """count += #(argmax(logits) == labels)  (main.py:182-183)."""
    K(logits).argmax_correct(logits, labels, count)


def preprocess(img_u8, out_hw, mean, std, mode: int = 0, cpad: int = 3,
               out_dtype=torch.bfloat16, pad=None, extents=None):
    """u8 [B,H,W,3] -> resized, normalized NHWC with ``cpad`` channels, optionally on a
    zero-bordered canvas ``pad`` = (top, bottom, left, right) (the pre-padded input layout
    of a pixel-pair stem, ``models.layers.Conv2d.input_spec``).

    mode 0: bilinear, no antialias (the train transform, main.py:62-65); mode 1: PIL-exact
    bicubic (the eval transform, evaluation_pipeline.py:89, data/pil_resize.py); mode 2:
    float antialiased bicubic (torch ``F.interpolate(antialias=True)`` semantics).
    ``extents`` (host int [B, 2]): image b occupies rows [0, h_b) and columns [0, w_b) of
    its slot (real images of different sizes decoded into one padded batch)."""
    k = K(img_u8)
    pad = list(pad) if pad else []
    if extents is not None:
        extents = np.asarray(extents, dtype=np.int64).reshape(-1, 2)
        B, Hp, Wp = img_u8.shape[:3]
        if extents.shape[0] != B or (extents < 1).any() or (extents[:, 0] > Hp).any() \
                or (extents[:, 1] > Wp).any():
            raise ValueError("preprocess: extents %s do not fit the [%d, %d] slot pitch"
                             % (extents.tolist(), Hp, Wp))
    if img_u8.is_cuda:
        if mode == 1:  # PIL-exact bicubic (the eval transform)
            tc = _PIL_TABLES.get(img_u8.device)
            if tc is None:
                from ..data.pil_resize import TableCache
                tc = _PIL_TABLES[img_u8.device] = TableCache(img_u8.device)
            B, Hp, Wp = img_u8.shape[:3]
            ext = extents if extents is not None else np.tile([[Hp, Wp]], (B, 1))
            e, sel, hb, hk, kh, vb, vk, kv = tc.tables(ext, tuple(out_hw), (Hp, Wp))
            return k.preprocess_pil(img_u8, e if extents is not None else _empty_i32(img_u8),
                                    sel, hb, hk, kh, vb, vk, kv, out_hw[0], out_hw[1],
                                    list(mean), list(std), cpad, pad)
        ext = None
        if extents is not None:
            ext = torch.from_numpy(extents.astype(np.int32)).to(img_u8.device, non_blocking=True)
        return k.preprocess(img_u8, out_hw[0], out_hw[1], list(mean), list(std), mode, cpad, pad,
                            ext)
    return k.preprocess(img_u8, out_hw[0], out_hw[1], list(mean), list(std), mode, cpad,
                        out_dtype, pad, extents)


_PIL_TABLES = {}


def _empty_i32(t: torch.Tensor) -> torch.Tensor:
    key = (t.device, torch.int32)
    e = _EMPTY.get(key)
    if e is None:
        e = _EMPTY[key] = torch.empty(0, device=t.device, dtype=torch.int32)
    return e
