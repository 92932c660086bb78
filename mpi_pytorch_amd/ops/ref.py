"""Plain-PyTorch implementation of the native kernel API (NHWC layout).

Two roles:
1. CPU execution path.  The reference framework is CPU-only (``main.py:50-51``), and
   BASELINE.json config 1 is a single-process CPU plumbing run, so CPU tensors run here.
2. Test oracle for every HIP kernel: the GPU tests call the same function here on the
   same inputs (computed in fp32) and compare.

It is NEVER used as a runtime fallback for GPU tensors (see ``ops/_ext.py``).

Every function mirrors a function of ``mpi_pytorch_amd._C`` with the same signature and
output dtypes: activations keep the input dtype (bf16 on GPU, fp32 on CPU), statistics
and gradient sinks are fp32.  Layouts: activations NHWC ``[N,H,W,C]``; conv weights
``[K,R,S,C]`` ("KRSC"); linear weights ``[out,in]``.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor


def _f(x: Tensor) -> Tensor:
    return x.float()


def _nchw(x: Tensor) -> Tensor:
    return x.permute(0, 3, 1, 2)


def _nhwc(x: Tensor) -> Tensor:
    return x.permute(0, 2, 3, 1).contiguous()


def _opt(t: Optional[Tensor]) -> Optional[Tensor]:
    if t is None or t.numel() == 0:
        return None
    return t


# ----------------------------------------------------------------------------------- conv
def conv_out_hw(H, W, R, S, sh, sw, ph, pw):
    return (H + 2 * ph - R) // sh + 1, (W + 2 * pw - S) // sw + 1


def affine_act(x, aff, relu):
    """relu?(x * aff[0] + aff[1]) per channel, in x's dtype (aff: bn_stats_affine's [2, C])."""
    y = _f(x) * aff[0].float() + aff[1].float()
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype)


def conv_fwd(x, w, bias, sh, sw, ph, pw, relu, stats, shift=None):
    y = F.conv2d(_nchw(_f(x)), _f(w).permute(0, 3, 1, 2), None if _opt(bias) is None else _f(bias),
                 (sh, sw), (ph, pw))
    y = _nhwc(y)
    if relu:
        y = torch.relu(y)
    y = y.to(x.dtype)
    st = _opt(stats)
    if st is not None:  # finalized (mean, biased var) of the output, like the native kernel
        yf = y.float().reshape(-1, y.shape[-1])
        st[0].copy_(yf.mean(0))
        st[1].copy_(yf.var(0, unbiased=False))
    return y


def conv_dgrad(dy, w, H, W, sh, sw, ph, pw, wt=None, accum=None):
    """wt: transposed weight copy (unused here); accum: add the result into this tensor
    (in place, one rounding of the fp32 sum) and return it."""
    N, P, Q, K = dy.shape
    Kw, R, S, C = w.shape
    gi = torch.ops.aten.convolution_backward(
        _nchw(_f(dy)).contiguous(), torch.empty(N, C, H, W, device=dy.device),
        _f(w).permute(0, 3, 1, 2).contiguous(), None, [sh, sw], [ph, pw], [1, 1], False,
        [0, 0], 1, [True, False, False])[0]
    if accum is not None:
        accum.copy_((_f(accum) + _nhwc(gi)).to(accum.dtype))
        return accum
    return _nhwc(gi).to(dy.dtype)


def conv_dgrad_res(dy, w, wt, H, W, ph, pw, res, rmask):
    """Stride-1 dgrad + the residual gradient res * (y > 0) (y's ReLU bit mask), summed in
    fp32 and rounded once."""
    d = _f(conv_dgrad(dy, w, H, W, 1, 1, ph, pw))
    g = _f(res) * bitmask_unpack(rmask, res.shape)
    return (d + g).to(dy.dtype)


def conv_dgrad_pair(dy, w, wt, H, W, sh, sw, ph, pw, dy2, w2, wt2, ph2, pw2, accum=None):
    """dx of two convs reading the same input with the same stride (3x3/s2 conv1 + its
    1x1/s2 shortcut), summed in fp32 and rounded once; None if the grids differ."""
    if sh == 1 and sw == 1:
        return None
    P2 = (H + 2 * ph2 - w2.shape[1]) // sh + 1
    Q2 = (W + 2 * pw2 - w2.shape[2]) // sw + 1
    if (P2, Q2) != tuple(dy.shape[1:3]):
        return None

    def gi(d, ww, p_h, p_w):
        N = d.shape[0]
        C = ww.shape[3]
        return torch.ops.aten.convolution_backward(
            _nchw(_f(d)).contiguous(), torch.empty(N, C, H, W, device=d.device),
            _f(ww).permute(0, 3, 1, 2).contiguous(), None, [sh, sw], [p_h, p_w], [1, 1],
            False, [0, 0], 1, [True, False, False])[0]

    tot = _nhwc(gi(dy, w, ph, pw) + gi(dy2, w2, ph2, pw2))
    if accum is not None:
        accum.copy_((_f(accum) + tot).to(accum.dtype))
        return accum
    return tot.to(dy.dtype)


def conv_wgrad(dy, x, dw, sh, sw, ph, pw, overwrite=False):
    K, R, S, C = dw.shape
    gw = torch.ops.aten.convolution_backward(
        _nchw(_f(dy)).contiguous(), _nchw(_f(x)).contiguous(),
        torch.empty(K, C, R, S, device=dy.device), None, [sh, sw], [ph, pw], [1, 1], False,
        [0, 0], 1, [False, True, False])[1]
    if overwrite:
        dw.copy_(gw.permute(0, 2, 3, 1))
    else:
        dw.add_(gw.permute(0, 2, 3, 1))


def act_bwd(dy, y, dbias):
    """g = dy * (y > 0) if y given else dy; dbias += sum_rows(g)."""
    g = dy if _opt(y) is None else (_f(dy) * (_f(y) > 0)).to(dy.dtype)
    db = _opt(dbias)
    if db is not None:
        db.add_(_f(g).reshape(-1, g.shape[-1]).sum(0))
    return g


# ------------------------------------------------------------------------------------ BN
def relu_bitmask(y):
    """uint8 [numel / 8]: bit j of byte i = (element 8 i + j of y, flattened) > 0."""
    b = (y.reshape(-1, 8) > 0).to(torch.int32)
    w = torch.tensor([1 << j for j in range(8)], dtype=torch.int32, device=y.device)
    return (b * w).sum(1).to(torch.uint8)


def bitmask_unpack(m, shape):
    """Inverse of relu_bitmask: bool tensor of ``shape``."""
    bits = torch.arange(8, device=m.device, dtype=torch.int32)
    return ((m.to(torch.int32).unsqueeze(1) >> bits) & 1).bool().reshape(shape)


def bn_stats_affine(x, stats, gamma, beta, rmean, rvar, momentum, eps, counter=None):
    """Statistics half of a train-mode BN whose apply runs in its consumer: (mean, rstd,
    [2, C] affine = [gamma rstd | beta - mean gamma rstd]); updates the running stats."""
    C = x.shape[-1]
    xf = _f(x).reshape(-1, C)
    M = xf.shape[0]
    mean = xf.mean(0)
    var = xf.var(0, unbiased=False)
    rstd = torch.rsqrt(var + eps)
    sc = gamma.float() * rstd
    with torch.no_grad():
        unbiased = var * (M / max(M - 1, 1))
        rmean.mul_(1 - momentum).add_(mean, alpha=momentum)
        rvar.mul_(1 - momentum).add_(unbiased, alpha=momentum)
        if _opt(counter) is not None:
            counter.add_(1)
    return mean, rstd, torch.stack([sc, beta.float() - mean * sc])


def bn_fwd_train(x, stats, gamma, beta, rmean, rvar, momentum, eps, residual, relu,
                 counter=None, mask=None, channels=0, res_affine=None, out=None):
    # the oracle always uses exact two-pass statistics (``stats`` from a fused producer
    # epilogue is accepted for API parity but not needed); channels > 0: BN of the first
    # ``channels`` channels of a wider buffer
    if channels:
        x = x[..., :channels]
    C = x.shape[-1]
    xf = _f(x).reshape(-1, C)
    M = xf.shape[0]
    mean = xf.mean(0)
    var = xf.var(0, unbiased=False)
    rstd = torch.rsqrt(var + eps)
    y = (xf - mean) * (rstd * gamma) + beta
    if _opt(residual) is not None:
        r = _f(residual).reshape(-1, C)
        if _opt(res_affine) is not None:  # the residual's deferred BN
            r = r * res_affine[0] + res_affine[1]
        y = y + r
    if relu:
        y = torch.relu(y)
    with torch.no_grad():
        unbiased = var * (M / max(M - 1, 1))
        rmean.mul_(1 - momentum).add_(mean, alpha=momentum)
        rvar.mul_(1 - momentum).add_(unbiased, alpha=momentum)
        if _opt(counter) is not None:
            counter.add_(1)
    y = y.reshape(x.shape).to(x.dtype)
    if _opt(mask) is not None:
        mask.copy_(relu_bitmask(y))
    if _opt(out) is not None:  # a channel window of a wider buffer
        # (through .data, like a native kernel's store: no autograd version bump of the
        # buffer the other branches' outputs are views of)
        out.data.copy_(y)
        y = out
    return y, mean.contiguous(), rstd.contiguous()


def bn_stats(x, shift=None):
    xf = _f(x).reshape(-1, x.shape[-1])
    return torch.stack([xf.mean(0), xf.var(0, unbiased=False)])


def bn_fwd_eval(x, gamma, beta, rmean, rvar, eps, residual, relu, channels=0):
    if channels:
        x = x[..., :channels]
    C = x.shape[-1]
    xf = _f(x).reshape(-1, C)
    rstd = torch.rsqrt(rvar + eps)
    y = (xf - rmean) * (rstd * gamma) + beta
    if _opt(residual) is not None:
        y = y + _f(residual).reshape(-1, C)
    if relu:
        y = torch.relu(y)
    return y.reshape(x.shape).to(x.dtype)


def bn_bwd(dy, x, y, mean, rstd, gamma, dgamma, dbeta, want_dx, want_g=True, zmask_beta=None,
           ymask=None, gacc=None, dx_out=None):
    """Returns (dx, g) where g = dy masked by ReLU (the residual-branch gradient).  The mask
    comes from ``ymask`` (bn_fwd_train's bit mask) if given, else from ``y``, else - with
    ``zmask_beta`` - is recomputed from x for y = relu(bn(x)).  x may be wider than dy (a
    channel prefix); ``gacc`` (fp32): dx is added into its first C channels instead."""
    C = dy.shape[-1]
    x = x[..., :C]
    g = _f(dy).reshape(-1, C)
    if _opt(ymask) is not None:
        g = g * bitmask_unpack(ymask, g.shape)
    elif _opt(y) is not None:
        g = g * (_f(y).reshape(-1, C) > 0)
    elif _opt(zmask_beta) is not None:
        sc = gamma * rstd
        t = (_f(x).reshape(-1, C) * sc + (zmask_beta - mean * sc)).to(torch.bfloat16).float()
        g = g * (t > 0)
    M = g.shape[0]
    xhat = (_f(x).reshape(-1, C) - mean) * rstd
    sg = g.sum(0)
    sgx = (g * xhat).sum(0)
    if _opt(dgamma) is not None:
        dgamma.add_(sgx)
    if _opt(dbeta) is not None:
        dbeta.add_(sg)
    dx = None
    if gacc is not None:
        d = (gamma * rstd) * (g - sg / M - xhat * (sgx / M))
        gacc[..., :C] += d.reshape(dy.shape)
    elif want_dx:
        dx = (gamma * rstd) * (g - sg / M - xhat * (sgx / M))
        dx = dx.reshape(dy.shape).to(dy.dtype)
        if dx_out is not None:
            dx_out.copy_(dx)
            dx = dx_out
    return dx, g.reshape(dy.shape).to(dy.dtype)


def bn_bwd_pair(dy, x, ymask, mean, rstd, gamma, dgamma, dbeta, x2, mean2, rstd2, gamma2,
                dgamma2, dbeta2):
    """Backward of relu(bn(x) + bn2(x2)), both BNs train-mode: [dx, dx2] from the shared
    g = dy * mask (kept in fp32, as the fused kernel does)."""
    C = dy.shape[-1]
    g = _f(dy).reshape(-1, C) * bitmask_unpack(ymask, (dy.numel() // C, C))
    M = g.shape[0]
    sg = g.sum(0)
    out = []
    for xx, mu, rs, ga, dga, dbe in ((x, mean, rstd, gamma, dgamma, dbeta),
                                     (x2, mean2, rstd2, gamma2, dgamma2, dbeta2)):
        xhat = (_f(xx).reshape(-1, C) - mu) * rs
        sgx = (g * xhat).sum(0)
        if _opt(dga) is not None:
            dga.add_(sgx)
        if _opt(dbe) is not None:
            dbe.add_(sg)
        d = (ga * rs) * (g - sg / M - xhat * (sgx / M))
        out.append(d.reshape(dy.shape).to(dy.dtype))
    return out


def bn_bwd_apply(dy, x, y, mean, rstd, gamma, dgamma, dbeta, sums, want_dx, want_g=True):
    """bn_bwd's apply pass with precomputed sums = [sum g | sum g*xhat]."""
    C = x.shape[-1]
    g = _f(dy).reshape(-1, C)
    if _opt(y) is not None:
        g = g * (_f(y).reshape(-1, C) > 0)
    M = g.shape[0]
    xhat = (_f(x).reshape(-1, C) - mean) * rstd
    sg, sgx = sums[:C], sums[C:]
    if _opt(dgamma) is not None:
        dgamma.add_(sgx)
    if _opt(dbeta) is not None:
        dbeta.add_(sg)
    dx = None
    if want_dx:
        dx = ((gamma * rstd) * (g - sg / M - xhat * (sgx / M))).reshape(x.shape).to(dy.dtype)
    return dx, g.reshape(x.shape).to(dy.dtype)


def conv_bnred_ok(K, C):
    return True


def conv_dgrad_bnred(dy, w, H, W, sh, sw, ph, pw, wt, z, y, mean, rstd, gamma=None, beta=None):
    """dgrad fused with the backward reduction of the ReLU(BN) that produced the conv
    input: returns (g = dx * (y > 0), [sum g | sum g * xhat]).  Without y, the mask is
    recomputed from z with the forward's affine (gamma, beta) - the halo kernel's form
    (y is the same mask when it is the forward's output)."""
    dx = conv_dgrad(dy, w, H, W, sh, sw, ph, pw)
    C = dx.shape[-1]
    g = _f(dx).reshape(-1, C)
    if _opt(y) is not None:
        g = g * (_f(y).reshape(-1, C) > 0)
    elif gamma is not None and beta is not None:
        sc = gamma.float() * rstd
        sh_ = beta.float() - mean * sc
        live = (_f(z).reshape(-1, C) * sc + sh_).to(torch.bfloat16).float() > 0
        g = g * live
    xhat = (_f(z).reshape(-1, C) - mean) * rstd
    sums = torch.cat([g.sum(0), (g * xhat).sum(0)])
    return g.reshape(dx.shape).to(dx.dtype), sums


def conv_dgrad_bnred_gacc(dz, w, wt, zbuf, mean, rstd, gamma, beta, G):
    """1x1 / stride-1 dgrad fused with the backward of the ReLU(BN) that produced its input
    (a DenseNet norm1 over the block buffer's first Ci channels): G[..., :Ci] += gamma*rstd *
    g with g the masked dgrad (no dy tensor); returns [sum g | sum g * xhat].  The rest of
    the BN backward is deferred to bn_defer_step."""
    Ci = w.shape[-1]
    N, H, W_ = dz.shape[:3]
    dx = conv_dgrad(dz, w, H, W_, 1, 1, 0, 0)
    g = _f(dx).to(dz.dtype).float().reshape(-1, Ci)  # the kernel rounds dy to bf16 first
    z = _f(zbuf[..., :Ci]).reshape(-1, Ci)
    sc = gamma.float()[:Ci] * rstd[:Ci]
    sh_ = beta.float()[:Ci] - mean[:Ci] * sc
    g = g * ((z * sc + sh_).to(torch.bfloat16).float() > 0)
    xhat = (z - mean[:Ci]) * rstd[:Ci]
    Gv = G[..., :Ci]
    Gv.copy_((Gv.float() + (sc * g).reshape(Gv.shape)).to(G.dtype))
    return torch.cat([g.sum(0), (g * xhat).sum(0)])


def bn_defer_step(sums, gamma, mean, rstd, s0, k12, dgamma, dbeta, G, x, out=None):
    """Fold a dense layer's norm1 sums into the block's deferred corrections k12 [2, Ctot]
    (channels < s0) and the (gamma, beta) gradients, and apply the final correction
    G += K1 + K2 * xhat to the channels [s0, Ci)."""
    Ci = sums.numel() // 2
    M = x.numel() // x.shape[-1]
    sg, sgx = sums[:Ci], sums[Ci:]
    if _opt(dgamma) is not None:
        dgamma.add_(sgx)
    if _opt(dbeta) is not None:
        dbeta.add_(sg)
    a = gamma.float()[:Ci] * rstd[:Ci]
    t1, t2 = -a * sg / M, -a * sgx / M
    k1 = k12[0, s0:Ci] + t1[s0:]
    k2 = k12[1, s0:Ci] + t2[s0:]
    k12[0, :s0] += t1[:s0]
    k12[1, :s0] += t2[:s0]
    xs = _f(x[..., s0:Ci])
    xhat = (xs - mean[s0:Ci]) * rstd[s0:Ci]
    Gv = G[..., s0:Ci]
    fin = (Gv.float() + k1 + k2 * xhat).to(G.dtype)
    if out is not None and out.numel():  # the consumer's copy only (G's is never read again)
        out.copy_(fin.to(out.dtype))
    else:
        Gv.copy_(fin)


def conv_fwd_into(x, w, bias, sh, sw, ph, pw, relu, stats, shift, out):
    """conv_fwd writing into ``out`` (a channel window of a wider buffer); ``stats`` may be
    a [2, K] window of a wider table."""
    st = _opt(stats)
    tmp = torch.empty(2, w.shape[0], dtype=torch.float32) if st is not None else stats
    y = conv_fwd(x, w, bias, sh, sw, ph, pw, relu, tmp, shift)
    out.copy_(y)
    if st is not None:
        st.copy_(tmp)


# ---------------------------------------------------------------------------------- pool
def _pool_out(H, k, s, p, ceil):
    if ceil:
        o = -(-(H + 2 * p - k) // s) + 1
        if (o - 1) * s >= H + p:
            o -= 1
    else:
        o = (H + 2 * p - k) // s + 1
    return o


def maxpool_fwd(x, kh, kw, sh, sw, ph, pw, ceil):
    y, idx = F.max_pool2d(_nchw(_f(x)), (kh, kw), (sh, sw), (ph, pw), ceil_mode=ceil,
                          return_indices=True)
    return _nhwc(y).to(x.dtype), _nhwc(idx.to(torch.int32))


def maxpool_bwd(dy, idx, H, W, kh, kw, sh, sw, ph, pw, ceil):
    N, P, Q, C = dy.shape
    out = torch.zeros(N, C, H * W, device=dy.device, dtype=torch.float32)
    out.scatter_add_(2, _nchw(idx).reshape(N, C, -1).long(), _nchw(_f(dy)).reshape(N, C, -1))
    return _nhwc(out.reshape(N, C, H, W)).to(dy.dtype)


def maxpool_bwd_relu(dy, idx, y, H, W, kh, kw, sh, sw, ph, pw):
    """Max-pool backward of a ReLU output handed over by its producer: the gradient routes
    only where the pooled value is > 0; returns (dx, per-channel sum of the routed
    gradient), or None when the fused kernel would not apply (not a 2x2/s2/p0 pool)."""
    if not (kh == kw == sh == sw == 2 and ph == pw == 0 and H % 2 == 0 and W % 2 == 0):
        return None
    g = _f(dy) * (_f(y) > 0)
    dx = maxpool_bwd(g, idx, H, W, kh, kw, sh, sw, ph, pw, False).to(dy.dtype)
    return dx, g.reshape(-1, g.shape[-1]).sum(0)


def bn_relu_maxpool_fwd(z, stats, gamma, beta, rmean, rvar, momentum, eps, kh, kw, sh, sw, ph,
                        pw, ceil, counter=None, zsel_out=None):
    y, mean, rstd = bn_fwd_train(z, stats, gamma, beta, rmean, rvar, momentum, eps, None, True,
                                 counter)
    p, idx = maxpool_fwd(y, kh, kw, sh, sw, ph, pw, ceil)
    if zsel_out is not None:  # raw z at each window's argmax
        N, H, W, C = z.shape
        flat = _nchw(idx).reshape(N, C, -1).long()  # ATen's flat h * W + w argmax
        zs = _nchw(z).reshape(N, C, -1).gather(2, flat)
        zsel_out.copy_(_nhwc(zs.reshape(N, C, p.shape[1], p.shape[2])))
    return p, idx, mean, rstd


def maxpool_bn_bwd(dp, idx, z, mean, rstd, gamma, beta, dgamma, dbeta, kh, kw, sh, sw, ph, pw,
                   zsel=None):
    N, H, W, C = z.shape
    g = maxpool_bwd(dp, idx, H, W, kh, kw, sh, sw, ph, pw, False)
    # ReLU mask recomputed from z: bn(z) > 0
    y = (_f(z) - mean) * (rstd * gamma) + beta
    dz, _ = bn_bwd(g, z, y, mean, rstd, gamma, dgamma, dbeta, True, False)
    return dz


def maxpool_bn_bwd_sums(dp, zsel, mean, rstd, gamma, beta, dgamma, dbeta):
    """Pooled-only half of the fused stem backward: [sum g | sum g xhat] with g the pooled
    gradient masked by bn(zsel) > 0 (zsel = raw z at each argmax); adds dgamma / dbeta."""
    C = dp.shape[-1]
    z = _f(zsel).reshape(-1, C)
    g = _f(dp).reshape(-1, C) * ((z - mean) * (rstd * gamma) + beta > 0)
    sg, sgx = g.sum(0), (g * ((z - mean) * rstd)).sum(0)
    if _opt(dgamma) is not None:
        dgamma.add_(sgx)
    if _opt(dbeta) is not None:
        dbeta.add_(sg)
    return torch.cat([sg, sgx])


def stem_pool_wgrad_ok(dp, idx, z, x, dw, sh, sw, ph, pw):
    return True


def stem_pool_wgrad(dp, idx, z, mean, rstd, gamma, beta, sums, x, dw, sh, sw, ph, pw,
                    overwrite=False):
    """Weight gradient of conv -> BN -> ReLU -> 3x3/s2/p1 max-pool from the pooled gradient:
    dz = a g + b + cco z (the BN backward with the pooled ``sums``), rounded to the
    activation dtype as the two-pass form stores it, then the conv weight gradient."""
    N, H, W, C = z.shape
    g = _f(maxpool_bwd(dp, idx, H, W, 3, 3, 2, 2, 1, 1, False)).reshape(-1, C)
    zf = _f(z).reshape(-1, C)
    g = g * ((zf - mean) * (rstd * gamma) + beta > 0)
    M = g.shape[0]
    a = gamma * rstd
    cco = -a * rstd * sums[C:] / M
    b = -a * sums[:C] / M - cco * mean
    dz = (a * g + b + cco * zf).reshape(z.shape).to(z.dtype)
    conv_wgrad(dz, x, dw, sh, sw, ph, pw, overwrite)


def avgpool_fwd(x, kh, kw, sh, sw, ph, pw, ceil, count_include_pad):
    y = F.avg_pool2d(_nchw(_f(x)), (kh, kw), (sh, sw), (ph, pw), ceil_mode=ceil,
                     count_include_pad=count_include_pad)
    return _nhwc(y).to(x.dtype)


def avgpool_bwd(dy, H, W, kh, kw, sh, sw, ph, pw, ceil, count_include_pad, dx_out=None):
    N, P, Q, C = dy.shape
    xin = torch.zeros(N, C, H, W, device=dy.device, requires_grad=True)
    with torch.enable_grad():
        y = F.avg_pool2d(xin, (kh, kw), (sh, sw), (ph, pw), ceil_mode=ceil,
                         count_include_pad=count_include_pad)
        (gx,) = torch.autograd.grad(y, xin, _nchw(_f(dy)))
    gx = _nhwc(gx).to(dy.dtype)
    if dx_out is not None:
        dx_out.copy_(gx)
        return dx_out
    return gx


def bn_relu_avgpool2_fwd(z, aff):
    """avg_pool2d(relu(z * aff[0] + aff[1]), 2, 2) over NHWC z."""
    y = torch.relu(_f(z) * aff[0] + aff[1])
    return _nhwc(F.avg_pool2d(_nchw(y), 2, 2)).to(z.dtype)


def adaptive_avgpool_fwd(x, oh, ow):
    return _nhwc(F.adaptive_avg_pool2d(_nchw(_f(x)), (oh, ow))).to(x.dtype)


def adaptive_avgpool_bwd(dy, H, W):
    N, P, Q, C = dy.shape
    xin = torch.zeros(N, C, H, W, device=dy.device, requires_grad=True)
    with torch.enable_grad():
        y = F.adaptive_avg_pool2d(xin, (P, Q))
        (gx,) = torch.autograd.grad(y, xin, _nchw(_f(dy)))
    return _nhwc(gx).to(dy.dtype)


# ------------------------------------------------------------------------------- linear
def linear_fwd(x, w, bias, relu):
    y = _f(x) @ _f(w).t()
    if _opt(bias) is not None:
        y = y + _f(bias)
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype)


def linear_dgrad(dy, w, wt=None):
    return (_f(dy) @ _f(w)).to(dy.dtype)


def linear_wgrad(dy, x, dw, overwrite=False):
    if overwrite:
        dw.copy_(_f(dy).t() @ _f(x))
    else:
        dw.add_(_f(dy).t() @ _f(x))


# --------------------------------------------------------------------------- loss / acc
def ce_fwd(logits, labels):
    lf = _f(logits)
    lse = torch.logsumexp(lf, dim=1)
    picked = lf.gather(1, labels.view(-1, 1).long()).squeeze(1)
    loss = (lse - picked).mean().reshape(1)
    return loss, lse


def ce_bwd(logits, labels, lse, grad_out, weight=1.0):
    B = logits.shape[0]
    p = torch.exp(_f(logits) - lse[:, None])
    p[torch.arange(B, device=logits.device), labels.long()] -= 1.0
    return (p * (_f(grad_out).reshape(()) * weight / B)).to(logits.dtype)


def ce_fwd_weighted(logits, labels, out, acc, weight, accumulate):
    loss, lse = ce_fwd(logits, labels)
    v = loss.reshape(1) * weight
    if accumulate:
        out[:1] += v
    else:
        out[:1] = v
    if acc is not None and acc.numel() > 0:
        acc[:1] += v
    return lse


def zero_f32(t):
    t.zero_()


def step_inc(step):
    step.add_(1.0)


def argmax_correct(logits, labels, count):
    pred = _f(logits).argmax(1)
    count.add_((pred == labels.long()).sum().to(count.dtype))


# ----------------------------------------------------------------------------- optimizer
def adam_step(master, grad, m, v, shadow, step_t, lr, b1, b2, eps, wd, grad_scale):
    step = float(step_t.item()) + 1.0
    g = grad * grad_scale
    if wd != 0.0:
        g = g + wd * master
    m.mul_(b1).add_(g, alpha=1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    master.addcdiv_(m, denom, value=-lr / bc1)
    if _opt(shadow) is not None:
        shadow.copy_(master)


def sgd_step(master, grad, buf, shadow, step_t, lr, momentum, dampening, wd, nesterov, grad_scale):
    first = float(step_t.item()) == 0.0
    g = grad * grad_scale
    if wd != 0.0:
        g = g + wd * master
    if momentum != 0.0:
        if first:
            buf.copy_(g)
        else:
            buf.mul_(momentum).add_(g, alpha=1 - dampening)
        g = g + momentum * buf if nesterov else buf
    master.add_(g, alpha=-lr)
    if _opt(shadow) is not None:
        shadow.copy_(master)


# ------------------------------------------------------------------------ preprocessing
def preprocess(img_u8, oh, ow, mean, std, mode, cpad, out_dtype, pad=None, extents=None):
    """u8 NHWC [B,H,W,3] -> normalized NHWC [B,oh,ow,cpad] (zero padded channels), on a
    zero-bordered canvas when pad = (top, bottom, left, right).

    mode 0: bilinear, no antialias  (train path: ToTensor -> Resize on tensor, main.py:62-65)
    mode 1: PIL bicubic (antialiased, 8-bit fixed point) -> u8 -> ToTensor -> Normalize
            (eval path, evaluation_pipeline.py:89,116-122): data/pil_resize.py, bit-exact
            with PIL.Image.resize
    mode 2: float bicubic with antialias (F.interpolate semantics)
    extents: image b occupies [:h_b, :w_b] of its slot.
    """
    if extents is not None:
        parts = [preprocess(img_u8[b:b + 1, :int(h), :int(w)], oh, ow, mean, std, mode, cpad,
                            out_dtype, pad) for b, (h, w) in enumerate(extents)]
        return torch.cat(parts, 0)
    if mode == 1:
        from ..data import pil_resize
        x = torch.from_numpy(pil_resize.reference(img_u8.cpu().numpy(), (oh, ow), mean, std))
        x = x.to(img_u8.device)
    else:
        x = _nchw(img_u8.float() / 255.0)
        if (oh, ow) != tuple(x.shape[-2:]):
            if mode == 0:
                x = F.interpolate(x, size=(oh, ow), mode="bilinear", align_corners=False)
            else:
                x = F.interpolate(x, size=(oh, ow), mode="bicubic", align_corners=False,
                                  antialias=True)
        m = torch.tensor(mean, device=x.device).view(1, 3, 1, 1)
        s = torch.tensor(std, device=x.device).view(1, 3, 1, 1)
        x = _nhwc((x - m) / s)
    if cpad > 3:
        x = F.pad(x, (0, cpad - 3))
    if pad:
        t, b, l, r = pad
        x = F.pad(x, (0, 0, l, r, t, b))
    return x.to(out_dtype)


# ---------------------------------------------------------------------------- dropout
def dropout_fwd(x, p, seed, offset):
    g = torch.Generator(device=x.device)
    g.manual_seed(int(seed) * 1000003 + int(offset))
    keep = (torch.rand(x.shape, generator=g, device=x.device) >= p)
    y = (_f(x) * keep / (1 - p)).to(x.dtype)
    return y, keep.to(torch.uint8)


def dropout_bwd(dy, mask, p):
    return (_f(dy) * mask.float() / (1 - p)).to(dy.dtype)


def concat_channels(xs):
    return torch.cat(list(xs), dim=-1)


def split_channels(dy, sizes):
    return [t.contiguous() for t in torch.split(dy, list(sizes), dim=-1)]


def chan_accum(g, off, src, assign):
    cs = src.shape[-1]
    if assign:
        g[..., off:off + cs] = src.float()
    else:
        g[..., off:off + cs] += src.float()


def zero_cols_f32(t, period, first, count):
    t.view(-1, period)[:, first:first + count] = 0


def add_bf16_(a, b):
    a.add_(b)


def add_f32_(dst, src):
    dst.add_(src)


def chan_slice(src, off, cs):
    return src[..., off:off + cs].clone()


def chan_insert(dst, off, src):
    dst.data[..., off:off + src.shape[-1]] = src


def chan_extract(g, off, cs):
    return g[..., off:off + cs].clone()


def relu_fwd(x):
    return torch.relu(x)
