"""DenseNet-121, NHWC, torchvision parameter names.

Reference: ``models.densenet121`` with ``classifier = nn.Linear(1024, num_classes)``
(``/root/reference/models.py:74-81``).  Pre-activation layers: BN+ReLU run as one fused
kernel over the concatenated features (channel concat = last-dim concat in NHWC).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from .layers import (Conv2d, BatchNorm2d, Linear, MaxPool2d, AvgPool2d, AdaptiveAvgPool2d,
                     ReLU)
from ..ops import functional as Fn


class _DenseLayer(nn.Module):
    def __init__(self, num_input_features, growth_rate, bn_size):
        super().__init__()
        self.norm1 = BatchNorm2d(num_input_features)
        self.relu1 = ReLU(True)
        self.conv1 = Conv2d(num_input_features, bn_size * growth_rate, 1, bias=False)
        self.norm2 = BatchNorm2d(bn_size * growth_rate)
        self.relu2 = ReLU(True)
        self.conv2 = Conv2d(bn_size * growth_rate, growth_rate, 3, 1, 1, bias=False)

    def forward(self, feats):
        x = feats[0] if len(feats) == 1 else Fn.cat_channels(feats)
        return self.tail(self.norm1(x, relu=True))

    def tail(self, x, stats=None, shift=None, link=None, out=None):
        """conv1 -> norm2 -> relu -> conv2 of the normalised input; ``stats`` receives the
        output's [mean | var] from conv2's epilogue; ``link`` (Fn.BNLink) describes norm1 for
        the fused conv1-dgrad / norm1-backward hand-off; ``out``: a channel window of the
        block buffer conv2 writes into."""
        z = Fn.conv_bn_act(x, self.conv1, self.norm2, relu=True, link_in=link)
        if stats is None:
            return self.conv2(z)
        return Fn.conv_act(z, self.conv2, stats=stats, shift=shift, out=out)


# MPA_DENSE_BLOCK_GRAD=0: per-layer concats under plain autograd (one split and one
# elementwise add per earlier feature and layer) instead of the block feature buffer
_BLOCK_GRAD = os.environ.get("MPA_DENSE_BLOCK_GRAD", "1") == "1"
# The block gradient accumulator holds activation gradients, which are bf16 everywhere in
# this engine: each contribution is added in fp32 and rounded once (the GradJoin policy;
# autograd's own bf16 sums of the concat's split do the same).  Same-box A/B, batch 256:
# 6652 img/s vs 6413 with an fp32 accumulator (twice the accumulator traffic).
# MPA_DENSE_GRAD_BF16=0 keeps the accumulator in fp32.
_GRAD_BF16 = os.environ.get("MPA_DENSE_GRAD_BF16", "1") == "1"
# Deferred norm1 backward (see _DenseBlockGrad.backward): conv1's dgrad epilogue adds
# gamma*rstd * g into the block gradient and reduces (sum g, sum g*xhat); the per-channel
# rest of every layer's BN backward is summed and applied once per channel.  No dy
# tensor, no norm1 reduce / apply passes over the O(L^2) channel prefixes.
# MPA_DENSE_DEFER=0 restores the per-layer bn_bwd(gacc=G).
_DEFER = os.environ.get("MPA_DENSE_DEFER", "1") == "1"
# conv2 writes each new feature (and its statistics) into the block buffer / table in place,
# and bn_defer_step hands the finished gradient slice to its consumer - no channel inserts
# or slice copies.  MPA_DENSE_DIRECT=0 restores the copies.
_DIRECT = os.environ.get("MPA_DENSE_DIRECT", "1") == "1"
# Transition: average-pool before the 1x1 conv (MPA_DENSE_POOL_FIRST=0: torchvision order)
_POOL_FIRST = os.environ.get("MPA_DENSE_POOL_FIRST", "1") == "1"
# ... and its norm + ReLU applied inside the pool pass (MPA_DENSE_FUSE_POOL=0: separate)
_FUSE_POOL = os.environ.get("MPA_DENSE_FUSE_POOL", "1") == "1"


# MPA_DENSE_WALK=0: each layer's backward as a nested torch.autograd.backward call
_WALK = os.environ.get("MPA_DENSE_WALK", "1") == "1"


def _chain_nodes(out: torch.Tensor, leaf: torch.Tensor):
    """The backward nodes from ``out`` to ``leaf`` when the layer's graph is a chain of
    custom Functions along their first input (conv2 <- conv1+norm2 <- leaf; the parameter
    inputs take no autograd gradient, the kernels write the arena); None otherwise."""
    nodes, node = [], out.grad_fn
    for _ in range(4):
        if node is None:
            return None
        if type(node).__name__ == "AccumulateGrad":
            return nodes if node.variable is leaf else None
        if not hasattr(node, "_forward_cls") or not node.next_functions:
            return None
        nodes.append(node)
        node = node.next_functions[0][0]
    return None


def _walk_backward(nodes, g):
    """Run a layer's backward by calling its nodes directly (see _chain_nodes): the nested
    engine pass per layer (graph task, dependency scan, reentrant dispatch) is host time
    a 58-layer DenseNet pays 58 times per step.  Returns the leaf's gradient."""
    for node in nodes:
        r = node.apply(g)
        g = r[0] if isinstance(r, tuple) else r
    return g


def _window(buf: torch.Tensor, c0: int, n: int) -> torch.Tensor:
    """buf[..., c0:c0 + n] as a plain alias of buf's storage, not an autograd view: conv2's
    custom Function returns it as its output, and the other layers' writes into buf must
    not count as in-place modifications of that output's base."""
    v = buf[..., c0:c0 + n]
    return torch.empty(0, dtype=buf.dtype, device=buf.device).set_(
        buf.untyped_storage(), v.storage_offset(), v.shape, v.stride())


def _defer_ok(c0: int, growth: int) -> bool:
    """bn_defer_step's slice shapes: 8-channel groups whose count divides 256."""
    return all(n % 8 == 0 and 256 % (n // 8) == 0 for n in (c0, growth))


class _DenseBlock(nn.ModuleDict):
    def __init__(self, num_layers, num_input_features, bn_size, growth_rate):
        super().__init__()
        for i in range(num_layers):
            self.add_module("denselayer%d" % (i + 1),
                            _DenseLayer(num_input_features + i * growth_rate, growth_rate,
                                        bn_size))

    def forward(self, x, fused: bool = True):
        """Returns (block output, its per-channel [mean | var] or None)."""
        if fused and _BLOCK_GRAD:
            if self.training and torch.is_grad_enabled() and x.requires_grad:
                # (the module walk of parameters() costs ~1 ms of host time per step over
                # the four blocks: the list is taken once, requires_grad read each step)
                ps = self.__dict__.get("_mpa_params")
                if ps is None:
                    ps = self.__dict__["_mpa_params"] = tuple(self.parameters())
                params = [p for p in ps if p.requires_grad]
                out = _DenseBlockGrad.apply(x, self, *params)
                return out, self.__dict__.pop("_stats", None)
            if not self.training and not (torch.is_grad_enabled() and x.requires_grad):
                return _block_eval(self, x), None  # (raw kernels: inference only)
        feats = [x]
        for layer in self.values():
            feats.append(layer(feats))
        return Fn.cat_channels(feats), None


def _growth(block) -> int:
    return next(iter(block.values())).conv2.weight.shape[0]


def _block_eval(block, x):
    """Eval forward on the block feature buffer: each layer's norm1 reads its input as the
    buffer's channel prefix (bn_fwd_eval(channels=C_i)), its output is inserted at its
    channel offset - no per-layer concat."""
    k = Fn.K(x)
    layers = list(block.values())
    c0 = x.shape[-1]
    buf = x.new_empty(x.shape[:-1] + (c0 + _growth(block) * len(layers),))
    k.chan_insert(buf, 0, x)
    ci = c0
    for layer in layers:
        n1 = layer.norm1
        y1 = k.bn_fwd_eval(buf, n1.weight, n1.bias, n1.running_mean, n1.running_var, n1.eps,
                           Fn._empty(x), True, channels=ci)
        out = layer.tail(y1)
        k.chan_insert(buf, ci, out)
        ci += out.shape[-1]
    return buf


class _DenseBlockGrad(torch.autograd.Function):
    """A dense block on ONE feature buffer, with ONE gradient accumulator G (bf16 by default,
    each contribution added in fp32 and rounded once; fp32 with MPA_DENSE_GRAD_BF16=0).
    Pinned against the fp32 accumulator over whole DenseNet-121 blocks (6 and 24 layers):
    block-input and parameter gradients agree to cosine >= 0.999 and a bounded max-relative
    error (tests/test_grouped_gpu.py::test_densenet_bf16_block_gradient_accumulator).

    Forward: the block input and every layer's 32-channel output live in a buffer
    [N, H, W, C_total] at their channel offsets (``chan_insert``), so layer i reads its
    input as the buffer's first C_i channels - no per-layer concat (the O(L^2) copies of
    torchvision's ``torch.cat(prev_features, 1)``).  Every feature's batch
    statistics are taken ONCE when it is produced (``bn_stats`` of the new 32 channels)
    into a block statistics table S [2, C_total]; each layer's norm1 (a different affine and
    running-stat update per layer, as in the reference) then normalises its prefix from S
    (``bn_fwd_train(channels=C_i)``) with no statistics pass.  The table also serves the
    transition / final norm that reads the whole block output.  The rest of each layer
    (conv1 -> norm2 -> relu -> conv2) runs as its own small autograd graph from a leaf on
    the normalised input.

    Backward: G = the block gradient in fp32 [..., C_total].  In reverse layer order, layer
    i's output gradient is read from G (``chan_extract``), its graph back-propagated to the
    leaf, and norm1's backward (reduce + apply on the buffer prefix, ReLU mask recomputed
    from the buffer) ADDS its input gradient straight into G's first C_i channels in fp32
    (``bn_bwd(gacc=G)``): no bf16 dx, no separate accumulate pass.  Parameter gradients land
    in the flat arena from the layers' own kernels.

    Reference: ``_DenseBlock`` / ``_DenseLayer`` of torchvision densenet121 reached from
    ``/root/reference/models.py:74-81``."""

    @staticmethod
    def forward(ctx, x, block, *params):
        k = Fn.K(x)
        layers = list(block.values())
        c0 = x.shape[-1]
        ctot = c0 + _growth(block) * len(layers)
        x = x.detach().contiguous()
        buf = x.new_empty(x.shape[:-1] + (ctot,))
        S = torch.empty(2, ctot, dtype=torch.float32, device=x.device)
        k.chan_insert(buf, 0, x)
        # shift for the sums: the consuming norm's running mean (any nearby value will do)
        k.chan_insert(S, 0, k.bn_stats(x, layers[0].norm1.running_mean[:c0]))
        recs = []
        ci = c0
        defer = _DEFER and _defer_ok(c0, _growth(block))
        for li, layer in enumerate(layers):
            n1 = layer.norm1
            y1, mean, rstd = k.bn_fwd_train(buf, S, n1.weight, n1.bias, n1.running_mean,
                                            n1.running_var, n1.momentum_value(), n1.eps,
                                            Fn._empty(x), True, n1.num_batches_tracked,
                                            channels=ci)
            leaf = y1.requires_grad_(True)
            g = layer.conv2.weight.shape[0]
            # conv2 writes its output and its statistics straight into the buffer / table
            direct = _DIRECT and g % 8 == 0
            st = S[:, ci:ci + g] if direct else torch.empty(2, g, dtype=torch.float32,
                                                             device=x.device)
            nxt = layers[li + 1].norm1.running_mean[ci:ci + g] if li + 1 < len(layers) else None
            link = None
            if defer and n1.weight is not None and n1.bias is not None:
                link = Fn.BNLink()  # norm1 = ReLU(BN) of buf[..., :ci] (z-mask form)
                link.z, link.mean, link.rstd = buf, mean, rstd
                link.gamma, link.beta = n1.weight, n1.bias
            with torch.enable_grad():  # the new feature's statistics from conv2's epilogue
                out = layer.tail(leaf, st, nxt, link, _window(buf, ci, g) if direct else None)
            if not direct:
                k.chan_insert(buf, ci, out.detach())
                k.chan_insert(S, ci, st)
            recs.append((leaf, out, mean, rstd, ci, link))
            ci += g
        ctx.block = block
        ctx.recs = recs
        ctx.buf = buf
        ctx.c0 = c0
        ctx.nparams = len(params)
        block._stats = S
        return buf

    @staticmethod
    def backward(ctx, gy):
        k = Fn.K(gy)
        gy = gy.contiguous()
        buf = ctx.buf
        layers = list(ctx.block.values())
        if _GRAD_BF16:
            # the block output's gradient comes from its one consumer's BN backward (the
            # transition / norm5: bn_bwd returns a fresh dx that nothing else references)
            # as a fresh tensor: accumulate into it in place; a view or a non-bf16 gradient
            # is copied first
            G = gy if (gy._base is None and gy.dtype == torch.bfloat16) else gy.clone()
        else:
            G = torch.empty(gy.shape, dtype=torch.float32, device=gy.device)
            k.chan_accum(G, 0, gy, True)
        # deferred corrections K1 | K2 per channel (see bn_defer_step)
        k12 = None
        if any(r[5] is not None for r in ctx.recs):
            k12 = torch.empty(2, G.shape[-1], dtype=torch.float32, device=G.device)
            k.zero_f32(k12)
        ready = dx_ready = None  # finished slices handed over by bn_defer_step
        for i in range(len(ctx.recs) - 1, -1, -1):
            leaf, out, mean, rstd, ci, link = ctx.recs[i]
            g = out.shape[-1]
            if ready is not None:
                g_out, ready = ready, None
            else:
                g_out = (k.chan_slice(G, ci, g) if _GRAD_BF16 else
                         k.chan_extract(G, ci, g).to(out.dtype))
            if link is not None:
                link.gacc = G
            nodes = _chain_nodes(out, leaf) if _WALK else None
            if nodes is not None:
                dy = _walk_backward(nodes, g_out)
            else:
                torch.autograd.backward(out, g_out)
                dy = leaf.grad
            n1 = layers[i].norm1
            gamma, beta = n1.weight, n1.bias
            if link is not None and link.sums is not None:
                # conv1's dgrad added gamma*rstd * g into G[..., :ci]; fold this layer's
                # corrections and finish the channels no earlier layer reads: layer i-1's
                # output (ci - growth .. ci), or the block input for layer 0
                s0 = 0 if i == 0 else ci - ctx.recs[i - 1][1].shape[-1]
                nxt = None
                if _DIRECT and _GRAD_BF16:  # the finished slice, contiguous, for its consumer
                    nxt = G.new_empty(G.shape[:-1] + (ci - s0,))
                k.bn_defer_step(link.sums, gamma, mean, rstd, s0, k12, Fn._sink(gamma, G),
                                Fn._sink(beta, G), G, buf, nxt)
                if i > 0:
                    ready = nxt
                else:
                    dx_ready = nxt
                link.sums = link.gacc = link.z = None
            elif link is not None:
                raise RuntimeError("dense block: conv1's fused BN-backward hand-off did not run "
                                   "(MPA_DENSE_DEFER=0 selects the per-layer form)")
            elif dy is not None:
                k.bn_bwd(dy.contiguous(), buf, Fn._empty(dy), mean, rstd, gamma,
                         Fn._sink(gamma, dy), Fn._sink(beta, dy), True, False, beta, gacc=G)
            Fn._done(gamma, beta)
            ctx.recs[i] = None
        if dx_ready is not None:
            dx = dx_ready
        else:
            dx = (k.chan_slice(G, 0, ctx.c0) if _GRAD_BF16 else
                  k.chan_extract(G, 0, ctx.c0).to(gy.dtype))
        ctx.buf = None
        return (dx, None) + (None,) * ctx.nparams


class _Transition(nn.Sequential):
    def __init__(self, num_input_features, num_output_features):
        super().__init__()
        self.norm = BatchNorm2d(num_input_features)
        self.relu = ReLU(True)
        self.conv = Conv2d(num_input_features, num_output_features, 1, bias=False)
        self.pool = AvgPool2d(2, 2)

    def forward(self, x, stats=None):
        """norm -> relu -> conv1x1 -> avgpool2x2 as torchvision, with the (linear) average
        pool commuted ahead of the (linear, bias-free) 1x1 conv: the same function, and the
        conv's forward / dgrad / wgrad run on a quarter of the pixels (the pool then sees
        the wider input - 2x the channels - which costs far less)."""
        if _POOL_FIRST and _FUSE_POOL and self.norm.training:
            # BN + ReLU applied while pooling: the normalized activation is never written
            return self.conv(Fn.bn_relu_avgpool2(x, self.norm, stats))
        x = self.norm(x, relu=True, stats=stats)
        if _POOL_FIRST:
            return self.conv(self.pool(x))
        return self.pool(self.conv(x))


class DenseNet(nn.Module):
    def __init__(self, growth_rate=32, block_config=(6, 12, 24, 16), num_init_features=64,
                 bn_size=4, num_classes=1000):
        super().__init__()
        self.features = nn.Sequential()
        self.features.add_module("conv0", Conv2d(3, num_init_features, 7, 2, 3, bias=False))
        self.features.add_module("norm0", BatchNorm2d(num_init_features))
        self.features.add_module("relu0", ReLU(True))
        self.features.add_module("pool0", MaxPool2d(3, 2, 1))
        nf = num_init_features
        for i, nl in enumerate(block_config):
            self.features.add_module("denseblock%d" % (i + 1),
                                     _DenseBlock(nl, nf, bn_size, growth_rate))
            nf = nf + nl * growth_rate
            if i != len(block_config) - 1:
                self.features.add_module("transition%d" % (i + 1), _Transition(nf, nf // 2))
                nf = nf // 2
        self.features.add_module("norm5", BatchNorm2d(nf))
        self.classifier = Linear(nf, num_classes)
        self.avgpool = AdaptiveAvgPool2d((1, 1))
        # dense blocks on one feature buffer (_DenseBlockGrad / _block_eval); utils/parity.py
        # turns it off to hook every _DenseLayer as a unit
        self.fused_blocks = True
        for m in self.modules():
            if isinstance(m, Conv2d):
                m.init_(nn.init.kaiming_normal_)
            elif isinstance(m, Linear):
                nn.init.zeros_(m.bias)

    def forward(self, x):
        f = self.features
        x = Fn.conv_bn_relu_maxpool(x, f.conv0, f.norm0, f.pool0)
        stats = None  # [mean | var] of x when the block that produced it already has them
        for name, m in f.named_children():
            if name.startswith("denseblock"):
                x, stats = m(x, self.fused_blocks)
            elif name.startswith("transition"):
                x, stats = m(x, stats), None
        # features.norm5 then F.relu (torchvision densenet forward)
        x = f.norm5(x, relu=True, stats=stats)
        x = self.avgpool(x).reshape(x.shape[0], -1)
        return self.classifier(x)


def densenet121(num_classes: int = 1000) -> DenseNet:
    return DenseNet(32, (6, 12, 24, 16), 64, num_classes=num_classes)
