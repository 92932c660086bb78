"""Inception-v3 with auxiliary head, NHWC, torchvision parameter names.

Reference: ``models.inception_v3`` with ``AuxLogits.fc`` and ``fc`` replaced by
``nn.Linear(., num_classes)`` (``/root/reference/models.py:83-95``).  In train mode the
model returns ``(logits, aux_logits)``; the trainer uses ``loss = CE(logits) + 0.4 *
CE(aux)`` - the reference feeds the tuple straight into ``criterion`` (``main.py:149-150``)
which cannot work; this is the documented fix.  Every BasicConv2d
(conv + BN(eps=1e-3) + ReLU) is one fused op; asymmetric 1x7/7x1/1x3/3x1 kernels go
through the same implicit-GEMM engine via its tap table.
"""
from __future__ import annotations

import os
from collections import namedtuple

import torch
import torch.nn as nn

from .layers import (Conv2d, BatchNorm2d, Linear, MaxPool2d, AdaptiveAvgPool2d, Dropout)
from ..ops import functional as Fn

# MPA_GRAD_JOIN=0: autograd's elementwise adds sum the branch gradients of a block input
_JOIN = os.environ.get("MPA_GRAD_JOIN", "1") == "1"

InceptionOutputs = namedtuple("InceptionOutputs", ["logits", "aux_logits"])


class BasicConv2d(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0):
        super().__init__()
        self.conv = Conv2d(in_channels, out_channels, kernel_size, stride, padding, bias=False)
        self.bn = BatchNorm2d(out_channels, eps=0.001)

    def forward(self, x, join=None, out=None, link_in=None, link_out=None):
        return Fn.conv_bn_act(x, self.conv, self.bn, relu=True, join_x=join, out=out,
                              link_in=link_in, link_out=link_out)


# MPA_INC_LINK=0: the BasicConv2d chains inside a branch run each BN's own reduce pass
_LINK = os.environ.get("MPA_INC_LINK", "1") == "1"


def _chain(mod, mods, x, out=None):
    """A branch's BasicConv2d chain (e.g. 7x7dbl_2 -> _3 -> _4 -> _5): each BN+ReLU output
    feeds ONLY the next conv, so that conv's dgrad performs its backward reduction
    (Fn.BNLink: no reduce pass); the last conv writes into ``out`` (the block buffer)."""
    link = None
    use = _LINK and mod.training and torch.is_grad_enabled()
    for k, m in enumerate(mods):
        last = k == len(mods) - 1
        nxt = Fn.BNLink() if (use and not last) else None
        x = m(x, out=out if last else None, link_in=link, link_out=nxt)
        link = nxt
    return x


def _avg3(x, join=None):
    return Fn.avg_pool2d(x, (3, 3), (1, 1), (1, 1), False, True, join=join)


# MPA_POOL_FIRST=1: branch_pool as torchvision writes it (3x3 average pool over the block
# input, then the 1x1 conv) instead of the commuted order below
_POOL_FIRST = os.environ.get("MPA_POOL_FIRST", "0") == "1"


class PoolBranch(BasicConv2d):
    """``branch_pool = BasicConv2d(avg_pool2d(x, 3, 1, 1))`` of InceptionA/C/E
    (torchvision inception.py, reached from ``/root/reference/models.py:83-95``).

    The 3x3/s1 average pool with count_include_pad (divisor 9 everywhere) and the 1x1 conv
    are both linear maps - one spatial per channel, one per-pixel channel mix - so they
    commute exactly: conv1x1(avg(x)) = avg(conv1x1(x)).  Run in that order the pool (forward
    and backward) works on the conv's 32-192 output channels instead of the block's 192-2048
    input channels, and x needs no pooled copy: Mixed_5b-7c read and write 3-10x fewer
    pool bytes.  BN statistics are taken over the pooled values, as in the reference."""

    # avg_pool2d(3, 1, 1, ceil_mode=False, count_include_pad=True) as the grouped GEMM's
    # (kh, kw, sh, sw, ph, pw, ceil, cip) for this member (Fn.conv1x1_group)
    pool_after = (3, 3, 1, 1, 1, 1, False, True)

    def forward(self, x, join=None, out=None):
        if _POOL_FIRST:
            return super().forward(_avg3(x, join), out=out)
        return Fn.bn_act(_avg3(Fn.conv_act(x, self.conv, relu=False, join=join)), self.bn,
                         relu=True, out=out)


def _max3s2(x, join=None):
    return Fn.max_pool2d(x, (3, 3), (2, 2), (0, 0), False, join=join)


def _cat(xs):
    return Fn.cat_channels(xs)


# MPA_CAT_INTO=0: branch outputs are separate tensors copied into the block output
# (concat_kernel forward, split backward) instead of written at their channel offsets
_CAT_INTO = os.environ.get("MPA_CAT_INTO", "1") == "1"


def _buffer(mod, x, hw, widths):
    """The block output every branch writes its result into at its channel offset (a
    Fn.ChannelBuffer), in training; None otherwise (the branches' outputs are then
    concatenated by a copy)."""
    if not (_CAT_INTO and mod.training and torch.is_grad_enabled()):
        return None
    return Fn.ChannelBuffer(x, hw, widths)


class _NoBuffer:
    """Stand-in for a missing ChannelBuffer: no destination windows, concat by copy."""

    @staticmethod
    def window(i):
        return None

    @staticmethod
    def gather(parts):
        return _cat(parts)


def _out(cb):
    return cb if cb is not None else _NoBuffer


class _SideBranch:
    """One branch chain of a block enqueued on the branch stream (Fn.branch_stream) while
    the block's other branches go to the compute stream; ``join`` before the block output
    is used.  Only with a ChannelBuffer (the chain writes its window) and for chains whose
    input is a grouped-head output, so the chain's input gradient goes to
    _ConvGroupBNAct.backward (which marks it used on the compute stream)."""

    def __init__(self, x, cb):
        self.s = Fn.branch_stream(x) if isinstance(cb, Fn.ChannelBuffer) else None
        if self.s is not None:
            self.main = torch.cuda.current_stream(x.device)
            self.s.wait_stream(self.main)
            x.record_stream(self.s)
            cb.buf.record_stream(self.s)

    def run(self, fn):
        if self.s is None:
            return fn()
        with torch.cuda.stream(self.s):
            return fn()

    def join(self):
        if self.s is not None:
            self.main.wait_stream(self.s)


def _half(n: int) -> int:
    return (n - 3) // 2 + 1  # 3x3 / stride 2 / no padding


def _heads(mod, x, heads):
    """Whether the block's 1x1 branch heads run as ONE grouped GEMM (Fn.conv1x1_group):
    training with their weights adjacent in the arena (Inception3._mpa_param_groups);
    ``merge_1x1 = False`` (utils/parity.py) keeps them separate modules."""
    return getattr(mod, "merge_1x1", True) and _MERGE and Fn.conv1x1_group_ok(x, heads)


# MPA_MERGE_1X1=0: every 1x1 branch head is its own GEMM reading the block input
_MERGE = os.environ.get("MPA_MERGE_1X1", "1") == "1"


def _join(mod, x, n, join=None):
    """The GradJoin of an input read by ``n`` branches (None outside training); a parent
    passes its own join when x has consumers outside this block (Mixed_6e -> aux head)."""
    if join is not None:
        return join
    if _JOIN and mod.training and torch.is_grad_enabled() and x.requires_grad:
        return Fn.GradJoin(n)
    return None


class InceptionA(nn.Module):
    def __init__(self, in_channels, pool_features):
        super().__init__()
        self.branch1x1 = BasicConv2d(in_channels, 64, 1)
        self.branch5x5_1 = BasicConv2d(in_channels, 48, 1)
        self.branch5x5_2 = BasicConv2d(48, 64, 5, padding=2)
        self.branch3x3dbl_1 = BasicConv2d(in_channels, 64, 1)
        self.branch3x3dbl_2 = BasicConv2d(64, 96, 3, padding=1)
        self.branch3x3dbl_3 = BasicConv2d(96, 96, 3, padding=1)
        self.branch_pool = PoolBranch(in_channels, pool_features, 1)

    def heads(self):
        return [self.branch1x1, self.branch5x5_1, self.branch3x3dbl_1, self.branch_pool]

    def forward(self, x, join=None):
        cb = _out(_buffer(self, x, x.shape[1:3],
                          [64, 64, 96, self.branch_pool.conv.out_channels]))
        side = None
        if _heads(self, x, self.heads()):  # every consumer of x in one grouped GEMM
            b1, b5, b3, bp = Fn.conv1x1_group(x, self.heads(), join,
                                              [cb.window(0), None, None, cb.window(3)])
            side = _SideBranch(b3, cb)
        else:
            j = _join(self, x, 4, join)
            b1 = self.branch1x1(x, j, out=cb.window(0))
            b5, b3 = self.branch5x5_1(x, j), self.branch3x3dbl_1(x, j)
            bp = self.branch_pool(x, j, out=cb.window(3))
        chain = [self.branch3x3dbl_2, self.branch3x3dbl_3]
        if side is not None:
            b3 = side.run(lambda: _chain(self, chain, b3, cb.window(2)))
        b5 = self.branch5x5_2(b5, out=cb.window(1))
        if side is not None:
            side.join()
        else:
            b3 = _chain(self, chain, b3, cb.window(2))
        return cb.gather([b1, b5, b3, bp])


class InceptionB(nn.Module):
    def __init__(self, in_channels):
        super().__init__()
        self.branch3x3 = BasicConv2d(in_channels, 384, 3, stride=2)
        self.branch3x3dbl_1 = BasicConv2d(in_channels, 64, 1)
        self.branch3x3dbl_2 = BasicConv2d(64, 96, 3, padding=1)
        self.branch3x3dbl_3 = BasicConv2d(96, 96, 3, stride=2)

    def forward(self, x, join=None):
        j = _join(self, x, 3, join)
        cb = _out(_buffer(self, x, (_half(x.shape[1]), _half(x.shape[2])),
                          [384, 96, x.shape[-1]]))
        b3 = self.branch3x3(x, j, out=cb.window(0))
        bd = _chain(self, [self.branch3x3dbl_2, self.branch3x3dbl_3],
                    self.branch3x3dbl_1(x, j), cb.window(1))
        return cb.gather([b3, bd, _max3s2(x, j)])


class InceptionC(nn.Module):
    def __init__(self, in_channels, channels_7x7):
        super().__init__()
        c7 = channels_7x7
        self.branch1x1 = BasicConv2d(in_channels, 192, 1)
        self.branch7x7_1 = BasicConv2d(in_channels, c7, 1)
        self.branch7x7_2 = BasicConv2d(c7, c7, (1, 7), padding=(0, 3))
        self.branch7x7_3 = BasicConv2d(c7, 192, (7, 1), padding=(3, 0))
        self.branch7x7dbl_1 = BasicConv2d(in_channels, c7, 1)
        self.branch7x7dbl_2 = BasicConv2d(c7, c7, (7, 1), padding=(3, 0))
        self.branch7x7dbl_3 = BasicConv2d(c7, c7, (1, 7), padding=(0, 3))
        self.branch7x7dbl_4 = BasicConv2d(c7, c7, (7, 1), padding=(3, 0))
        self.branch7x7dbl_5 = BasicConv2d(c7, 192, (1, 7), padding=(0, 3))
        self.branch_pool = PoolBranch(in_channels, 192, 1)

    def heads(self):
        return [self.branch1x1, self.branch7x7_1, self.branch7x7dbl_1, self.branch_pool]

    def forward(self, x, join=None):
        cb = _out(_buffer(self, x, x.shape[1:3], [192, 192, 192, 192]))
        side = None
        if _heads(self, x, self.heads()):  # every consumer of x in one grouped GEMM
            b1, b7, bd, bp = Fn.conv1x1_group(x, self.heads(), join,
                                              [cb.window(0), None, None, cb.window(3)])
            side = _SideBranch(bd, cb)
        else:
            j = _join(self, x, 4, join)
            b1 = self.branch1x1(x, j, out=cb.window(0))
            b7, bd = self.branch7x7_1(x, j), self.branch7x7dbl_1(x, j)
            bp = self.branch_pool(x, j, out=cb.window(3))
        dbl = [self.branch7x7dbl_2, self.branch7x7dbl_3, self.branch7x7dbl_4,
               self.branch7x7dbl_5]
        if side is not None:  # the 4-conv chain beside the 2-conv one
            bd = side.run(lambda: _chain(self, dbl, bd, cb.window(2)))
        b7 = _chain(self, [self.branch7x7_2, self.branch7x7_3], b7, cb.window(1))
        if side is not None:
            side.join()
        else:
            bd = _chain(self, dbl, bd, cb.window(2))
        return cb.gather([b1, b7, bd, bp])


class InceptionD(nn.Module):
    def __init__(self, in_channels):
        super().__init__()
        self.branch3x3_1 = BasicConv2d(in_channels, 192, 1)
        self.branch3x3_2 = BasicConv2d(192, 320, 3, stride=2)
        self.branch7x7x3_1 = BasicConv2d(in_channels, 192, 1)
        self.branch7x7x3_2 = BasicConv2d(192, 192, (1, 7), padding=(0, 3))
        self.branch7x7x3_3 = BasicConv2d(192, 192, (7, 1), padding=(3, 0))
        self.branch7x7x3_4 = BasicConv2d(192, 192, 3, stride=2)

    def heads(self):
        return [self.branch3x3_1, self.branch7x7x3_1]

    def forward(self, x, join=None):
        # (a join handed in by the parent counts this block's consumers: see Inception3)
        grouped = _heads(self, x, self.heads())
        if grouped:
            j = _join(self, x, 2, join)
            b3, b7 = Fn.conv1x1_group(x, self.heads(), j)
        else:
            j = _join(self, x, 3, join)
            b3, b7 = self.branch3x3_1(x, j), self.branch7x7x3_1(x, j)
        cb = _out(_buffer(self, x, (_half(x.shape[1]), _half(x.shape[2])),
                          [320, 192, x.shape[-1]]))
        side = _SideBranch(b7, cb) if grouped else None
        chain = [self.branch7x7x3_2, self.branch7x7x3_3, self.branch7x7x3_4]
        if side is not None:  # the 3-conv chain beside the 3x3/s2 conv and the pool
            b7 = side.run(lambda: _chain(self, chain, b7, cb.window(1)))
        b3 = self.branch3x3_2(b3, out=cb.window(0))
        if side is None:
            b7 = _chain(self, chain, b7, cb.window(1))
        mp = _max3s2(x, j)
        if side is not None:
            side.join()
        return cb.gather([b3, b7, mp])


class InceptionE(nn.Module):
    def __init__(self, in_channels):
        super().__init__()
        self.branch1x1 = BasicConv2d(in_channels, 320, 1)
        self.branch3x3_1 = BasicConv2d(in_channels, 384, 1)
        self.branch3x3_2a = BasicConv2d(384, 384, (1, 3), padding=(0, 1))
        self.branch3x3_2b = BasicConv2d(384, 384, (3, 1), padding=(1, 0))
        self.branch3x3dbl_1 = BasicConv2d(in_channels, 448, 1)
        self.branch3x3dbl_2 = BasicConv2d(448, 384, 3, padding=1)
        self.branch3x3dbl_3a = BasicConv2d(384, 384, (1, 3), padding=(0, 1))
        self.branch3x3dbl_3b = BasicConv2d(384, 384, (3, 1), padding=(1, 0))
        self.branch_pool = PoolBranch(in_channels, 192, 1)

    def heads(self):
        return [self.branch1x1, self.branch3x3_1, self.branch3x3dbl_1, self.branch_pool]

    def forward(self, x, join=None):
        # torchvision: cat([b1, cat([2a, 2b]), cat([3a, 3b]), bp]) - the same channel order
        # as one flat buffer of six windows
        cb = _out(_buffer(self, x, x.shape[1:3], [320, 384, 384, 384, 384, 192]))
        side = None
        if _heads(self, x, self.heads()):  # every consumer of x in one grouped GEMM
            b1, b3, bd, bp = Fn.conv1x1_group(x, self.heads(), join,
                                              [cb.window(0), None, None, cb.window(5)])
            side = _SideBranch(bd, cb)
        else:
            j = _join(self, x, 4, join)
            b1 = self.branch1x1(x, j, out=cb.window(0))
            b3, bd = self.branch3x3_1(x, j), self.branch3x3dbl_1(x, j)
            bp = self.branch_pool(x, j, out=cb.window(5))

        def dbl(bd):  # 3x3 conv, then its (1x3) and (3x1) heads (all on one stream)
            bd = self.branch3x3dbl_2(bd)
            jd = _join(self, bd, 2)
            return (self.branch3x3dbl_3a(bd, jd, out=cb.window(3)),
                    self.branch3x3dbl_3b(bd, jd, out=cb.window(4)))

        if side is not None:
            bda, bdb = side.run(lambda: dbl(bd))
        j3 = _join(self, b3, 2)  # b3 and bd each feed a (1x3) and a (3x1) conv
        b3a = self.branch3x3_2a(b3, j3, out=cb.window(1))
        b3b = self.branch3x3_2b(b3, j3, out=cb.window(2))
        if side is not None:
            side.join()
        else:
            bda, bdb = dbl(bd)
        return cb.gather([b1, b3a, b3b, bda, bdb, bp])


class InceptionAux(nn.Module):
    def __init__(self, in_channels, num_classes):
        super().__init__()
        self.conv0 = BasicConv2d(in_channels, 128, 1)
        self.conv1 = BasicConv2d(128, 768, 5)
        self.conv1.stddev = 0.01
        self.fc = Linear(768, num_classes)
        self.fc.stddev = 0.001
        self.avgpool = AdaptiveAvgPool2d((1, 1))

    def forward(self, x, join=None):
        x = Fn.avg_pool2d(x, (5, 5), (3, 3), (0, 0), False, True, join=join)
        x = self.conv1(self.conv0(x))
        x = self.avgpool(x).reshape(x.shape[0], -1)
        return self.fc(x)


class Inception3(nn.Module):
    def __init__(self, num_classes: int = 1000, aux_logits: bool = True, dropout: float = 0.5):
        super().__init__()
        self.aux_logits = aux_logits
        self.transform_input = False
        self.cross_join = True
        # Conv2d_2b -> maxpool1 and Conv2d_4a -> maxpool2 as the fused conv + BN + ReLU +
        # max-pool op (one pass over the conv output, as the ResNet / DenseNet stems);
        # utils/parity.py turns it off to hook the two BasicConv2d units
        self.fuse_stem_pools = True
        self.Conv2d_1a_3x3 = BasicConv2d(3, 32, 3, stride=2)
        self.Conv2d_2a_3x3 = BasicConv2d(32, 32, 3)
        self.Conv2d_2b_3x3 = BasicConv2d(32, 64, 3, padding=1)
        self.maxpool1 = MaxPool2d(3, 2)
        self.Conv2d_3b_1x1 = BasicConv2d(64, 80, 1)
        self.Conv2d_4a_3x3 = BasicConv2d(80, 192, 3)
        self.maxpool2 = MaxPool2d(3, 2)
        self.Mixed_5b = InceptionA(192, 32)
        self.Mixed_5c = InceptionA(256, 64)
        self.Mixed_5d = InceptionA(288, 64)
        self.Mixed_6a = InceptionB(288)
        self.Mixed_6b = InceptionC(768, 128)
        self.Mixed_6c = InceptionC(768, 160)
        self.Mixed_6d = InceptionC(768, 160)
        self.Mixed_6e = InceptionC(768, 192)
        self.AuxLogits = InceptionAux(768, num_classes) if aux_logits else None
        self.Mixed_7a = InceptionD(768)
        self.Mixed_7b = InceptionE(1280)
        self.Mixed_7c = InceptionE(2048)
        self.avgpool = AdaptiveAvgPool2d((1, 1))
        self.dropout = Dropout(dropout)
        self.fc = Linear(2048, num_classes)
        for m in self.modules():
            if isinstance(m, (Conv2d, Linear)):
                std = float(getattr(m, "stddev", 0.1))
                m.init_(lambda w, s=std: nn.init.trunc_normal_(w, 0.0, s, -2, 2))

    def forward(self, x):
        x = _chain(self, [self.Conv2d_1a_3x3, self.Conv2d_2a_3x3], x)
        if self.fuse_stem_pools:
            x = Fn.conv_bn_relu_maxpool(x, self.Conv2d_2b_3x3.conv, self.Conv2d_2b_3x3.bn,
                                        self.maxpool1)
            x = Fn.conv_bn_relu_maxpool(self.Conv2d_3b_1x1(x), self.Conv2d_4a_3x3.conv,
                                        self.Conv2d_4a_3x3.bn, self.maxpool2)
        else:
            x = self.maxpool1(self.Conv2d_2b_3x3(x))
            x = self.maxpool2(self.Conv2d_4a_3x3(self.Conv2d_3b_1x1(x)))
        for m in (self.Mixed_5b, self.Mixed_5c, self.Mixed_5d, self.Mixed_6a, self.Mixed_6b,
                  self.Mixed_6c, self.Mixed_6d, self.Mixed_6e):
            x = m(x)
        aux = None
        if self.AuxLogits is not None and self.training:
            # Mixed_6e's output feeds the aux head's pool and Mixed_7a's three branches
            # (cross_join = False keeps the two modules' input gradients apart, for the
            # per-unit parity check of utils/parity.py)
            n7a = 3 if _heads(self.Mixed_7a, x, self.Mixed_7a.heads()) else 4
            j = _join(self.Mixed_7a, x, n7a) if self.cross_join else None
            aux = self.AuxLogits(x, j)
            x = self.Mixed_7a(x, j)
        else:
            x = self.Mixed_7a(x)
        for m in (self.Mixed_7b, self.Mixed_7c):
            x = m(x)
        x = self.avgpool(x).reshape(x.shape[0], -1)
        x = self.dropout(x)
        x = self.fc(x)
        if self.training and self.aux_logits:
            return InceptionOutputs(x, aux)
        return x


def _param_groups(self):
    """Weights of each block's 1x1 branch heads, back to back in the arena (Fn.conv1x1_group)."""
    return [[h.conv.weight for h in m.heads()] for m in self.modules()
            if isinstance(m, (InceptionA, InceptionC, InceptionD, InceptionE))]


Inception3._mpa_param_groups = _param_groups


def inception_v3(num_classes: int = 1000) -> Inception3:
    return Inception3(num_classes)
