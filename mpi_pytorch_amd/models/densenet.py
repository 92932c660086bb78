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
        x = self.norm1(x, relu=True)
        x = Fn.conv_bn_act(x, self.conv1, self.norm2, relu=True)
        return self.conv2(x)


# MPA_DENSE_BLOCK_GRAD=0: plain autograd through the per-layer concats (one split and one
# elementwise add per earlier feature and layer) instead of the block-level accumulator
_BLOCK_GRAD = os.environ.get("MPA_DENSE_BLOCK_GRAD", "1") == "1"


class _DenseBlock(nn.ModuleDict):
    def __init__(self, num_layers, num_input_features, bn_size, growth_rate):
        super().__init__()
        for i in range(num_layers):
            self.add_module("denselayer%d" % (i + 1),
                            _DenseLayer(num_input_features + i * growth_rate, growth_rate,
                                        bn_size))

    def forward(self, x):
        if _BLOCK_GRAD and self.training and torch.is_grad_enabled() and x.requires_grad:
            params = [p for p in self.parameters() if p.requires_grad]
            return _DenseBlockGrad.apply(x, self, *params)
        feats = [x]
        for layer in self.values():
            feats.append(layer(feats))
        return Fn.cat_channels(feats)


class _DenseBlockGrad(torch.autograd.Function):
    """A dense block whose backward sums every feature's gradient in ONE fp32 buffer.

    Each feature feeds every later layer (through that layer's input concat) and the
    block output, so plain autograd splits each layer's input gradient into per-feature
    pieces and adds them feature by feature: O(L^2) small split / add launches per block
    (535 ATen adds per DenseNet-121 step).  Here the forward runs each layer on a leaf
    copy of its concatenated input (its own small autograd graph, kept for backward), and
    the backward walks the layers in reverse with G = the block gradient [..., C_total] in
    fp32: layer i's output gradient is read from G's channels of feature i
    (``chan_extract``), its graph is back-propagated, and its input gradient is added to
    G's first C_i channels (``chan_accum``, one launch).  Parameter gradients land in the
    flat arena from the layers' own kernels, as in every other model."""

    @staticmethod
    def forward(ctx, x, block, *params):
        feats = [x.detach()]
        recs = []
        with torch.enable_grad():
            for layer in block.values():
                inp = Fn.cat_channels(feats) if len(feats) > 1 else feats[0]
                inp = inp.detach().requires_grad_(True)
                out = layer([inp])
                recs.append((inp, out))
                feats.append(out.detach())
        ctx.recs = recs
        ctx.sizes = [f.shape[-1] for f in feats]
        ctx.nparams = len(params)
        return Fn.cat_channels(feats)

    @staticmethod
    def backward(ctx, gy):
        k = Fn.K(gy)
        gy = gy.contiguous()
        ctot = gy.shape[-1]
        g = torch.empty(gy.shape, dtype=torch.float32, device=gy.device)
        k.chan_accum(g, 0, gy, True)
        offs = []
        o = 0
        for c in ctx.sizes:
            offs.append(o)
            o += c
        for i in range(len(ctx.recs) - 1, -1, -1):
            inp, out = ctx.recs[i]
            g_out = k.chan_extract(g, offs[i + 1], ctx.sizes[i + 1]).to(out.dtype)
            torch.autograd.backward(out, g_out)
            if inp.grad is not None:
                k.chan_accum(g, 0, inp.grad, False)
            ctx.recs[i] = None
        dx = k.chan_extract(g, 0, ctx.sizes[0]).to(gy.dtype)
        return (dx, None) + (None,) * ctx.nparams


class _Transition(nn.Sequential):
    def __init__(self, num_input_features, num_output_features):
        super().__init__()
        self.norm = BatchNorm2d(num_input_features)
        self.relu = ReLU(True)
        self.conv = Conv2d(num_input_features, num_output_features, 1, bias=False)
        self.pool = AvgPool2d(2, 2)

    def forward(self, x):
        x = self.norm(x, relu=True)
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
        for m in self.modules():
            if isinstance(m, Conv2d):
                m.init_(nn.init.kaiming_normal_)
            elif isinstance(m, Linear):
                nn.init.zeros_(m.bias)

    def forward(self, x):
        f = self.features
        x = Fn.conv_bn_relu_maxpool(x, f.conv0, f.norm0, f.pool0)
        for name, m in f.named_children():
            if name.startswith("denseblock") or name.startswith("transition"):
                x = m(x)
        x = f.norm5(x, relu=True)  # features.norm5 then F.relu (torchvision densenet forward)
        x = self.avgpool(x).reshape(x.shape[0], -1)
        return self.classifier(x)


def densenet121(num_classes: int = 1000) -> DenseNet:
    return DenseNet(32, (6, 12, 24, 16), 64, num_classes=num_classes)
