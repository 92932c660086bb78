"""DenseNet-121, NHWC, torchvision parameter names.

Reference: ``models.densenet121`` with ``classifier = nn.Linear(1024, num_classes)``
(``/root/reference/models.py:74-81``).  Pre-activation layers: BN+ReLU run as one fused
kernel over the concatenated features (channel concat = last-dim concat in NHWC).
"""
from __future__ import annotations

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


class _DenseBlock(nn.ModuleDict):
    def __init__(self, num_layers, num_input_features, bn_size, growth_rate):
        super().__init__()
        for i in range(num_layers):
            self.add_module("denselayer%d" % (i + 1),
                            _DenseLayer(num_input_features + i * growth_rate, growth_rate,
                                        bn_size))

    def forward(self, x):
        feats = [x]
        for layer in self.values():
            feats.append(layer(feats))
        return Fn.cat_channels(feats)


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
