"""SqueezeNet 1.0, NHWC, torchvision parameter names.

Reference: ``models.squeezenet1_0`` with ``classifier[1] = nn.Conv2d(512, num_classes,
1)`` and ``num_classes`` attribute (``/root/reference/models.py:65-72``).  The Fire
module's channel concat is a last-dim concat in NHWC.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .layers import Conv2d, MaxPool2d, AdaptiveAvgPool2d, ReLU, Dropout, FusedSequential
from ..ops import functional as Fn


class Fire(nn.Module):
    def __init__(self, inplanes, squeeze_planes, expand1x1_planes, expand3x3_planes):
        super().__init__()
        self.inplanes = inplanes
        self.squeeze = Conv2d(inplanes, squeeze_planes, 1)
        self.squeeze_activation = ReLU(True)
        self.expand1x1 = Conv2d(squeeze_planes, expand1x1_planes, 1)
        self.expand1x1_activation = ReLU(True)
        self.expand3x3 = Conv2d(squeeze_planes, expand3x3_planes, 3, padding=1)
        self.expand3x3_activation = ReLU(True)

    def forward(self, x):
        s = self.squeeze(x, relu=True)
        return Fn.cat_channels([self.expand1x1(s, relu=True), self.expand3x3(s, relu=True)])


class SqueezeNet(nn.Module):
    def __init__(self, num_classes: int = 1000, dropout: float = 0.5):
        super().__init__()
        self.num_classes = num_classes
        self.features = FusedSequential(
            Conv2d(3, 96, 7, 2), ReLU(True), MaxPool2d(3, 2, ceil_mode=True),
            Fire(96, 16, 64, 64), Fire(128, 16, 64, 64), Fire(128, 32, 128, 128),
            MaxPool2d(3, 2, ceil_mode=True),
            Fire(256, 32, 128, 128), Fire(256, 48, 192, 192), Fire(384, 48, 192, 192),
            Fire(384, 64, 256, 256), MaxPool2d(3, 2, ceil_mode=True),
            Fire(512, 64, 256, 256))
        final_conv = Conv2d(512, num_classes, 1, pad_out=True)
        self.classifier = FusedSequential(Dropout(dropout), final_conv, ReLU(True),
                                          AdaptiveAvgPool2d((1, 1)))
        for m in self.modules():
            if isinstance(m, Conv2d):
                if m is final_conv:
                    m.init_(lambda w: nn.init.normal_(w, 0.0, 0.01))
                else:
                    m.init_(nn.init.kaiming_uniform_)
                nn.init.zeros_(m.bias)

    def replace_head(self, num_classes: int) -> None:
        """``classifier[1] = Conv2d(512, nc, 1)``; ``num_classes = nc`` (models.py:70-71)."""
        self.classifier[1] = Conv2d(512, num_classes, 1, pad_out=True)
        self.num_classes = num_classes

    def forward(self, x):
        x = self.features(x)
        x = self.classifier(x)
        # the head conv stores its output channels padded to a multiple of 32
        return x.reshape(x.shape[0], -1)[:, :self.num_classes]


def squeezenet1_0(num_classes: int = 1000) -> SqueezeNet:
    return SqueezeNet(num_classes)
