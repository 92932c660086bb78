"""VGG11_bn / VGG16 and AlexNet, NHWC, torchvision parameter names / indices.

Reference: ``models.vgg11_bn`` (key ``"vgg"``, ``/root/reference/models.py:56-63``) and
``models.alexnet`` (``models.py:47-54``) with ``classifier[6]`` replaced by
``nn.Linear(4096, num_classes)``; VGG-16 is the BASELINE.json config-4 model.  The first
classifier Linear consumes an NHWC flatten; its weight is stored in (h,w,c) column order
and exported in torchvision's (c,h,w) order (``Linear(in_chw=...)``).
"""
from __future__ import annotations

import torch.nn as nn

from .layers import (Conv2d, BatchNorm2d, Linear, MaxPool2d, AdaptiveAvgPool2d, ReLU,
                     Dropout, FusedSequential)

CFGS = {
    "A": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "D": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
}


def make_layers(cfg, batch_norm: bool) -> FusedSequential:
    layers = []
    c = 3
    for v in cfg:
        if v == "M":
            layers.append(MaxPool2d(2, 2))
        else:
            layers.append(Conv2d(c, v, 3, 1, 1, bias=True))
            if batch_norm:
                layers.append(BatchNorm2d(v))
            layers.append(ReLU(True))
            c = v
    return FusedSequential(*layers)


class VGG(nn.Module):
    def __init__(self, features: FusedSequential, num_classes: int = 1000, dropout: float = 0.5):
        super().__init__()
        self.features = features
        self.avgpool = AdaptiveAvgPool2d((7, 7))
        self.classifier = FusedSequential(
            Linear(512 * 7 * 7, 4096, in_chw=(512, 7, 7)), ReLU(True), Dropout(dropout),
            Linear(4096, 4096), ReLU(True), Dropout(dropout),
            Linear(4096, num_classes))
        for m in self.modules():
            if isinstance(m, Conv2d):
                m.init_(lambda w: nn.init.kaiming_normal_(w, mode="fan_out", nonlinearity="relu"))
                nn.init.zeros_(m.bias)
            elif isinstance(m, Linear):
                m.init_(lambda w: nn.init.normal_(w, 0, 0.01))
                nn.init.zeros_(m.bias)

    def forward(self, x):
        x = self.features(x)
        x = self.avgpool(x)
        x = x.reshape(x.shape[0], -1)
        return self.classifier(x)


def vgg11_bn(num_classes: int = 1000) -> VGG:
    return VGG(make_layers(CFGS["A"], True), num_classes)


def vgg16(num_classes: int = 1000) -> VGG:
    return VGG(make_layers(CFGS["D"], False), num_classes)


class AlexNet(nn.Module):
    def __init__(self, num_classes: int = 1000, dropout: float = 0.5):
        super().__init__()
        self.features = FusedSequential(
            Conv2d(3, 64, 11, 4, 2), ReLU(True), MaxPool2d(3, 2),
            Conv2d(64, 192, 5, 1, 2), ReLU(True), MaxPool2d(3, 2),
            Conv2d(192, 384, 3, 1, 1), ReLU(True),
            Conv2d(384, 256, 3, 1, 1), ReLU(True),
            Conv2d(256, 256, 3, 1, 1), ReLU(True), MaxPool2d(3, 2))
        self.avgpool = AdaptiveAvgPool2d((6, 6))
        self.classifier = FusedSequential(
            Dropout(dropout), Linear(256 * 6 * 6, 4096, in_chw=(256, 6, 6)), ReLU(True),
            Dropout(dropout), Linear(4096, 4096), ReLU(True),
            Linear(4096, num_classes))

    def forward(self, x):
        x = self.features(x)
        x = self.avgpool(x)
        x = x.reshape(x.shape[0], -1)
        return self.classifier(x)


def alexnet(num_classes: int = 1000) -> AlexNet:
    return AlexNet(num_classes)
