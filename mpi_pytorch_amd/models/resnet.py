"""ResNet-18/34 (BasicBlock), NHWC, torchvision parameter names.

Reference: ``models.resnet18`` / ``models.resnet34`` with ``fc`` replaced by
``nn.Linear(512, num_classes)`` (``/root/reference/models.py:30-45``).  Each
conv->bn(->add)->relu runs as one fused op (``conv_bn_act``), the residual add folded
into the BN-apply kernel.
"""
from __future__ import annotations

import os

import torch.nn as nn

from .layers import Conv2d, BatchNorm2d, Linear, MaxPool2d, AdaptiveAvgPool2d, ReLU
from ..ops import functional as Fn


# The conv1 -> conv2 BN-backward hand-off (Fn.BNLink): conv2's halo dgrad epilogue does
# bn1's backward reduction (mask recomputed from z, sums of g and g*xhat), so bn1's reduce
# pass (8 per ResNet-18 step) disappears.  Rounds 1-3 measured it slower (-9 % at batch
# 1024): that flavour spilled 250-550 B/lane to scratch in its 8-wave form.  Unspilled
# (4-wave blocks, per-tile DPP reduction) it is +0.5 % (profiles/bn_link_ab_r4.txt).
# MPA_BN_LINK=0 turns it off.
_LINK = os.environ.get("MPA_BN_LINK", "1") == "1"
# MPA_GRAD_JOIN=0 restores autograd's separate add of the two input-gradient contributions
_JOIN = os.environ.get("MPA_GRAD_JOIN", "1") == "1"
# MPA_DS_DEFER=0: the downsample BN writes its output (instead of bn2 applying it on read)
_DS_DEFER = os.environ.get("MPA_DS_DEFER", "1") == "1"
class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample=None):
        super().__init__()
        self.conv1 = Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = BatchNorm2d(planes)
        self.relu = ReLU(inplace=True)
        self.conv2 = Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        # conv1's output feeds only conv2: conv2's dgrad performs bn1's backward reduction
        link = None
        if self.bn1.training and _LINK:
            link = Fn.BNLink()
        # x's gradient = conv1's dgrad + the shortcut's: summed inside the second dgrad
        join = Fn.GradJoin() if (self.bn1.training and _JOIN and x.requires_grad) else None
        out = Fn.conv_bn_act(x, self.conv1, self.bn1, relu=True, link_out=link, join_x=join)
        dsd = None
        if self.downsample is not None:
            # the downsample's BN is applied by bn2 while it reads the residual (Fn.BNDefer)
            dsd = Fn.BNDefer() if (self.bn2.training and _DS_DEFER) else None
            identity = Fn.conv_bn_act(x, self.downsample[0], self.downsample[1], relu=False,
                                      join_x=join, defer=dsd)
            join_res = None
        else:
            identity = x
            join_res = join
        return Fn.conv_bn_act(out, self.conv2, self.bn2, relu=True, residual=identity,
                              link_in=link, join_res=join_res, res_defer=dsd)


class Downsample(nn.Sequential):
    pass


class ResNet(nn.Module):
    def __init__(self, layers, num_classes: int = 1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = BatchNorm2d(64)
        self.relu = ReLU(inplace=True)
        self.maxpool = MaxPool2d(3, 2, 1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], stride=2)
        self.layer3 = self._make_layer(256, layers[2], stride=2)
        self.layer4 = self._make_layer(512, layers[3], stride=2)
        self.avgpool = AdaptiveAvgPool2d((1, 1))
        self.fc = Linear(512, num_classes)
        for m in self.modules():
            if isinstance(m, Conv2d):
                m.init_(lambda w: nn.init.kaiming_normal_(w, mode="fan_out", nonlinearity="relu"))

    def _make_layer(self, planes: int, blocks: int, stride: int = 1):
        downsample = None
        if stride != 1 or self.inplanes != planes:
            downsample = Downsample(Conv2d(self.inplanes, planes, 1, stride, 0, bias=False),
                                    BatchNorm2d(planes))
        layers = [BasicBlock(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes
        for _ in range(1, blocks):
            layers.append(BasicBlock(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = Fn.conv_bn_relu_maxpool(x, self.conv1, self.bn1, self.maxpool)
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for blk in layer:
                x = blk(x)
        x = self.avgpool(x)
        x = x.reshape(x.shape[0], -1)
        return self.fc(x)


def resnet18(num_classes: int = 1000) -> ResNet:
    return ResNet([2, 2, 2, 2], num_classes)


def resnet34(num_classes: int = 1000) -> ResNet:
    return ResNet([3, 4, 6, 3], num_classes)
