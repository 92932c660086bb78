"""Model zoo: the reference's 7 model keys plus ``vgg16`` (BASELINE.json config 4).

``initialize_model(model_name, num_classes, feature_extract, use_pretrained)`` mirrors
``/root/reference/models.py:16-101``: build the torchvision architecture, optionally
freeze it (``set_parameter_requires_grad``, ``models.py:5-13``), replace the classifier
head with a fresh ``num_classes``-wide layer, and return ``(model, input_size)``.

Differences (documented, deliberate):
* architectures are implemented in-repo (torchvision is not installed) with identical
  parameter names and state_dict shapes; internal layouts are NHWC/KRSC;
* ``use_pretrained=True`` cannot download hub weights offline - it loads a local
  torchvision-format state_dict when ``MPA_PRETRAINED_DIR`` holds ``<arch>.pth``
  (weights_only), otherwise keeps random init and says so;
* an invalid name raises ``ValueError`` instead of ``exit()`` (``models.py:97-99``).
"""
from __future__ import annotations

import os
import warnings
from typing import Tuple

import torch
import torch.nn as nn

from .layers import Conv2d, Linear
from .resnet import resnet18, resnet34, ResNet
from .vgg import vgg11_bn, vgg16, alexnet, VGG, AlexNet
from .squeezenet import squeezenet1_0, SqueezeNet
from .densenet import densenet121, DenseNet
from .inception import inception_v3, Inception3, InceptionOutputs

ARCH = {
    "resnet18": ("resnet18", resnet18, 224),
    "resnet34": ("resnet34", resnet34, 128),   # models.py:45 returns 128 for resnet34
    "alexnet": ("alexnet", alexnet, 224),
    "vgg": ("vgg11_bn", vgg11_bn, 224),
    "vgg16": ("vgg16", vgg16, 224),
    "squeezenet": ("squeezenet1_0", squeezenet1_0, 224),
    "densenet": ("densenet121", densenet121, 224),
    "inception": ("inception_v3", inception_v3, 299),
}


def set_parameter_requires_grad(model: nn.Module, feature_extracting: bool) -> None:
    if feature_extracting:
        for p in model.parameters():
            p.requires_grad = False


def _maybe_pretrained(model: nn.Module, arch: str) -> None:
    d = os.environ.get("MPA_PRETRAINED_DIR", "")
    path = os.path.join(d, arch + ".pth") if d else ""
    if path and os.path.exists(path):
        sd = torch.load(path, map_location="cpu", weights_only=True)
        model.load_state_dict(sd)
    else:
        warnings.warn("use_pretrained=True but no local weights for {} (no network); using "
                      "random init".format(arch))


def initialize_model(model_name: str, num_classes: int, feature_extract: bool,
                     use_pretrained: bool = False) -> Tuple[nn.Module, int]:
    if model_name not in ARCH:
        raise ValueError("Invalid model name {!r}".format(model_name))
    arch, ctor, input_size = ARCH[model_name]
    model = ctor(1000)
    if use_pretrained:
        _maybe_pretrained(model, arch)
    set_parameter_requires_grad(model, feature_extract)
    if model_name in ("resnet18", "resnet34"):
        model.fc = Linear(model.fc.in_features, num_classes, bias=True)
    elif model_name in ("alexnet", "vgg", "vgg16"):
        model.classifier[6] = Linear(model.classifier[6].in_features, num_classes)
    elif model_name == "squeezenet":
        model.replace_head(num_classes)
    elif model_name == "densenet":
        model.classifier = Linear(model.classifier.in_features, num_classes)
    elif model_name == "inception":
        model.AuxLogits.fc = Linear(model.AuxLogits.fc.in_features, num_classes)
        model.fc = Linear(model.fc.in_features, num_classes)
    return model, input_size


def input_spec(model: nn.Module, hw) -> dict:
    """Image layout the model's stem wants from the data pipeline for ``hw`` images:
    ``{"cpad": channels, "pad": (top, bottom, left, right) | None}`` - a 4-channel zero
    canvas for pixel-pair stems (``layers.Conv2d``), 8 channels otherwise.  The preprocess
    kernel writes it directly; any other layout is converted by the stem (slower)."""
    for m in model.modules():
        if isinstance(m, Conv2d) and m.in_channels <= 4:
            return m.input_spec(tuple(hw))
    return {"cpad": 8, "pad": None}


def head_parameters(model: nn.Module):
    """Parameters of the replaced classifier head(s)."""
    for name in ("fc", "classifier", "AuxLogits"):
        m = getattr(model, name, None)
        if m is not None:
            yield from m.parameters()


__all__ = ["initialize_model", "set_parameter_requires_grad", "ARCH", "InceptionOutputs",
           "input_spec",
           "resnet18", "resnet34", "vgg11_bn", "vgg16", "alexnet", "squeezenet1_0",
           "densenet121", "inception_v3"]
