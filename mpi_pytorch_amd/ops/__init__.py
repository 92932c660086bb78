"""Kernel-backed ops.  ``functional`` holds the autograd layer; ``_ext`` the native
module loader; ``ref`` the plain-PyTorch CPU path / test oracle."""
from . import functional  # noqa: F401
from .functional import (conv_bn_act, conv_act, bn_act, linear_act, max_pool2d,  # noqa: F401
                         avg_pool2d, adaptive_avg_pool2d, dropout, cross_entropy,
                         count_correct, preprocess)
