"""NHWC building blocks with torchvision-compatible parameter names and state_dict layout.

Internally conv weights are stored ``[K, R, S, C]`` ("KRSC", the layout the implicit-GEMM
MFMA kernels read with 16-byte vector loads along C) and activations are NHWC.  The
state_dict converts to/from torchvision's OIHW at save/load time, so checkpoints keep the
reference contract (``main.py:163-168``: ``model.state_dict()`` of a torchvision model;
loaded by ``evaluation_pipeline.py:142-144`` / ``helpers.py:13``).

``FusedSequential`` keeps torchvision's ``nn.Sequential`` indices (``features.0``,
``features.1`` ...) but executes Conv->BN->ReLU and Conv->ReLU runs as single fused ops.
"""
from __future__ import annotations

import math
import os
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import functional as Fn


def _pair(v) -> Tuple[int, int]:
    if isinstance(v, (tuple, list)):
        return int(v[0]), int(v[1])
    return int(v), int(v)


def _pad_rows(n: int) -> int:
    """Stored output width of a padded classifier (Linear / head conv): a multiple of 32."""
    return n if n % 32 == 0 else (n + 31) // 32 * 32


def _krsc_to_oihw(t):
    return t.permute(0, 3, 1, 2)


def _oihw_to_krsc(t):
    return t.permute(0, 2, 3, 1)


_PAIR_STEM = os.environ.get("MPA_PAIR_STEM", "1") == "1"


class Conv2d(nn.Module):
    """Conv2d with KRSC weight storage. ``state_dict`` exposes OIHW like ``nn.Conv2d``.

    Image-input stems (``in_channels < 8``) store their weight with the channel dim
    zero-padded to 8 (``cin_store``): the input images are produced with 8 channels by the
    preprocess kernel, so the stem conv takes the 16-byte vector gather path; the zero
    channels contribute exactly nothing and receive exactly zero gradient.  The padding is
    invisible in state_dict / optimizer state (sliced off on export, re-added on import).

    **Pixel-pair stems** (image input, horizontal stride 2 - the 7x7/s2 stems of ResNet,
    DenseNet and SqueezeNet, Inception's 3x3/s2): the image is stored with 4 channels
    (RGB + 0) on a zero-bordered canvas (``input_spec``, written directly by the preprocess
    kernel), so two horizontally adjacent pixels are one 16-B, 8-"channel" vector.  A
    stride-2 conv with an S-wide kernel over 4-channel pixels is then exactly a stride-1
    conv with a ceil(S/2)-wide kernel over 8-channel pixel pairs, padding 0: weight
    ``[K][R][S][3]`` is stored as ``[K][R][ceil(S/2)][2 x 4]`` (zero for the 4th channel
    and, for odd S, the column past the kernel).  Against the plain 8-channel layout this
    halves the stem's MFMA work (K = R x 32 instead of R x 2 x 32 for 7x7), its wgrad
    columns (224 vs 392) and the image bytes.  The column past an odd kernel would get a
    nonzero gradient (its input pixels are real), so ``fix_grad`` zeroes it after wgrad;
    the 4th channel's gradient is exactly zero (its input is).
    """

    def __init__(self, in_channels: int, out_channels: int, kernel_size, stride=1, padding=0,
                 bias: bool = True, pad_out: bool = False):
        super().__init__()
        self.in_channels = in_channels
        kh0, kw0 = _pair(kernel_size)
        self.pair = (_PAIR_STEM and in_channels <= 4 and _pair(stride)[1] == 2 and kw0 >= 2)
        self.cin_store = 8 if in_channels < 8 else in_channels
        self.out_channels = out_channels
        # pad_out: store the output channels rounded up to a multiple of 32 (zero filters) -
        # for classifier convs (SqueezeNet's 512 -> 64,500 1x1 head) so their dgrad / wgrad
        # stay on the 16-B LDS-DMA paths; the model slices the logits back
        self.cout_store = _pad_rows(out_channels) if pad_out else out_channels
        self.kernel_size = _pair(kernel_size)
        self.stride = _pair(stride)
        self.padding = _pair(padding)
        kh, kw = self.kernel_size
        self.sp = (kw + 1) // 2  # pixel-pair kernel width
        # geometry of the conv the kernels actually run: (sh, sw, ph, pw)
        if self.pair:
            self.kgeom = (self.stride[0], 1, 0, 0)
        else:
            self.kgeom = (self.stride[0], self.stride[1], self.padding[0], self.padding[1])
        w = torch.empty(out_channels, in_channels, kh, kw)
        nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        self.weight = nn.Parameter(self._imp(w).contiguous())
        self.weight._mpa_export = self._exp
        self.weight._mpa_import = self._imp
        # (K, R*S, C) of the stored KRSC weight: the arena keeps a [C][R*S][K] copy for dgrad
        ks = self.sp if self.pair else kw
        self.weight._mpa_tlayout = (self.cout_store, kh * ks, self.cin_store)
        if bias:
            fan_in = in_channels * kh * kw
            bound = 1 / math.sqrt(fan_in)
            b = torch.empty(out_channels).uniform_(-bound, bound)
            self.bias = nn.Parameter(self._imp_bias(b))
            if self.cout_store != out_channels:
                self.bias._mpa_export = self._exp_bias
                self.bias._mpa_import = self._imp_bias
        else:
            self.register_parameter("bias", None)

    def _exp(self, t):  # internal KRSC (maybe channel padded / pixel pairs) -> OIHW
        if self.pair:  # [K][R][Sp][2 x 4] -> [K][R][S][3]
            kh, kw = self.kernel_size
            t = t.reshape(t.shape[0], kh, 2 * self.sp, 4)[:, :, :kw, :self.in_channels]
        elif self.cin_store != self.in_channels:
            t = t[..., :self.in_channels]
        if self.cout_store != self.out_channels:
            t = t[:self.out_channels]
        return _krsc_to_oihw(t)

    def _imp(self, t):  # OIHW -> internal KRSC
        t = _oihw_to_krsc(t)
        if self.pair:
            kh, kw = self.kernel_size
            t = F.pad(t, (0, 4 - self.in_channels, 0, 2 * self.sp - kw))
            t = t.reshape(t.shape[0], kh, self.sp, 8)
        elif self.cin_store != self.in_channels:
            t = F.pad(t, (0, self.cin_store - self.in_channels))
        if t.shape[0] < self.cout_store:
            t = F.pad(t, (0, 0, 0, 0, 0, 0, 0, self.cout_store - t.shape[0]))
        return t

    def _exp_bias(self, t):
        return t[:self.out_channels]

    def _imp_bias(self, t):
        return F.pad(t, (0, self.cout_store - t.shape[0])) if t.shape[0] < self.cout_store else t

    # init helpers operate in OIHW space so the distributions match torchvision
    def init_(self, fn) -> "Conv2d":
        with torch.no_grad():
            w = torch.empty(self.out_channels, self.in_channels, *self.kernel_size)
            fn(w)
            self.weight.copy_(self._imp(w))
        return self

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        super()._save_to_state_dict(destination, prefix, keep_vars)
        k = prefix + "weight"
        if k in destination:
            w = destination[k]
            destination[k] = self._exp(w) if keep_vars else self._exp(w).contiguous()
        k = prefix + "bias"
        if k in destination and destination[k] is not None and self.cout_store != self.out_channels:
            b = self._exp_bias(destination[k])
            destination[k] = b if keep_vars else b.contiguous()

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        k = prefix + "weight"
        if k in state_dict:
            w = state_dict[k]
            if tuple(w.shape) == (self.out_channels, self.in_channels, *self.kernel_size):
                state_dict[k] = self._imp(w)
        k = prefix + "bias"
        if k in state_dict and tuple(state_dict[k].shape) == (self.out_channels,):
            state_dict[k] = self._imp_bias(state_dict[k])
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys,
                                      unexpected_keys, error_msgs)

    def forward(self, x, relu: bool = False):
        return Fn.conv_act(x, self, relu=relu)

    def input_spec(self, hw) -> dict:
        """Layout the data pipeline should produce for an ``hw`` image fed to this conv:
        ``cpad`` channels on a zero canvas ``pad`` = (top, bottom, left, right)."""
        if not self.pair:
            return {"cpad": self.cin_store, "pad": None}
        H, W = hw
        (kh, kw), (ph, pw) = self.kernel_size, self.padding
        Q = (W + 2 * pw - kw) // 2 + 1
        right = 2 * (Q - 1 + self.sp) - W - pw
        return {"cpad": 4, "pad": (ph, ph, pw, right)}

    def fit_input(self, x):
        """Bring an image input into the stored layout.  Plain convs: zero-pad the channel
        dim to the stored width (no-op normally).  Pixel-pair stems: a 4-channel input is
        taken to be the pre-padded canvas of ``input_spec`` (what the data pipeline
        produces); 3/8-channel images are converted here.  Returns the [N][Hp][Wp/2][8]
        pixel-pair view."""
        c = x.shape[-1]
        if self.pair:
            if c != 4:
                N, H, W = x.shape[:3]
                t, b, l, r = self.input_spec((H, W))["pad"]
                if r < 0:
                    raise ValueError("pixel-pair stem: image width %d too small" % W)
                x = F.pad(x[..., :3], (0, 1, l, r, t, b))
            N, Hp, Wp = x.shape[:3]
            if Wp % 2:
                raise ValueError("pixel-pair stem: canvas width %d is odd" % Wp)
            return x.contiguous().view(N, Hp, Wp // 2, 8)
        if c < self.cin_store:
            x = F.pad(x, (0, self.cin_store - c))
        return x

    def fix_grad(self, g) -> None:
        """Pixel-pair stem with an odd kernel width: the stored column past the kernel
        (second pixel of the last pair) must keep exactly zero weight."""
        kw = self.kernel_size[1]
        if self.pair and kw % 2 and g is not None:
            # g as [K * kh][sp * 8]: the last pair's second pixel = columns (sp-1)*8+4 .. sp*8
            Fn.K(g).zero_cols_f32(g, self.sp * 8, (self.sp - 1) * 8 + 4, 4)

    def extra_repr(self):
        return "{}, {}, kernel_size={}, stride={}, padding={}, bias={}".format(
            self.in_channels, self.out_channels, self.kernel_size, self.stride, self.padding,
            self.bias is not None)


class BatchNorm2d(nn.Module):
    """BatchNorm over the channel (last, NHWC) dim; same names/buffers as nn.BatchNorm2d."""

    def __init__(self, num_features: int, eps: float = 1e-5, momentum: float = 0.1):
        super().__init__()
        self.num_features = num_features
        self.eps = eps
        self.momentum = momentum
        self.weight = nn.Parameter(torch.ones(num_features))
        self.bias = nn.Parameter(torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))
        # host shadow of num_batches_tracked (the device buffer is bumped inside the BN
        # kernel): momentum=None's cumulative average needs the count without a device sync
        self._batches_host = 0

    def momentum_value(self) -> float:
        """Momentum for this training step (nn.BatchNorm2d semantics, incl. None = cumulative
        moving average 1 / num_batches_tracked), advancing the host batch count."""
        self._batches_host += 1
        if self.momentum is None:
            return 1.0 / self._batches_host
        return float(self.momentum)

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)
        key = prefix + "num_batches_tracked"
        if key in state_dict:
            self._batches_host = int(state_dict[key])

    def forward(self, x, relu: bool = False, stats=None):
        return Fn.bn_act(x, self, relu=relu, stats=stats)

    def extra_repr(self):
        return "{}, eps={}, momentum={}".format(self.num_features, self.eps, self.momentum)


class Linear(nn.Module):
    """Linear layer.  ``in_chw=(C,H,W)`` marks a layer fed by an NHWC flatten: its input
    columns are stored in (h,w,c) order internally and exported in torchvision's
    NCHW-flatten (c,h,w) order.

    The output dim is stored rounded up to a multiple of 32 (``out_store``) with zero
    weight rows and bias entries: a 64,500-class head becomes 64,512 rows, so its forward,
    dgrad, wgrad and bias-gradient all run on the 16-B-granular LDS-DMA GEMM paths
    instead of scalar/8-byte fallbacks.  ``forward`` returns the first ``out_features``
    columns (a view); the padding is invisible in state_dict and optimizer state, and the
    padded rows never receive gradient (the cross-entropy backward writes zeros there).
    """

    def __init__(self, in_features: int, out_features: int, bias: bool = True,
                 in_chw: Optional[Tuple[int, int, int]] = None):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.out_store = _pad_rows(out_features)
        self.in_chw = in_chw
        w = torch.empty(out_features, in_features)
        nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        self.weight = nn.Parameter(self._imp(w).contiguous())
        if in_chw is not None or self.out_store != out_features:
            self.weight._mpa_export = self._exp
            self.weight._mpa_import = self._imp
        # [in][out] copy for dgrad - except for the wide classifier heads (64,500 classes):
        # their dgrad (M = batch, N = in, K = 64,512, split-K) reads the forward weight with
        # transposing LDS loads as fast or faster (tools/bench_head.py: 61.9 vs 65.7 us), and
        # skipping the copy saves transposing 33 M weights (~24 us) after every update
        if out_features < 16384:
            self.weight._mpa_tlayout = (self.out_store, 1, in_features)
        if bias:
            bound = 1 / math.sqrt(in_features)
            b = torch.empty(out_features).uniform_(-bound, bound)
            self.bias = nn.Parameter(self._imp_bias(b))
            if self.out_store != out_features:
                self.bias._mpa_export = self._exp_bias
                self.bias._mpa_import = self._imp_bias
        else:
            self.register_parameter("bias", None)

    def _exp(self, t):  # internal (o_store, h*w*c) -> torchvision (o, c*h*w)
        t = t[:self.out_features]
        if self.in_chw is None:
            return t
        C, H, W = self.in_chw
        return t.reshape(t.shape[0], H, W, C).permute(0, 3, 1, 2).reshape(t.shape[0], C * H * W)

    def _imp(self, t):
        if self.in_chw is not None:
            C, H, W = self.in_chw
            t = t.reshape(t.shape[0], C, H, W).permute(0, 2, 3, 1).reshape(t.shape[0], H * W * C)
        if t.shape[0] < self.out_store:
            t = F.pad(t, (0, 0, 0, self.out_store - t.shape[0]))
        return t

    def _exp_bias(self, t):
        return t[:self.out_features]

    def _imp_bias(self, t):
        return F.pad(t, (0, self.out_store - t.shape[0])) if t.shape[0] < self.out_store else t

    def init_(self, fn) -> "Linear":
        with torch.no_grad():
            w = torch.empty(self.out_features, self.in_features)
            fn(w)
            self.weight.copy_(self._imp(w))
        return self

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        super()._save_to_state_dict(destination, prefix, keep_vars)
        k = prefix + "weight"
        if k in destination:
            w = self._exp(destination[k])
            destination[k] = w if keep_vars else w.contiguous()
        k = prefix + "bias"
        if k in destination and destination[k] is not None:
            b = self._exp_bias(destination[k])
            destination[k] = b if keep_vars else b.contiguous()

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        k = prefix + "weight"
        if k in state_dict and tuple(state_dict[k].shape) == (self.out_features, self.in_features):
            state_dict[k] = self._imp(state_dict[k])
        k = prefix + "bias"
        if k in state_dict and tuple(state_dict[k].shape) == (self.out_features,):
            state_dict[k] = self._imp_bias(state_dict[k])
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys,
                                      unexpected_keys, error_msgs)

    def forward(self, x, relu: bool = False):
        return Fn.linear_act(x, self, relu=relu)

    def extra_repr(self):
        return "in_features={}, out_features={}, bias={}".format(
            self.in_features, self.out_features, self.bias is not None)


class ReLU(nn.Module):
    def __init__(self, inplace: bool = False):
        super().__init__()

    def forward(self, x):
        # only reached when not fused into a producer; keep it a kernel op
        return Fn.K(x).relu_fwd(x) if not x.requires_grad else _relu_autograd(x)


def _relu_autograd(x):
    return _ReLUFn.apply(x)


class _ReLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = Fn.K(x).relu_fwd(x)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return Fn.K(dy).act_bwd(dy.contiguous(), y, Fn._empty(dy))


class MaxPool2d(nn.Module):
    def __init__(self, kernel_size, stride=None, padding=0, ceil_mode=False):
        super().__init__()
        self.kernel_size = _pair(kernel_size)
        self.stride = _pair(stride if stride is not None else kernel_size)
        self.padding = _pair(padding)
        self.ceil_mode = ceil_mode

    def forward(self, x):
        return Fn.max_pool2d(x, self.kernel_size, self.stride, self.padding, self.ceil_mode)


class AvgPool2d(nn.Module):
    def __init__(self, kernel_size, stride=None, padding=0, ceil_mode=False,
                 count_include_pad=True):
        super().__init__()
        self.kernel_size = _pair(kernel_size)
        self.stride = _pair(stride if stride is not None else kernel_size)
        self.padding = _pair(padding)
        self.ceil_mode = ceil_mode
        self.count_include_pad = count_include_pad

    def forward(self, x):
        return Fn.avg_pool2d(x, self.kernel_size, self.stride, self.padding, self.ceil_mode,
                             self.count_include_pad)


class AdaptiveAvgPool2d(nn.Module):
    def __init__(self, output_size):
        super().__init__()
        self.output_size = _pair(output_size)

    def forward(self, x):
        return Fn.adaptive_avg_pool2d(x, self.output_size)


class Dropout(nn.Module):
    def __init__(self, p: float = 0.5, inplace: bool = False):
        super().__init__()
        self.p = p

    def forward(self, x):
        return Fn.dropout(x, self.p, self.training)


class Flatten(nn.Module):
    def forward(self, x):
        return x.reshape(x.shape[0], -1)


# MPA_SEQ_LINK=0: conv -> ReLU -> conv chains of the feature stacks run the separate ReLU
# backward (act_bwd) / BN reduce pass instead of the consumer dgrad's fused reduction
_LINK = os.environ.get("MPA_SEQ_LINK", "1") == "1"


class FusedSequential(nn.Sequential):
    """``nn.Sequential`` with torchvision indices, executed with producer fusion:
    Conv(no bias)->BN[->ReLU] => conv_bn_act; Conv->ReLU => conv_act(relu); Linear->ReLU
    => linear_act(relu)."""

    def groups(self):
        """The fused execution groups: (first index, end index, kind) over the children."""
        mods = list(self._modules.values())
        out, i, n = [], 0, len(mods)
        while i < n:
            m = mods[i]
            nxt = mods[i + 1] if i + 1 < n else None
            nxt2 = mods[i + 2] if i + 2 < n else None
            if isinstance(m, Conv2d) and isinstance(nxt, BatchNorm2d):
                k = 3 if isinstance(nxt2, ReLU) else 2
                out.append((i, i + k, "conv_bn_relu" if k == 3 else "conv_bn"))
            elif isinstance(m, (Conv2d, Linear, BatchNorm2d)) and isinstance(nxt, ReLU):
                k = 2
                out.append((i, i + 2, "relu"))
            else:
                k = 1
                out.append((i, i + 1, "plain"))
            i += k
        return out

    def run_group(self, g, x, link_in=None, link_out=None):
        """Execute fused group ``g`` = (first, end, kind) of :meth:`groups` on ``x``;
        ``link_in`` / ``link_out``: BN-backward hand-offs (Fn.BNLink) with the neighbouring
        conv group (see :meth:`links`)."""
        mods = list(self._modules.values())
        i, _e, kind = g
        if kind.startswith("conv_bn"):
            return Fn.conv_bn_act(x, mods[i], mods[i + 1], relu=kind == "conv_bn_relu",
                                  link_in=link_in, link_out=link_out)
        if kind == "relu":
            if isinstance(mods[i], Conv2d):
                return Fn.conv_act(x, mods[i], relu=True, link_in=link_in, link_out=link_out)
            return mods[i](x, relu=True)
        if link_in is not None and isinstance(mods[i], MaxPool2d):
            m = mods[i]
            return Fn.max_pool2d(x, m.kernel_size, m.stride, m.padding, m.ceil_mode,
                                 link_in=link_in)
        return mods[i](x)

    def links(self, gs):
        """Which consecutive groups hand the backward over: a conv -> (BN ->) ReLU group
        whose output feeds ONLY the next conv group (VGG / AlexNet feature stacks).  The
        consumer's dgrad then applies the producer's ReLU mask and reduces its BN (or
        bias) gradient sums in its epilogue - no reduce / act_bwd pass (Fn.BNLink)."""
        mods = list(self._modules.values())
        out = [False] * len(gs)
        if not (self.training and torch.is_grad_enabled() and _LINK):
            return out
        for k in range(len(gs) - 1):
            (i, _e, kind), (j, _f, kind2) = gs[k], gs[k + 1]
            if (kind in ("relu", "conv_bn_relu") and isinstance(mods[i], Conv2d)
                    and kind2 in ("relu", "conv_bn_relu", "conv_bn")
                    and isinstance(mods[j], Conv2d) and not mods[j].pair):
                out[k] = True
            # conv -> ReLU -> 2x2/s2 max pool (VGG block ends): the pool's backward applies
            # the ReLU mask and reduces the conv's bias gradient (no act_bwd pass)
            m = mods[j]
            if (kind == "relu" and isinstance(mods[i], Conv2d) and kind2 == "plain"
                    and isinstance(m, MaxPool2d) and m.kernel_size == (2, 2)
                    and m.stride == (2, 2) and m.padding == (0, 0)):
                out[k] = True
        return out

    def forward(self, x):
        run = self.run_group
        gs = self.groups()
        lk = self.links(gs)
        link = None
        for k, g in enumerate(gs):
            nxt = Fn.BNLink() if lk[k] else None
            x = run(g, x, link_in=link, link_out=nxt)
            link = nxt
        return x
