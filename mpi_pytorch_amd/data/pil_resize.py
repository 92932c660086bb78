"""PIL-exact bicubic resize (the evaluation transform) - coefficient tables and the
host reference.

Reference: ``evaluation_pipeline.py:89`` resizes a uint8 PIL image with ``Image.resize``
(default BICUBIC, antialiased: the filter support grows with the downscale factor), then
``ToTensor`` (u8 / 255) and ``Normalize`` (``evaluation_pipeline.py:116-122``).  Pillow's
8-bit resampler is fixed-point and two-pass:

* per output position, a window [xmin, xmin + xsize) of source positions and double
  weights ``bicubic((x + xmin - center + 0.5) / filterscale)`` normalised by their
  (sequential) sum, then rounded to 22-bit fixed point (``PRECISION_BITS = 32 - 8 - 2``);
* a horizontal pass first, whose result is rounded and clipped to uint8, then a vertical
  pass over that uint8 image: ``clip8((2^21 + sum_i u8_i * k_i) >> 22)``.

:func:`coeffs` reproduces the tables bit for bit (the same double arithmetic and C
truncations), :func:`resize_u8` the two passes; ``tests/test_pil_parity_cpu.py`` compares
both with ``PIL.Image.resize`` itself.  The GPU kernels (``csrc/kernels/preprocess.hip``,
``preprocess_pil``) consume the same integer tables, so device output equals this module's
(and therefore PIL's) uint8 image exactly before normalisation.
"""
from __future__ import annotations

import math
from functools import lru_cache
from typing import Sequence, Tuple

import numpy as np

PRECISION_BITS = 32 - 8 - 2  # Pillow's 8-bpc fixed point


def _bicubic(x: np.ndarray) -> np.ndarray:
    a = -0.5
    x = np.abs(x)
    out = np.zeros_like(x)
    m1 = x < 1.0
    m2 = (x >= 1.0) & (x < 2.0)
    xm = x[m1]
    out[m1] = ((a + 2.0) * xm - (a + 3.0)) * xm * xm + 1
    xm = x[m2]
    out[m2] = (((xm - 5) * xm + 8) * xm - 4) * a
    return out


@lru_cache(maxsize=256)
def coeffs(in_size: int, out_size: int) -> Tuple[np.ndarray, np.ndarray, int]:
    """Pillow ``precompute_coeffs`` + ``normalize_coeffs_8bpc`` for the full-image box.

    Returns (bounds int32 [out, 2] = (xmin, xsize), kk int32 [out, ksize], ksize)."""
    scale = float(in_size) / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    ss = 1.0 / filterscale
    center = (np.arange(out_size, dtype=np.float64) + 0.5) * scale
    xmin = np.trunc(center - support + 0.5).astype(np.int64)   # C (int) cast
    xmin = np.maximum(xmin, 0)
    xmax = np.minimum(np.trunc(center + support + 0.5).astype(np.int64), in_size) - xmin
    t = np.arange(ksize, dtype=np.int64)
    w = _bicubic((t[None, :] + xmin[:, None] - center[:, None] + 0.5) * ss)
    w[t[None, :] >= xmax[:, None]] = 0.0
    ww = np.cumsum(w, axis=1)[:, -1]  # left-to-right double sum, like the C loop
    k = np.where(ww[:, None] != 0.0, w / np.where(ww == 0.0, 1.0, ww)[:, None], w)
    one = float(1 << PRECISION_BITS)
    kk = np.where(k < 0, np.trunc(-0.5 + k * one), np.trunc(0.5 + k * one)).astype(np.int32)
    kk[t[None, :] >= xmax[:, None]] = 0
    bounds = np.stack([xmin, xmax], axis=1).astype(np.int32)
    return bounds, kk, ksize


def _pass(img: np.ndarray, axis: int, in_size: int, out_size: int) -> np.ndarray:
    """One fixed-point pass along ``axis`` (1 = rows/vertical, 2 = columns/horizontal) of
    a uint8 [B, H, W, C] batch."""
    bounds, kk, ksize = coeffs(in_size, out_size)
    idx = np.minimum(bounds[:, :1] + np.arange(ksize)[None, :], in_size - 1)  # [out, k]
    src = np.take(img.astype(np.int64), idx, axis=axis)  # axis -> (out, k)
    if axis == 2:   # [B, H, out, k, C]
        acc = (src * kk[None, None, :, :, None]).sum(axis=3)
    else:           # [B, out, k, W, C]
        acc = (src * kk[None, :, :, None, None]).sum(axis=2)
    acc = (acc + (1 << (PRECISION_BITS - 1))) >> PRECISION_BITS
    return np.clip(acc, 0, 255).astype(np.uint8)


def resize_u8(img: np.ndarray, out_hw: Tuple[int, int]) -> np.ndarray:
    """``PIL.Image.resize((W, H), BICUBIC)`` of every image of a uint8 [B, H, W, 3] batch
    (horizontal pass first; a pass whose size does not change is skipped, as in PIL)."""
    img = np.asarray(img, dtype=np.uint8)
    squeeze = img.ndim == 3
    if squeeze:
        img = img[None]
    H, W = img.shape[1:3]
    OH, OW = out_hw
    if OW != W:
        img = _pass(img, 2, W, OW)
    if OH != H:
        img = _pass(img, 1, H, OH)
    return img[0] if squeeze else img


def normalize(u8: np.ndarray, mean: Sequence[float], std: Sequence[float]) -> np.ndarray:
    """``ToTensor`` + ``Normalize`` in float32 with torchvision's operation order:
    (u8 / 255 - mean) / std, every step rounded to float32."""
    x = u8.astype(np.float32) / np.float32(255.0)
    m = np.asarray(mean, dtype=np.float32)
    s = np.asarray(std, dtype=np.float32)
    return (x - m) / s


class TableCache:
    """Device copies of the integer tables, concatenated per batch.

    For a batch whose images have source extents (h_i, w_i), ``tables(extents, out_hw)``
    returns the int32 device tensors the ``preprocess_pil`` kernels read:
    ``hb``/``hk`` (horizontal bounds / coefficients of every distinct source width,
    stacked, rows padded to ``kh`` taps), ``vb``/``vk`` likewise for heights, and ``sel``
    [B, 2] = each image's (width table, height table) index.  Uniform batches hit a cache."""

    def __init__(self, device):
        import torch
        self.torch = torch
        self.device = device
        self._cache = {}

    def _stack(self, sizes, out):
        tabs = [coeffs(int(s), out) for s in sizes]
        k = max(t[2] for t in tabs)
        b = np.concatenate([t[0] for t in tabs], 0)
        kk = np.concatenate([np.pad(t[1], ((0, 0), (0, k - t[2]))) for t in tabs], 0)
        return b, kk, k

    def tables(self, extents: np.ndarray, out_hw: Tuple[int, int], pitch: Tuple[int, int]):
        """(ext, sel, hb, hk, kh, vb, vk, kv) for the ``preprocess_pil`` binding.  Checks on
        the host what the kernels index: every extent inside the slot pitch, every table
        window inside its source size (so inside the image)."""
        torch = self.torch
        ext = np.asarray(extents, dtype=np.int64).reshape(-1, 2)
        key = (ext.tobytes(), tuple(out_hw), tuple(pitch))
        hit = self._cache.get(key)
        if hit is not None:
            return hit
        if (ext < 1).any() or (ext[:, 0] > pitch[0]).any() or (ext[:, 1] > pitch[1]).any():
            raise ValueError("preprocess: image extents %s outside the slot pitch %s"
                             % (ext.tolist(), tuple(pitch)))
        ws, wi = np.unique(ext[:, 1], return_inverse=True)
        hs, hi = np.unique(ext[:, 0], return_inverse=True)
        hb, hk, kh = self._stack(ws, out_hw[1])
        vb, vk, kv = self._stack(hs, out_hw[0])
        for b, sizes in ((hb, ws), (vb, hs)):
            lim = np.repeat(sizes, b.shape[0] // len(sizes))
            if (b[:, 0] < 0).any() or (b[:, 0] + b[:, 1] > lim).any():
                raise AssertionError("PIL resize table window outside its source")
        sel = np.stack([wi, hi], 1).astype(np.int32)
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(self.device)
        out = (dev(ext), dev(sel), dev(hb), dev(hk), int(kh), dev(vb), dev(vk), int(kv))
        if len(self._cache) > 64:
            self._cache.clear()
        self._cache[key] = out
        return out


def reference(img_u8, out_hw, mean, std, extents=None) -> np.ndarray:
    """Host oracle of the eval transform on a uint8 [B, Hp, Wp, 3] batch whose image b
    occupies [:h_b, :w_b]: PIL resize -> ToTensor -> Normalize, float32 [B, OH, OW, 3]."""
    img = np.asarray(img_u8)
    out = np.empty((img.shape[0], out_hw[0], out_hw[1], 3), dtype=np.float32)
    for b in range(img.shape[0]):
        h, w = (img.shape[1], img.shape[2]) if extents is None else tuple(extents[b])
        out[b] = normalize(resize_u8(img[b, :h, :w], out_hw), mean, std)
    return out
