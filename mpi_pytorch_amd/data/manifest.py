"""Manifest (CSV) handling and per-row image sources.

Reference: rank 0 reads ``test_sample.csv`` / ``train_sample.csv`` (``main.py:73-82``);
in DEBUG it draws ``sample(1000, random_state=0)`` from the test manifest and splits it
80/20 with ``train_test_split`` (800 training rows).  ``GetData`` (``data_loader.py:6-39``)
opens ``TRAIN_DIR/file_name`` with PIL and returns ``(transform(img), label)``; labels
are the raw ``category_id`` values used directly as class indices (``data_loader.py:37``).

Image sources:
* :class:`FolderImages` - real JPEGs decoded by PIL worker threads (PIL releases the
  GIL while decoding), uint8 HWC arrays of varying size;
* :class:`SyntheticImages` - no Herbarium images exist offline (BASELINE.json: synthetic
  data), so each manifest row gets a deterministic pseudo-random uint8 image keyed by its
  file name (same pixels on every rank/epoch) at a fixed "decoded" size.
"""
from __future__ import annotations

import os
import zlib
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

try:
    import pandas as pd
except Exception:  # pragma: no cover
    pd = None


def read_manifests(cfg):
    """Rank-0 manifest read (main.py:73-82).  Returns (train_df, test_df)."""
    if cfg.DEBUG:
        from sklearn.model_selection import train_test_split
        df_test = pd.read_csv(cfg.TEST_CSV)
        sample = df_test.sample(min(cfg.DEBUG_SAMPLE, len(df_test)), random_state=0)
        sample = sample.reset_index(drop=True).copy()
        train_sample, test_sample = train_test_split(sample, test_size=0.2,
                                                     random_state=cfg.seed)
        return train_sample.copy(), test_sample.copy()
    return pd.read_csv(cfg.TRAIN_CSV), pd.read_csv(cfg.TEST_CSV)


def synthetic_manifest(n: int, num_classes: int, seed: int = 0):
    rng = np.random.default_rng(seed)
    return pd.DataFrame({
        "file_name": ["synthetic/{:08d}.jpg".format(i) for i in range(n)],
        "category_id": rng.integers(0, num_classes, size=n),
    })


class SyntheticImages:
    """Deterministic synthetic uint8 HWC images, one per file name (no dataset needed).

    Image ``name`` is a window of one shared uniform-noise texture, at a row/column offset
    derived from crc32(name): generation is a strided memcpy (~GB/s per thread) instead of
    a per-image RNG pass, so the host side never limits the evaluation pipeline."""

    def __init__(self, hw: Tuple[int, int], seed: int = 0):
        self.hw = hw
        rng = np.random.default_rng(seed)
        self.tex = rng.integers(0, 256, size=(2 * hw[0], 2 * hw[1], 3), dtype=np.uint8)

    def load(self, names: Sequence[str], out: Optional[np.ndarray] = None) -> np.ndarray:
        H, W = self.hw
        if out is None:
            out = np.empty((len(names), H, W, 3), dtype=np.uint8)
        for i, n in enumerate(names):
            r, c = self._offset(n)
            out[i] = self.tex[r:r + H, c:c + W]
        return out

    def _offset(self, name) -> Tuple[int, int]:
        H, W = self.hw
        h = zlib.crc32(str(name).encode())
        return h % H, (h // H) % W

    def load_device(self, names: Sequence[str], device) -> torch.Tensor:
        """``load(names)`` produced on ``device`` as one gather from a device copy of the
        texture (bitwise the same images): the training driver's synthetic batches then
        cost no host copy, pinning or H2D transfer."""
        device = torch.device(device)
        if getattr(self, "_tex_dev", None) is None or self._tex_dev.device != device:
            self._tex_dev = torch.from_numpy(self.tex).to(device)
        H, W = self.hw
        rc = torch.tensor([self._offset(n) for n in names], dtype=torch.int64).to(device)
        rows = (rc[:, 0:1] + torch.arange(H, device=device))[:, :, None]
        cols = (rc[:, 1:2] + torch.arange(W, device=device))[:, None, :]
        return self._tex_dev[rows, cols]


class FolderImages:
    """PIL decode of ``root/file_name`` in a thread pool; returns a list of HWC uint8."""

    def __init__(self, root: str, workers: int = 4):
        self.root = root
        self.pool = ThreadPoolExecutor(max_workers=max(1, workers))

    def _one(self, name: str) -> np.ndarray:
        from PIL import Image
        with Image.open(os.path.join(self.root, name)) as im:
            return np.asarray(im.convert("RGB"))

    def load(self, names: Sequence[str]) -> List[np.ndarray]:
        return list(self.pool.map(self._one, names))


def images_available(root: str, names: Sequence[str]) -> bool:
    return bool(names) and os.path.exists(os.path.join(root, str(names[0])))
