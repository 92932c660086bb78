"""``GetData``: the reference's per-image torch Dataset (``/root/reference/data_loader.py:6-39``),
kept for API compatibility.  ``__getitem__`` opens ``Dir/FNames[i]`` with PIL; a ``Dir``
containing "train" yields ``(Transform(img), label)``, one containing "test" yields
``(Transform(img), file_name)``.  The reference implicitly returns ``None`` otherwise; here
that case returns ``(Transform(img), label)`` as well.

The engine itself does not use this class in its hot path (see ``data/loader.py``): the
transform runs as a GPU kernel on whole batches.  :func:`default_transform` gives the
reference's train transform (ToTensor -> Resize(bilinear) -> Normalize) as a CPU callable
built on the same reference ops.
"""
from __future__ import annotations

import os
from typing import Callable, Optional, Sequence

import numpy as np
import torch

from .loader import IMAGENET_MEAN, IMAGENET_STD


def default_transform(width: int = 128, height: int = 128, mode: int = 0) -> Callable:
    from ..ops import ref

    def tf(img):
        a = torch.from_numpy(np.asarray(img.convert("RGB")))[None]
        x = ref.preprocess(a, height, width, IMAGENET_MEAN, IMAGENET_STD, mode, 3, torch.float32)
        return x[0].permute(2, 0, 1).contiguous()  # CHW like ToTensor

    return tf


class GetData(torch.utils.data.Dataset):
    def __init__(self, Dir: str, FNames: Sequence[str], Labels: Sequence[int],
                 Transform: Optional[Callable] = None):
        self.dir = Dir
        self.fnames = FNames
        self.transform = Transform or default_transform()
        self.labels = Labels

    def __len__(self):
        return len(self.fnames)

    def __getitem__(self, index):
        from PIL import Image
        x = Image.open(os.path.join(self.dir, self.fnames[index]))
        if "test" in self.dir and "train" not in self.dir:
            return self.transform(x), self.fnames[index]
        return self.transform(x), self.labels[index]
