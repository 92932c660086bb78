"""Device-side batch pipeline: native pinned ring -> async H2D on a copy stream -> GPU
preprocess kernel (resize + normalize + bf16 NHWC) on the copy stream, one batch ahead.

Replaces the reference's serial ``DataLoader(num_workers=0)`` + per-image PIL/torchvision
transform (``/root/reference/main.py:62-65,99-102``, ``data_loader.py:29-37``): host
threads produce uint8 batches ahead of time (``csrc/runtime/runtime.cpp``), the copy of
batch i+1 overlaps compute on batch i, and the transform runs as one HIP kernel
(``csrc/kernels/preprocess.hip``).  On CPU the same interface yields fp32 NHWC batches
computed by the reference ops.
"""
from __future__ import annotations

from typing import Iterator, Optional, Tuple

import numpy as np
import torch

from ..ops import functional as Fn

IMAGENET_MEAN = (0.485, 0.456, 0.406)   # main.py:65
IMAGENET_STD = (0.229, 0.224, 0.225)


def _ext():
    from ..ops import _ext as E
    return E.ext()


class SyntheticSource:
    """CPU fallback-free synthetic source (numpy); used on the CPU path and in tests."""

    def __init__(self, batch: int, hw: Tuple[int, int], num_classes: int, seed: int = 0,
                 start_index: int = 0, stride: int = 1):
        self.batch = batch
        self.hw = hw
        self.nc = num_classes
        self.seed = seed
        self.index = start_index
        self.stride = stride

    def next(self):
        rng = np.random.default_rng(self.seed * 1_000_003 + self.index)
        self.index += self.stride
        img = rng.integers(0, 256, size=(self.batch, self.hw[0], self.hw[1], 3), dtype=np.uint8)
        lab = rng.integers(0, self.nc, size=(self.batch,), dtype=np.int64)
        return torch.from_numpy(img), torch.from_numpy(lab)


class DevicePrefetcher:
    """Yields ``(images_nhwc, labels)`` on ``device`` ready for the model.

    GPU: backed by the native ``BatchRing`` (pinned slots, C++ producer threads); a slot is
    returned to the ring once its H2D copy event has completed.  ``out_hw`` is the model
    input size; ``src_hw`` the decoded image size (resize happens on the GPU when they
    differ, bilinear like the reference train transform).

    ``lookahead`` (default): each ``next()`` also issues the NEXT batch's H2D copy and
    preprocess kernel on the copy stream, so they run beside the current step's kernels
    instead of at the head of the next step, where nothing else is ready to run (the
    preprocess is 0.2 ms of a 37 ms ResNet-18 b2048 step, profiles/r18_b2048_step_*_r6.txt).
    """

    def __init__(self, device: torch.device, batch: int, src_hw: Tuple[int, int],
                 out_hw: Tuple[int, int], num_classes: int, seed: int = 0, rank: int = 0,
                 world: int = 1, depth: int = 4, threads: int = 2, mode: int = 0,
                 cpad: int = 8, ring=None, pad=None, lookahead: bool = True):
        self.device = torch.device(device)
        self.batch = batch
        self.src_hw = src_hw
        self.out_hw = out_hw
        self.mode = mode
        self.cpad = cpad
        self.pad = list(pad) if pad else []  # zero canvas border (models.input_spec)
        self.cuda = self.device.type == "cuda"
        if self.cuda:
            self.ring = ring if ring is not None else _ext().BatchRing(
                batch, src_hw[0], src_hw[1], num_classes, depth, threads, seed, rank, world, True)
            self.copy_stream = torch.cuda.Stream(device=self.device)
            self._pending = []  # (slot, event)
            self.lookahead = lookahead
            self._ahead = None  # (x, labels, ready event) issued by the previous next()
        else:
            self.src = SyntheticSource(batch, src_hw, num_classes, seed, rank, world)

    def _recycle(self, force: bool = False) -> None:
        keep = []
        depth = self.ring.depth()
        for k, (slot, ev) in enumerate(self._pending):
            # never hold every slot: the ring could then produce nothing and acquire()
            # would wait forever - wait for the oldest copies instead
            if force or ev.query() or len(self._pending) - k >= depth - 1:
                ev.synchronize()
                self.ring.release(slot)
            else:
                keep.append((slot, ev))
        self._pending = keep

    def next(self):
        if not self.cuda:
            img, lab = self.src.next()
            x = Fn.preprocess(img, self.out_hw, IMAGENET_MEAN, IMAGENET_STD, self.mode, self.cpad,
                              out_dtype=torch.float32, pad=self.pad)
            return x, lab
        if self._ahead is None:
            self._ahead = self._issue()
        x, lab_d, ready = self._ahead
        self._ahead = None
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(ready)
        x.record_stream(cur)
        lab_d.record_stream(cur)
        if self.lookahead:
            self._ahead = self._issue()
        return x, lab_d

    def _issue(self):
        """Acquire the next ring slot; its H2D copy and preprocess go on the copy stream."""
        self._recycle()
        slot, img_h, lab_h, _bidx = self.ring.acquire()
        cs = self.copy_stream
        with torch.cuda.stream(cs):
            img_d = img_h.to(self.device, non_blocking=True)
            lab_d = lab_h.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(cs)  # the pinned slot is free once the copy has landed
            x = _ext().preprocess(img_d, self.out_hw[0], self.out_hw[1], list(IMAGENET_MEAN),
                                  list(IMAGENET_STD), self.mode, self.cpad, self.pad)
            ready = torch.cuda.Event()
            ready.record(cs)
        self._pending.append((slot, ev))
        return x, lab_d, ready

    def ring_stats(self, reset: bool = True) -> Optional[dict]:
        """Consumer starvation of the native ring since the last reset: ``acquires`` (batches
        taken), ``waits`` (of them, how many found their batch not produced yet) and
        ``blocked_ms`` (host time spent waiting for producers).  None on the CPU path."""
        if not self.cuda:
            return None
        n, w, ms = self.ring.stats(reset)
        return {"acquires": int(n), "waits": int(w), "blocked_ms": round(float(ms), 3)}

    def __iter__(self) -> Iterator:
        while True:
            yield self.next()

    def close(self) -> None:
        if self.cuda:
            if self._ahead is not None:
                self._ahead[2].synchronize()
                self._ahead = None
            self._recycle(force=True)
            self.ring.stop()
