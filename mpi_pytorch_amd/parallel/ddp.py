"""Bucketed gradient all-reduce overlapped with backward (the DP engine's comm half).

Replaces the reference's per-parameter, blocking, post-backward loop
``mpi_avg_grads`` (``/root/reference/mpi_tools.py:30-37``, called at ``main.py:154``).

Design for MI355X / RCCL over xGMI:

* Buckets are cut from the flat fp32 gradient arena (:mod:`.arena`) at parameter
  boundaries, ``bucket_mb`` each (a parameter larger than a bucket gets its own).  The
  default 16 MiB is sized for the exposed tail: the LAST bucket (layer2..stem) can only
  start when backward ends, so it is kept small (ResNet-18 @64,500: 126 + 9 + 9.5 + 16 +
  8.4 MiB), while 8-16 MiB messages still run near RCCL's large-message ring bandwidth
  on one xGMI link per ring hop.  Since
  the arena is in reverse registration order, bucket 0 holds the classifier head, whose
  gradient is produced first; its all-reduce runs under the whole conv backward.
* Each backward kernel calls ``arena.notify(p)`` after its weight-gradient launch.  When a
  bucket's last parameter lands, its ``all_reduce`` is issued asynchronously.  With the
  ``nccl`` (RCCL) backend the collective runs on RCCL's own HIP stream, ordered after the
  producing kernels by an event - so it overlaps the rest of backward.
* The reduction is a SUM; the 1/N average of ``mpi_tools.py:36`` is folded into the fused
  optimizer kernel's ``grad_scale`` (no extra pass over the gradients).
* Optional bf16 wire format halves xGMI bytes (cast kernels around the collective).
* ``world_size == 1`` is a no-op, like ``mpi_tools.py:32-33``.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .arena import ParamArena


class GradBucketer:
    def __init__(self, arena: ParamArena, world_size: int, bucket_mb: float = 16.0,
                 overlap: bool = True, comm_dtype: str = "fp32", group=None):
        self.arena = arena
        self.world_size = world_size
        self.overlap = overlap
        self.comm_dtype = comm_dtype
        self.group = group
        cap = max(int(bucket_mb * 1024 * 1024 // 4), 1)
        self.buckets: List[List[nn.Parameter]] = []
        self.ranges: List[tuple] = []
        cur: List[nn.Parameter] = []
        start = 0
        end = 0
        for p in arena.trainable:
            o, e = arena.slice_of(p)
            # close the bucket when p would overflow it - unless it is still tiny (the
            # classifier bias ahead of the 126 MiB head weight): no sub-MiB collective
            if cur and (e - start) > cap and (end - start) >= cap // 8:
                self.buckets.append(cur)
                self.ranges.append((start, end))
                cur, start = [], o
            if not cur:
                start = o
            cur.append(p)
            end = arena.offsets[id(p)] + ((p.numel() + 63) // 64) * 64
        if cur:
            self.buckets.append(cur)
            self.ranges.append((start, end))
        self.bucket_of = {}
        for bi, ps in enumerate(self.buckets):
            for p in ps:
                self.bucket_of[id(p)] = bi
        self._pending = [0] * len(self.buckets)
        self._works: List[Optional[object]] = [None] * len(self.buckets)
        self._wire: List[Optional[torch.Tensor]] = [None] * len(self.buckets)
        self.active = world_size > 1
        if self.active:
            arena.add_listener(self._on_grad)
        self.reset()

    # ------------------------------------------------------------------------------
    def reset(self) -> None:
        for i, ps in enumerate(self.buckets):
            self._pending[i] = len(ps)
            self._works[i] = None

    def _on_grad(self, p: nn.Parameter) -> None:
        if not (self.active and self.overlap):
            return
        bi = self.bucket_of.get(id(p))
        if bi is None:
            return
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._launch(bi)

    def _launch(self, bi: int) -> None:
        if self._works[bi] is not None:
            return
        s, e = self.ranges[bi]
        g = self.arena.grad[s:e]
        if self.comm_dtype == "bf16" and g.is_cuda:
            w = g.to(torch.bfloat16)
            self._wire[bi] = w
            self._works[bi] = dist.all_reduce(w, op=dist.ReduceOp.SUM, group=self.group,
                                              async_op=True)
        else:
            self._works[bi] = dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group,
                                              async_op=True)

    def finish(self) -> None:
        """Issue any bucket not yet launched, then make the compute stream wait for all."""
        if not self.active:
            return
        for bi in range(len(self.buckets)):
            if self._works[bi] is None:
                self._launch(bi)
        for bi in range(len(self.buckets)):
            w = self._works[bi]
            if w is not None:
                w.wait()
            if self._wire[bi] is not None:
                s, e = self.ranges[bi]
                self.arena.grad[s:e].copy_(self._wire[bi])
                self._wire[bi] = None
        self.reset()

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world_size

    def describe(self) -> List[dict]:
        return [{"bucket": i, "params": len(ps), "numel": r[1] - r[0],
                 "bytes": (r[1] - r[0]) * 4}
                for i, (ps, r) in enumerate(zip(self.buckets, self.ranges))]
