"""Flat parameter / gradient arena.

Every parameter of a model is re-homed into ONE contiguous fp32 master buffer, and every
trainable parameter's ``.grad`` becomes a view into ONE contiguous fp32 gradient buffer.
On the GPU a bf16 shadow of the master buffer holds the weights the MFMA kernels read.

Why (MI355X-first, not a translation of ``mpi_tools.py``):

* The reference all-reduces one tensor at a time (62 blocking calls/step for ResNet-18,
  ``/root/reference/mpi_tools.py:30-37``) and broadcasts one tensor at a time
  (``mpi_tools.py:47-53``).  With a flat arena the broadcast is one RCCL call and the
  gradient all-reduce is a handful of large buckets cut from one buffer, which is what a
  per-link-bound xGMI ring wants.
* The optimizer (Adam/SGD) becomes ONE streaming HIP kernel over the flat buffers that
  also writes the bf16 shadow - no per-tensor launches, no separate cast pass.
* Layout: trainable parameters come first, in *reverse registration order*, so the
  gradients produced first by backward (the classifier head) sit at the front of the
  gradient buffer and close the first bucket while the conv stack still back-propagates.
  Frozen parameters (``feature_extract``, ``models.py:5-13`` of the reference) sit after
  the trainable region and get no gradient storage.

Backward kernels write weight gradients straight into ``p.grad`` (atomic fp32
accumulation into the zeroed arena), then call :meth:`ParamArena.notify` so the
bucketer can launch the bucket's all-reduce as soon as its last gradient lands.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

import torch
import torch.nn as nn

ALIGN = 64  # elements (256 B fp32) - keeps every slice 16-B aligned for dwordx4 access


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


def _group_params(trainable: List[nn.Parameter], groups) -> List[nn.Parameter]:
    """Reorder so each group's parameters sit back to back, in the group's order, at the
    position of its first member (model hint ``_mpa_param_groups``: e.g. the weights of
    1x1 convs that read the same input and run as ONE GEMM over their joint rows)."""
    pos = {id(p): i for i, p in enumerate(trainable)}
    taken, firsts = set(), {}
    for g in groups:
        ids = [id(p) for p in g]
        if len(g) < 2 or any(i not in pos or i in taken for i in ids) or len(set(ids)) < len(ids):
            continue
        firsts[min(pos[i] for i in ids)] = list(g)
        taken.update(ids)
    out: List[nn.Parameter] = []
    for i, p in enumerate(trainable):
        if i in firsts:
            out.extend(firsts[i])
        elif id(p) not in taken:
            out.append(p)
    return out


class ParamArena:
    def __init__(self, model: nn.Module, device: torch.device, shadow: Optional[bool] = None):
        self.device = torch.device(device)
        if shadow is None:
            shadow = self.device.type == "cuda"
        seen = set()
        params: List[nn.Parameter] = []
        names: Dict[int, str] = {}
        for n, p in model.named_parameters():
            if id(p) in seen:
                continue
            seen.add(id(p))
            params.append(p)
            names[id(p)] = n
        trainable = [p for p in params if p.requires_grad][::-1]
        groups = getattr(model, "_mpa_param_groups", None)
        if callable(groups):
            trainable = _group_params(trainable, groups())
        frozen = [p for p in params if not p.requires_grad]
        self.params: List[nn.Parameter] = trainable + frozen
        self.trainable: List[nn.Parameter] = trainable
        self.names = names
        self.offsets: Dict[int, int] = {}
        off = 0
        for p in self.params:
            self.offsets[id(p)] = off
            off += _align(p.numel())
        self.numel = off
        self.n_train = sum(_align(p.numel()) for p in trainable)
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(max(self.n_train, ALIGN), dtype=torch.float32, device=self.device)
        self.shadow = (torch.zeros(self.numel, dtype=torch.bfloat16, device=self.device)
                       if shadow else None)
        with torch.no_grad():
            for p in self.params:
                o = self.offsets[id(p)]
                view = self.master[o:o + p.numel()].view_as(p)
                view.copy_(p.data.to(self.device, torch.float32))
                p.data = view
                if self.shadow is not None:
                    p._mpa_shadow = self.shadow[o:o + p.numel()].view(p.shape)
                else:
                    p._mpa_shadow = None
                if p.requires_grad:
                    p.grad = self.grad[o:o + p.numel()].view_as(p)
                p._mpa_arena = self
        self._listeners: List[Callable[[nn.Parameter], None]] = []
        # parameters whose gradient slice still holds the zeros of the last zero_grad():
        # their first weight-gradient kernel stores instead of read-modify-writing
        self._fresh = {id(p) for p in trainable}
        self._init_transposed()
        self.sync_shadow()

    def _init_transposed(self) -> None:
        """Transposed bf16 weight shadow for dgrad: a conv weight stored KRSC is also kept
        as [C][R*S][K] (``p._mpa_shadow_t``), so the dgrad GEMM reads its B operand
        K-contiguous like the forward GEMM instead of through transposing LDS reads.  One
        batched transpose launch refreshes every such weight after the optimizer step."""
        self.shadow_t = None
        self._tseg = None
        self._ttiles = 0
        if self.shadow is None:
            return
        rows, off, tiles = [], 0, 0
        tp = [p for p in self.params if getattr(p, "_mpa_tlayout", None) is not None]
        for p in tp:
            K, RS, C = p._mpa_tlayout
            if K * RS * C != p.numel() or K % 8 or C % 8:
                continue
            rows.append((p, [self.offsets[id(p)], off, K, RS, C, tiles]))
            tiles += RS * ((K + 63) // 64) * ((C + 63) // 64)
            off += _align(p.numel())
        if not rows:
            return
        self.shadow_t = torch.zeros(off, dtype=torch.bfloat16, device=self.device)
        for p, r in rows:
            K, RS, C = p._mpa_tlayout
            p._mpa_shadow_t = self.shadow_t[r[1]:r[1] + p.numel()].view(C, RS, K)
        self._tseg = torch.tensor([r for _, r in rows], dtype=torch.int64, device=self.device)
        self._ttiles = tiles

    def refresh_transposed(self, step_inc: Optional[torch.Tensor] = None) -> None:
        """Re-derive the transposed shadow from the bf16 shadow (after each update);
        ``step_inc``: the optimizer's step counter, incremented by the same launch."""
        if self._tseg is not None:
            from ..ops import _ext
            _ext.ext().transpose_krsc(self.shadow, self.shadow_t, self._tseg, self._ttiles,
                                      step_inc)
        elif step_inc is not None:
            if step_inc.is_cuda:
                from ..ops import _ext
                _ext.ext().step_inc(step_inc)
            else:
                step_inc.add_(1.0)

    # ------------------------------------------------------------------------------
    def slice_of(self, p: nn.Parameter):
        o = self.offsets[id(p)]
        return o, o + p.numel()

    def flat_view(self, params: List[nn.Parameter], which: str) -> Optional[torch.Tensor]:
        """ONE flat view of ``params`` in the master / grad / shadow buffer when they sit
        back to back without alignment padding (see ``_mpa_param_groups``), else None."""
        o0 = o = self.offsets.get(id(params[0]), -1)
        if o0 < 0:
            return None
        for p in params:
            if self.offsets.get(id(p)) != o:
                return None
            o += p.numel()
        t = getattr(self, which)
        if t is None or o > t.numel():
            return None
        return t[o0:o]

    def sync_shadow(self) -> None:
        """Refresh the bf16 weight shadow from the fp32 masters (after init/load)."""
        if self.shadow is not None:
            with torch.no_grad():
                self.shadow.copy_(self.master)
            self.refresh_transposed()

    def zero_grad(self) -> None:
        if self.grad.is_cuda:
            from ..ops import _ext
            _ext.ext().zero_f32(self.grad)
        else:
            self.grad.zero_()
        self._fresh = {id(p) for p in self.trainable}

    def take_fresh(self, p: nn.Parameter) -> bool:
        """True (once per zero_grad) if ``p``'s gradient is still all zeros: the caller's
        kernel may overwrite it instead of accumulating (the 132 MB classifier gradient is
        then written, not read and written)."""
        i = id(p)
        if i in self._fresh:
            self._fresh.discard(i)
            return True
        return False

    def add_listener(self, fn: Callable[[nn.Parameter], None]) -> None:
        self._listeners.append(fn)

    def notify(self, p: nn.Parameter) -> None:
        # whatever wrote p's gradient, it is no longer all zeros: a later kernel for the
        # same parameter (tied weights, a second use) must accumulate, not overwrite
        self._fresh.discard(id(p))
        for fn in self._listeners:
            fn(p)

    def train_master(self) -> torch.Tensor:
        return self.master[:self.n_train]

    def train_shadow(self) -> Optional[torch.Tensor]:
        return None if self.shadow is None else self.shadow[:self.n_train]


def weight_of(p: nn.Parameter) -> torch.Tensor:
    """The tensor a compute kernel should read for parameter ``p`` (bf16 on GPU)."""
    s = getattr(p, "_mpa_shadow", None)
    return s if s is not None else p


def weight_t_of(p: nn.Parameter) -> Optional[torch.Tensor]:
    """The [C][R*S][K] transposed bf16 shadow of a conv/linear weight, or None."""
    return getattr(p, "_mpa_shadow_t", None)


def grad_sink(p: nn.Parameter) -> Optional[torch.Tensor]:
    """Where a backward kernel accumulates ``p``'s gradient (None when frozen)."""
    if not p.requires_grad:
        return None
    if p.grad is None:
        p.grad = torch.zeros_like(p, dtype=torch.float32)
    return p.grad


def grad_done(p: nn.Parameter) -> None:
    a = getattr(p, "_mpa_arena", None)
    if a is not None and p.requires_grad:
        a.notify(p)
