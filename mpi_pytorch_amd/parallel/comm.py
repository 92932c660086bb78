"""``mpi_tools``-compatible communication helpers on torch.distributed (RCCL / gloo).

API parity with ``/root/reference/mpi_tools.py``:

=====================  =============================  ====================================
reference              here                           notes
=====================  =============================  ====================================
``num_processes``      :func:`num_processes`          ``mpi_tools.py:5-9``
``mpi_all_reduce``     :func:`mpi_all_reduce`         ``mpi_tools.py:12-16`` (in-place SUM)
``mpi_sum``            :func:`mpi_sum`                ``mpi_tools.py:19-27`` scalar or array
``mpi_avg_grads``      :func:`mpi_avg_grads`          ``mpi_tools.py:30-37``; flat-arena
                                                      buckets instead of 1 call / tensor
``mpi_broadcast``      :func:`mpi_broadcast`          ``mpi_tools.py:40-44``
``sync_params``        :func:`sync_params`            ``mpi_tools.py:47-53``; ONE broadcast
                                                      of the flat master arena
=====================  =============================  ====================================

Also the object-level collectives the drivers need (``comm.scatter`` at ``main.py:91``,
``comm.reduce`` at ``evaluation_pipeline.py:196``): :func:`scatter_object`,
:func:`reduce_scalar`.
"""
from __future__ import annotations

from typing import Any, List, Optional

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn

from .dist import get_world


def num_processes() -> int:
    return get_world().world_size


def _comm_tensor(x: torch.Tensor) -> torch.Tensor:
    w = get_world()
    if w.backend == "nccl" and not x.is_cuda:
        return x.to(w.device)
    return x


def mpi_all_reduce(x: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
    """In-place all-reduce of a tensor (reference wraps ``COMM_WORLD.Allreduce``)."""
    if num_processes() == 1:
        return x
    t = _comm_tensor(x)
    dist.all_reduce(t, op=op)
    if t is not x:
        x.copy_(t)
    return x


def mpi_sum(x: Any, op=dist.ReduceOp.SUM):
    """Sum a scalar or array over ranks; returns the same kind (float32 like the ref)."""
    scalar = np.isscalar(x)
    t = torch.as_tensor(np.asarray([x] if scalar else x, dtype=np.float32)).clone()
    mpi_all_reduce(t, op=op)
    out = t.cpu().numpy()
    return out[0] if scalar else out


def mpi_avg_grads(model: nn.Module) -> None:
    """Average ``p.grad`` over ranks.  Uses the model's arena buckets when present."""
    n = num_processes()
    if n == 1:
        return None
    bucketer = getattr(model, "_mpa_bucketer", None)
    if bucketer is not None:
        bucketer.finish()
        bucketer.arena.grad.mul_(1.0 / n)
        return None
    for p in model.parameters():
        if p.grad is None:
            continue
        mpi_all_reduce(p.grad)
        p.grad.mul_(1.0 / n)
    return None


def mpi_broadcast(x: torch.Tensor, root: int = 0) -> None:
    if num_processes() == 1:
        return
    t = _comm_tensor(x)
    dist.broadcast(t, src=root)
    if t is not x:
        x.copy_(t)


def sync_params(model: nn.Module, root: int = 0, buffers: bool = False) -> None:
    """Make every replica identical to ``root`` (``mpi_tools.py:47-53``).

    With a flat arena this is a single broadcast of the fp32 master buffer (plus a bf16
    shadow refresh) instead of one ``Bcast`` per parameter.  ``buffers=True`` additionally
    broadcasts BN running statistics, which the reference never syncs.
    """
    if num_processes() == 1:
        return None
    arena = getattr(model, "_mpa_arena", None)
    if arena is not None:
        mpi_broadcast(arena.master, root)
        arena.sync_shadow()
    else:
        for p in model.parameters():
            mpi_broadcast(p.data, root)
    if buffers:
        for b in model.buffers():
            if b.dtype.is_floating_point:
                mpi_broadcast(b, root)
    return None


def scatter_object(objs: Optional[List[Any]], root: int = 0) -> Any:
    """Pickled scatter (``comm.scatter`` at ``main.py:91``)."""
    w = get_world()
    if w.world_size == 1:
        return objs[0]
    out: List[Any] = [None]
    dist.scatter_object_list(out, objs if w.rank == root else None, src=root)
    return out[0]


def broadcast_object(obj: Any, root: int = 0) -> Any:
    w = get_world()
    if w.world_size == 1:
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=root)
    return lst[0]


def reduce_scalar(x: float, root: int = 0) -> Optional[float]:
    """SUM-reduce a Python float to ``root`` (``comm.reduce`` at evaluation_pipeline.py:196)."""
    w = get_world()
    if w.world_size == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64)
    t = _comm_tensor(t)
    dist.reduce(t, dst=root, op=dist.ReduceOp.SUM)
    return float(t.item()) if w.rank == root else None


def all_gather_object(obj: Any) -> List[Any]:
    w = get_world()
    if w.world_size == 1:
        return [obj]
    out: List[Any] = [None] * w.world_size
    dist.all_gather_object(out, obj)
    return out


def replica_checksum(model: nn.Module) -> bool:
    """Cross-rank replica-divergence check: all ranks compare a checksum
    of the flat master arena.  Returns True when every replica matches rank 0."""
    w = get_world()
    if w.world_size == 1:
        return True
    arena = getattr(model, "_mpa_arena", None)
    src = arena.master if arena is not None else torch.cat(
        [p.detach().reshape(-1).float() for p in model.parameters()])
    idx = torch.arange(src.numel(), device=src.device, dtype=torch.float64) % 9973 + 1
    v = torch.stack([src.double().sum(), (src.double() * idx).sum()])
    mn = _comm_tensor(v.clone())
    mx = _comm_tensor(v.clone())
    dist.all_reduce(mn, op=dist.ReduceOp.MIN)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    return bool(torch.equal(mn.cpu(), mx.cpu()))


def agree_tuned_tiles(get=None, load=None, root: int = 0) -> Optional[str]:
    """Make every rank run the same GEMM tiles: the native autotuner times candidates on
    each process's first launch of a shape and caches its own winner, so data-parallel
    ranks could pick different tiles and step at different speeds (the job runs at the
    slowest).  After a step that tuned new shapes, rank ``root`` broadcasts its table and
    every rank adopts it (``_C.igemm_tuned_load``).  ``get`` / ``load`` override the native
    table (tests).  Collective: every rank must call it at the same step.  Returns the
    agreed table (None on one rank or without the native extension).  The reference's
    ranks run identical code (``mpi_tools.py:30-37``); this keeps that property for a
    timing-based kernel choice."""
    w = get_world()
    if w.world_size == 1:
        return None
    if get is None or load is None:
        from ..ops import _ext
        k = _ext.ext() if w.device.type == "cuda" else None
        if k is None or not hasattr(k, "igemm_tuned_load"):
            return None
        get = get or k.igemm_tuned_table
        load = load or (lambda t: k.igemm_tuned_load(t, True))
    table = broadcast_object(get() if w.rank == root else None, root)
    load(table)
    return table
