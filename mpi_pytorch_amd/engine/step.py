"""The data-parallel training step (the engine's hot loop), shared by ``main.py``,
``bench.py`` and ``__graft_entry__.smoke``.

Reference hot loop (``/root/reference/main.py:142-156``): forward -> CE loss ->
zero_grad -> backward -> per-tensor blocking Allreduce average -> Adam.step ->
``loss.item()`` (a host sync every step).

Here:
  zero the flat gradient arena (one memset) -> forward on fused NHWC/bf16 MFMA ops ->
  fused CE -> backward, during which each gradient bucket's RCCL all-reduce starts as
  soon as its last gradient lands (overlap) -> wait for outstanding buckets -> ONE fused
  optimizer kernel (1/N average folded in, bf16 weights written) -> loss accumulated on
  the device (no per-step host sync).

With ``graph=True`` the whole step (forward, backward, optimizer) is captured once into a
HIP graph and replayed, removing per-kernel launch overhead (single-process only: the
RCCL collectives of the multi-GPU path run eagerly and overlap with backward).
"""
from __future__ import annotations

import contextlib
import gc
import os
from typing import Optional

import torch
import torch.nn as nn

from ..models import initialize_model, InceptionOutputs
from ..ops import functional as Fn
from ..optim import build_optimizer
from ..parallel import ParamArena, GradBucketer, sync_params, World, agree_tuned_tiles


def build_model(name: str, num_classes: int, feature_extract: bool, device: torch.device,
                world: World, use_pretrained: bool = False, bucket_mb: float = 16.0,
                overlap: bool = True, comm_dtype: str = "fp32", comm_ctas: Optional[int] = None):
    model, input_size = initialize_model(name, num_classes, feature_extract, use_pretrained)
    model = model.to(device)
    arena = ParamArena(model, device)
    model._mpa_arena = arena
    model._mpa_bucketer = GradBucketer(arena, world.world_size, bucket_mb, overlap, comm_dtype,
                                       comm_ctas=comm_ctas)
    return model, input_size


def loss_fn(out, labels, acc=None):
    """CE; Inception's train-mode (logits, aux) uses loss + 0.4 * aux_loss (the documented
    fix of the reference's broken Inception path), one fused native op.
    ``acc``: device scalar the loss is also added to (the trainer's running sum)."""
    if isinstance(out, (tuple, InceptionOutputs)):
        logits, aux = out[0], out[1]
        heads = [(aux, 0.4)] if aux is not None else None
        return Fn.cross_entropy(logits, labels, acc=acc, heads=heads)
    return Fn.cross_entropy(out, labels, acc=acc)


# MPA_WGRAD_STREAM_DDP=1: side-stream weight gradients with several ranks too (the bucket
# collectives then wait for both streams, GradBucketer._launch).  Off by default until the
# 8-GPU run measures it (bench.py records both in its multi_gpu decisions)
_WGRAD_DDP = os.environ.get("MPA_WGRAD_STREAM_DDP", "0") == "1"
# MPA_STEP_GC=1 leaves Python's cyclic collector running inside the training loop
_STEP_GC = os.environ.get("MPA_STEP_GC", "0") == "1"


@contextlib.contextmanager
def steps_without_gc():
    """Run a loop of training steps with Python's *cyclic* garbage collector paused, and
    collect once on entry and once on exit (epoch boundaries).

    A step's autograd graph, activations and workspaces are freed by reference counting as
    usual; only the collector's periodic generation scans are deferred.  Mid-backward a
    full scan over the step's ~10^5 tracked objects (DenseNet's 58 per-layer graphs)
    stalled the launch stream for 0.3-0.4 ms twice per step, with the GPU idle
    (profiles/densenet_b256_step_breakdown_r3.txt).  The few reference cycles autograd
    leaves are reclaimed at the boundary."""
    if _STEP_GC:
        yield
        return
    was = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()
        gc.collect()


class _NoMarkers:
    """roctx stand-in on hosts without the native extension (CPU runs)."""

    def range_push(self, name: str) -> int:
        return 0

    def range_pop(self) -> int:
        return 0

    def mark(self, name: str) -> None:
        pass


def markers():
    """The roctx API of the native extension (``range_push`` / ``range_pop`` / ``mark``,
    csrc/runtime/runtime.cpp) - or a no-op stand-in when it is not built (CPU)."""
    from ..ops import _ext
    if torch.cuda.is_available() and _ext.available():
        return _ext.ext()
    return _NoMarkers()


class StepTimer:
    """Per-step phase times from HIP events on the compute stream:

    * ``data``      - previous step's end to this step's start: the batch hand-off, H2D
                      copy and preprocess kernel the loader enqueued in between;
    * ``forward``   - gradient-arena zero, forward and loss;
    * ``backward``  - backward, with the overlapped bucket all-reduces launched inside it;
    * ``comm_wait`` - the exposed part of the gradient all-reduce (``GradBucketer.finish``);
    * ``optimizer`` - the fused optimizer kernel (+ transposed-weight refresh).

    Events are resolved lazily (``summary``), so timing adds no host sync to the step.
    The reference has only the per-epoch ``MPI.Wtime()`` (``/root/reference/main.py:145,158``).
    """

    PHASES = ("data", "forward", "backward", "comm_wait", "optimizer")
    _MAX_PENDING = 64

    def __init__(self, event_factory=None):
        # HIP timing events; a stand-in factory lets the bookkeeping be tested on the CPU
        self._event = event_factory or (lambda: torch.cuda.Event(enable_timing=True))
        self._pending = []
        self._cur = None
        self.reset()

    def reset(self) -> None:
        self.totals = {k: 0.0 for k in self.PHASES}
        self.steps = 0
        self.data_steps = 0
        self._last_end = None  # e.g. an epoch's checkpoint / validation is no data time

    def mark(self, i: int) -> None:
        ev = self._event()
        ev.record()
        if i == 0:
            self._cur = [self._last_end, ev]
        else:
            self._cur.append(ev)
            if i == 4:
                self._last_end = ev
                self._pending.append(self._cur)
                self._cur = None
                if len(self._pending) > self._MAX_PENDING:
                    self._resolve(self._pending[: self._MAX_PENDING // 2])
                    del self._pending[: self._MAX_PENDING // 2]

    def _resolve(self, recs) -> None:
        for rec in recs:
            rec[-1].synchronize()
            prev, evs = rec[0], rec[1:]
            if prev is not None:
                self.totals["data"] += prev.elapsed_time(evs[0])
                self.data_steps += 1
            for k, a, b in zip(self.PHASES[1:], evs[:-1], evs[1:]):
                self.totals[k] += a.elapsed_time(b)
            self.steps += 1

    def summary(self, reset: bool = True) -> dict:
        """Mean milliseconds per step of each phase (plus ``step``) since the last reset."""
        self._resolve(self._pending)
        self._pending = []
        n = max(self.steps, 1)
        out = {k: round(v / n, 4) for k, v in self.totals.items()}
        out["data"] = round(self.totals["data"] / max(self.data_steps, 1), 4)
        out["step"] = round(sum(out[k] for k in self.PHASES), 4)
        out["steps"] = self.steps
        if reset:
            self.reset()
        return out


class TrainStep:
    def __init__(self, model: nn.Module, optimizer, world: World):
        self.model = model
        self.opt = optimizer
        self.world = world
        self.arena: ParamArena = model._mpa_arena
        self.bucketer: GradBucketer = model._mpa_bucketer
        self.opt.grad_scale = 1.0 / world.world_size
        dev = self.arena.device
        # running loss sum, added to by the loss kernel itself (graph-safe: fixed address,
        # reset in place) - one host sync per epoch; the backward seed is a constant
        self.loss_sum = torch.zeros(4, dtype=torch.float32, device=dev)
        self._one = torch.ones((), dtype=torch.float32, device=dev)
        self.steps = 0
        self._graph = None
        self._static_x = None
        self._static_y = None
        self._static_loss = None
        # Back-to-back replays need no host sync: in deterministic mode 100 replays equal
        # 100 eager steps bitwise (tests/test_determinism_gpu.py, tools/graph_bisect.py;
        # docs/NOTES.md "HIP graph replay").
        self.timer: Optional[StepTimer] = None
        # roctx ranges fwd / bwd / comm_wait / opt around the host enqueue of each phase
        # (rocprofv3 --marker-trace shows them beside the kernels); MPA_ROCTX=1
        self.markers = markers() if os.environ.get("MPA_ROCTX", "0") == "1" else None
        self.wgrad_stream_ddp = _WGRAD_DDP
        self._agreed = set()  # batch shapes whose tuned tiles the ranks have agreed on
        # (an early classifier update on a side stream under the rest of the backward was
        # measured slower on one MI355X - ResNet-18 b1024 48.0k vs 48.2k, Inception 6.99k vs
        # 7.09k img/s, profiles/early_head_ab_r3.txt - and removed in round 5)

    def enable_timers(self) -> StepTimer:
        """Turn on per-phase HIP-event timing of eager steps (GPU only)."""
        if self.timer is None and self.arena.device.type == "cuda":
            self.timer = StepTimer()
        return self.timer

    def _eager(self, x, y):
        t = self.timer if self._graph is None else None
        m = self.markers
        if t is not None:
            t.mark(0)
        if m is not None:
            m.range_push("fwd")
        self.arena.zero_grad()
        # (single GPU: an Inception block's longest branch chain may run on a second
        # stream, forward and backward; joined after the backward)
        single = self.bucketer is None or not self.bucketer.active
        Fn.branch_streams(single)
        try:
            out = self.model(x)
            loss = loss_fn(out, y, acc=self.loss_sum)
        except BaseException:
            Fn.branch_streams(False)
            raise
        if t is not None:
            t.mark(1)
        if m is not None:
            m.range_pop()
            m.range_push("bwd")
        # (single GPU: conv weight gradients may run on a side stream, joined right after)
        Fn.wgrad_stream_begin(single or self.wgrad_stream_ddp)
        try:
            loss.backward(self._one)
        finally:
            Fn.join_wgrad_stream()
            if Fn._BR["on"]:
                Fn.branch_streams(False)
                Fn.join_branch_stream()
        if t is not None:
            t.mark(2)
        if m is not None:
            m.range_pop()
            m.range_push("comm_wait")
        self.bucketer.finish()
        if t is not None:
            t.mark(3)
        if m is not None:
            m.range_pop()
            m.range_push("opt")
        self.opt.step()
        if t is not None:
            t.mark(4)
        if m is not None:
            m.range_pop()
        return loss.detach()

    def __call__(self, x, y) -> torch.Tensor:
        if self._graph is not None and x.shape == self._static_x.shape:
            self._static_x.copy_(x)
            self._static_y.copy_(y)
            self._graph.replay()
            loss = self._static_loss
        else:  # eager (also a short last batch of a graph-captured loop)
            loss = self._eager(x, y)
            if self.world.world_size > 1 and tuple(x.shape) not in self._agreed:
                # the first step of a batch shape tuned its GEMM tiles per rank: adopt
                # rank 0's choices everywhere (every rank reaches this at the same step)
                self._agreed.add(tuple(x.shape))
                agree_tuned_tiles()
        self._accumulate(loss)
        return loss

    def _accumulate(self, loss):
        self.steps += 1  # (the loss kernel already added the loss to self.loss_sum)

    def mean_loss(self, reset: bool = True) -> float:
        v = float(self.loss_sum[0].item()) / max(self.steps, 1) if self.steps else 0.0
        if reset:
            Fn.K(self.loss_sum).zero_f32(self.loss_sum)
            self.steps = 0
        return v

    # --------------------------------------------------------------------- HIP graphs
    def _training_state(self):
        """Everything a training step mutates besides the (per-step zeroed) gradients:
        master / bf16 / transposed weights, optimizer moments and step counter, BN running
        statistics and batch counts, the running loss sum, the dropout stream position."""
        a = self.arena
        dev = [t for t in (a.master, a.shadow, a.shadow_t, self.loss_sum) if t is not None]
        dev += [v for v in vars(self.opt).values() if torch.is_tensor(v)]
        dev += list(self.model.buffers())
        bns = [m for m in self.model.modules() if hasattr(m, "_batches_host")]
        return dev, bns

    def snapshot(self):
        """Device copies of the training state (see :meth:`restore`)."""
        dev, bns = self._training_state()
        return ([t.clone() for t in dev], [m._batches_host for m in bns], Fn.DropoutRNG.state(),
                self.steps)

    def restore(self, snap) -> None:
        dev, bns = self._training_state()
        with torch.no_grad():
            for t, c in zip(dev, snap[0]):
                t.copy_(c)
        for m, n in zip(bns, snap[1]):
            m._batches_host = n
        Fn.DropoutRNG.set_state(snap[2])
        self.steps = snap[3]

    def capture(self, x, y, warmup: int = 2) -> bool:
        """Capture one full step into a HIP graph (world size 1 only).

        The warm-up steps that capture needs run on a snapshot of the training state and
        are rolled back afterwards, so capturing does not train on ``x`` (the caller's
        following ``step(x, y)`` - the first replay - is that batch's only update) and
        adds nothing to the running loss."""
        if self.world.world_size != 1 or not x.is_cuda:
            return False
        self._static_x = x.clone()
        self._static_y = y.clone()
        self.timer = None  # replayed steps are not phase-timed
        snap = self.snapshot()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._eager(self._static_x, self._static_y)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._static_loss = self._eager(self._static_x, self._static_y)
        self._graph = g
        self.restore(snap)
        return True


def reserve_device_memory(device, gib: float) -> float:
    """Grow PyTorch's caching allocator by ONE segment of ``gib`` GiB (capped at 90 % of the
    free device memory) up front, so a training run's tensors are carved from it instead of
    hipMalloc'ing new segments during the first steps.

    Why: the caching allocator keeps growing for several steps (tensors used on the side
    stream are record_stream'ed and come back late), and a hipMalloc right after another
    process released tens of GB can stall the host for milliseconds while the driver still
    reclaims that memory - a process then runs 1.6-5x slower for its whole life (batch 2048
    ResNet-18, SqueezeNet b512; docs/NOTES.md "Slow processes").  Returns the GiB reserved."""
    if gib <= 0 or device.type != "cuda":
        return 0.0
    free, _ = torch.cuda.mem_get_info(device)
    n = int(min(gib * 2**30, 0.9 * free))
    while n >= 2**30:  # (ranks sharing a GPU race for it: halve on failure)
        try:
            t = torch.empty(n, dtype=torch.uint8, device=device)
        except torch.cuda.OutOfMemoryError:
            n //= 2
            continue
        del t  # (the allocator keeps the segment cached)
        return round(n / 2**30, 1)
    return 0.0


def build_training(name: str, num_classes: int, device, world: World, lr: float,
                   optimizer: str = "adam", momentum: float = 0.9, weight_decay: float = 0.0,
                   feature_extract: bool = False, bucket_mb: float = 16.0, overlap: bool = True,
                   comm_dtype: str = "fp32", comm_ctas: Optional[int] = None):
    model, input_size = build_model(name, num_classes, feature_extract, device, world,
                                    bucket_mb=bucket_mb, overlap=overlap, comm_dtype=comm_dtype,
                                    comm_ctas=comm_ctas)
    opt = build_optimizer(optimizer, model, lr, momentum, weight_decay)
    sync_params(model)
    model.train()
    return model, opt, TrainStep(model, opt, world), input_size
