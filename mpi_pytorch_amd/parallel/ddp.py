"""Bucketed gradient all-reduce overlapped with backward (the DP engine's comm half).

Replaces the reference's per-parameter, blocking, post-backward loop
``mpi_avg_grads`` (``/root/reference/mpi_tools.py:30-37``, called at ``main.py:154``).

Design for MI355X / RCCL over xGMI:

* Buckets are cut from the flat fp32 gradient arena (:mod:`.arena`) at parameter
  boundaries, ``bucket_mb`` each (a parameter larger than a bucket gets its own).  The
  default 16 MiB keeps every bucket's launch close to its last gradient while 8-16 MiB
  messages still run near RCCL's large-message ring bandwidth on one xGMI link per ring
  hop (ResNet-18 @64,500: 126 + 9 + 9.5 + 16 + 8.3 MiB + 55 KB).  The final parameters
  (the stem) get a tiny bucket of their own (``_split_tail``): it is the only collective
  that can start only when backward ends.  Since
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
* Comm-aware persistent grids (``comm_ctas``, ``MPA_COMM_CTAS``, opt-in, e.g. 8; 0 = off): the
  buckets that overlap backward run on a second RCCL communicator capped at ``comm_ctas``
  CTAs (``ncclConfig_t.maxCTAs``), and while one is in flight the persistent conv kernels size
  their grids to the CUs the collective leaves free (``_ext.set_comm_reserve``).  Without
  it an RCCL CTA sits on a CU that a persistent conv block (146-150 KB of LDS) cannot
  share, and that block's static tile share starts only when another block finishes
  (``bench.py --emulate-comm``, docs/KERNELS.md §2c).  The 126 MiB head bucket needs only
  ~35 GB/s of bus bandwidth to hide under a ~7 ms backward, so a few CTAs suffice; the
  last bucket, which nothing overlaps, keeps the default (uncapped) communicator.
"""
from __future__ import annotations

import os
import time
from typing import List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .arena import ParamArena


def _set_reserve(cus: int) -> None:
    from ..ops import _ext
    _ext.ext().set_comm_reserve(int(cus))


# CTA cap of the overlapped buckets' communicator when neither the caller nor MPA_COMM_CTAS
# says otherwise.  profiles/comm_reserve_emulated_r2.txt (1 GPU, emulated collective):
# 8 or 32 CTAs held for 2 / 6 ms of backward cost +0.70 / +1.84 ms per step with static
# persistent grids, +0.38 / +0.61 ms with the reservation - the straggle depends on how
# long ANY CU is held, not on how many, so few CTAs plus a reservation is the cheap shape.
# Opt-in (MPA_COMM_CTAS=8) until a real multi-GPU run has measured it: the second
# communicator and the reservation have only met an emulated collective, and the default
# single-communicator path is RCCL's standard one (round-3 advisor finding).
DEFAULT_COMM_CTAS = 0


def capped_group(max_ctas: int, device: torch.device):
    """A second RCCL communicator over all ranks whose collectives use at most ``max_ctas``
    CTAs (None on non-RCCL backends, or if RCCL rejects the config - checked with one tiny
    all-reduce, so a failure shows here and not inside backward).  Collective call: every
    rank must make it."""
    if device.type != "cuda" or dist.get_backend() != "nccl":
        return None
    g, err = None, None
    try:
        opts = dist.ProcessGroupNCCL.Options()
        opts.config.max_ctas = int(max_ctas)
        g = dist.new_group(ranks=list(range(dist.get_world_size())), backend="nccl",
                           pg_options=opts)
        probe = torch.ones(64, device=device)
        dist.all_reduce(probe, group=g)
        torch.cuda.synchronize(device)
        if float(probe[0]) != float(dist.get_world_size()):
            raise RuntimeError("capped communicator returned %s" % float(probe[0]))
    except Exception as ex:
        err = ex
    # every rank must agree: a rank sending its overlapped buckets to the default group
    # while the others use the capped one would never match its collectives
    ok = torch.tensor([0 if err is not None else 1], dtype=torch.int32, device=device)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()) == 1:
        return g
    import sys
    print("GradBucketer: no CTA-capped communicator (%s); overlapped buckets use the "
          "default one" % (err or "failed on another rank"), file=sys.stderr)
    if g is not None:
        try:
            dist.destroy_process_group(g)
        except Exception:
            pass
    return None


def _wgrad_streams():
    from ..ops.functional import wgrad_streams
    return wgrad_streams()


class GradBucketer:
    def __init__(self, arena: ParamArena, world_size: int, bucket_mb: float = 16.0,
                 overlap: bool = True, comm_dtype: str = "fp32", group=None,
                 comm_ctas: Optional[int] = None, tail_elems: int = 32768):
        self.arena = arena
        self.world_size = world_size
        self.overlap = overlap
        self.comm_dtype = comm_dtype
        self.group = group
        if comm_ctas is None:
            comm_ctas = int(os.environ.get("MPA_COMM_CTAS", DEFAULT_COMM_CTAS))
        self.comm_ctas = max(int(comm_ctas), 0)
        self.overlap_group = None
        self._reserved = False
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
        self._split_tail(tail_elems)
        self.bucket_of = {}
        for bi, ps in enumerate(self.buckets):
            for p in ps:
                self.bucket_of[id(p)] = bi
        self._pending = [0] * len(self.buckets)
        self._launch_stream = None  # (side-stream weight gradients under DP: _launch)
        self._works: List[Optional[object]] = [None] * len(self.buckets)
        self._wire: List[Optional[torch.Tensor]] = [None] * len(self.buckets)
        # [bucket, wire bytes, work (None once resolved), host t0, host t1 | resolved ms,
        #  step number]
        self._stats: Optional[list] = None
        self._held = 0
        self._steps_done = 0
        self.active = world_size > 1
        # RCCL reports each collective's own device time; other backends are host-timed
        self._host_timed = self.active and dist.is_initialized() and \
            dist.get_backend(self.group) != "nccl"
        if self.active:
            arena.add_listener(self._on_grad)
            # (the capped communicator spans the whole world: only for the default group)
            if (self.comm_ctas > 0 and self.overlap and len(self.buckets) > 1
                    and self.group is None):
                self.overlap_group = capped_group(self.comm_ctas, arena.device)
        self.reset()

    def set_comm_ctas(self, comm_ctas: int) -> bool:
        """Switch the overlapped buckets to a CTA-capped communicator (``comm_ctas`` > 0, with
        the persistent-grid reservation) or back to the default one (0).  Collective: every
        rank must call it between steps.  Returns whether a capped communicator is in use
        (False on host backends or if RCCL rejected the config)."""
        if not self.active:
            return False
        self.comm_ctas = max(int(comm_ctas), 0)
        old, self.overlap_group = self.overlap_group, None
        if old is not None:
            try:
                dist.destroy_process_group(old)
            except Exception:
                pass
        if self.comm_ctas > 0 and self.overlap and len(self.buckets) > 1 and self.group is None:
            self.overlap_group = capped_group(self.comm_ctas, self.arena.device)
        return self.overlap_group is not None

    def _split_tail(self, tail_elems: int) -> None:
        """Give the last parameters of the arena (the first layers, whose gradients land
        last - for a ResNet the stem conv + BN, after a ~0.7 ms pool / BN / wgrad backward)
        a tiny bucket of their own (<= ``tail_elems`` elements), so the bulk of the old last
        bucket (layer2..layer1, 8.4 MiB for ResNet-18) launches before that stem backward
        and only a sub-128 KB collective is left exposed after backward."""
        if tail_elems <= 0 or not self.buckets or len(self.buckets[-1]) < 2:
            return
        ps = self.buckets[-1]
        k, n = len(ps), 0
        while k > 1:
            o, e = self.arena.slice_of(ps[k - 1])
            if n + (e - o) > tail_elems:
                break
            n += e - o
            k -= 1
        if k == len(ps):
            return
        s, e = self.ranges[-1]
        mid = self.arena.offsets[id(ps[k])]
        self.buckets[-1:] = [ps[:k], ps[k:]]
        self.ranges[-1:] = [(s, mid), (mid, e)]

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
        group = self.group
        if self.overlap_group is not None and bi != len(self.buckets) - 1:
            # an overlapped bucket: capped communicator, persistent grids give way
            group = self.overlap_group
            if not self._reserved:
                _set_reserve(self.comm_ctas)
                self._reserved = True
        streams = _wgrad_streams() if g.is_cuda else None
        if streams is not None:
            # side-stream weight gradients (TrainStep.wgrad_stream_ddp): this bucket's
            # gradients come from both the compute and the side stream, so the collective
            # is issued from a helper stream that waits for both (neither stream blocks)
            if self._launch_stream is None:
                self._launch_stream = torch.cuda.Stream(g.device)
            h = self._launch_stream
            h.wait_stream(streams[0])
            h.wait_stream(streams[1])
            with torch.cuda.stream(h):
                self._works[bi] = self._issue(bi, g, group)
        else:
            self._works[bi] = self._issue(bi, g, group)
        if self._stats is not None and len(self._stats) < self._MAX_STATS:
            # bytes actually sent: the bf16 wire copy is made inside _issue(), g is the
            # fp32 arena slice
            self._stats.append([bi, g.numel() * self.wire_elem_bytes, self._works[bi],
                                time.perf_counter(), None, self._steps_done])
            self._held += 1
            if self._held > self._MAX_HELD:
                self._resolve_old()

    def _issue(self, bi: int, g: torch.Tensor, group):
        if self.comm_dtype == "bf16" and g.is_cuda:
            g = g.to(torch.bfloat16)
            self._wire[bi] = g
        return dist.all_reduce(g, op=dist.ReduceOp.SUM, group=group, async_op=True)

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
                if self._stats is not None and self._host_timed:
                    # host backends (gloo): wait() returned when the collective did
                    for rec in self._stats[::-1]:
                        if rec[2] is w:
                            rec[4] = time.perf_counter()
                            break
            if self._wire[bi] is not None:
                s, e = self.ranges[bi]
                self.arena.grad[s:e].copy_(self._wire[bi])
                if self._launch_stream is not None:
                    self._wire[bi].record_stream(torch.cuda.current_stream())
                self._wire[bi] = None
        if self._reserved:
            # kernels enqueued from here on (optimizer, next forward) run after the waits
            _set_reserve(0)
            self._reserved = False
        self._steps_done += 1  # every record of this step has been waited on
        self.reset()

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world_size

    @property
    def wire_elem_bytes(self) -> int:
        return 2 if (self.comm_dtype == "bf16" and self.arena.grad.is_cuda) else 4

    def describe(self) -> List[dict]:
        """Bucket layout; ``bytes`` is what each all-reduce actually sends (wire dtype)."""
        return [{"bucket": i, "params": len(ps), "numel": r[1] - r[0],
                 "bytes": (r[1] - r[0]) * self.wire_elem_bytes}
                for i, (ps, r) in enumerate(zip(self.buckets, self.ranges))]

    def wire_mb(self) -> float:
        return round(sum(b["bytes"] for b in self.describe()) / 2**20, 2)

    # ------------------------------------------------------------------ comm statistics
    _MAX_STATS = 8192
    _MAX_HELD = 64  # Work objects kept alive for their durations (see _resolve_old)

    def _resolve_old(self) -> None:
        """Turn the older half of the held Work records into durations and drop the Work
        objects: a Work keeps its collective's output alive, and with the bf16 wire format
        that is a fresh bucket-sized tensor per launch - holding every step's Works until
        comm_stats() grew device memory by half the gradient size per step.  The records
        resolved here are steps old, so reading their duration does not stall the step."""
        # only records of steps whose collectives finish() has already waited on: their
        # device events are complete (RCCL) and their host end stamps set (gloo)
        held = [r for r in self._stats if r[2] is not None and r[5] < self._steps_done]
        for rec in held[: max(len(held) // 2, 1)]:
            rec[4] = self._duration_ms(rec)
            rec[2] = None
        self._held = sum(1 for r in self._stats if r[2] is not None)

    def _duration_ms(self, rec) -> Optional[float]:
        bi, nbytes, work, t0, t1 = rec[:5]
        if t1 is not None and work is None:
            return t1
        if self._host_timed:
            return (t1 - t0) * 1e3 if t1 is not None else None
        try:
            return float(work._get_duration())
        except Exception:
            return None

    def enable_comm_stats(self) -> None:
        """Record every bucket all-reduce of the following steps for :meth:`comm_stats`.

        RCCL: the collective's own duration on its stream, from the start/end events
        ProcessGroupNCCL records when ``TORCH_NCCL_ENABLE_TIMING=1`` was set before the
        process group came up (``Work._get_duration``).  Host backends (gloo): launch to
        completion of ``wait()``.  Nothing is synchronised until :meth:`comm_stats`."""
        if self.active:
            self._stats = []
            self._held = 0

    def comm_stats(self, reset: bool = True) -> Optional[dict]:
        """Per-bucket mean all-reduce time, algorithm and bus bandwidth (ring all-reduce:
        busbw = algbw * 2(n-1)/n, the per-link rate nccl-tests reports), plus the totals
        per step.  Call after the device has been synchronised."""
        if self._stats is None:
            return None
        n = self.world_size
        per = {}
        for rec in self._stats:
            bi, nbytes = rec[0], rec[1]
            ms = rec[4] if rec[2] is None else self._duration_ms(rec)
            d = per.setdefault(bi, {"bucket": bi, "bytes": nbytes, "ms": [], "n": 0})
            d["n"] += 1
            if ms is not None and ms > 0:
                d["ms"].append(ms)
        out = []
        tot_ms, tot_bytes, steps = 0.0, 0, 0
        for bi in sorted(per):
            d = per[bi]
            rec = {"bucket": bi, "mb": round(d["bytes"] / 2**20, 3), "calls": d["n"]}
            if d["ms"]:
                ms = sum(d["ms"]) / len(d["ms"])
                algbw = d["bytes"] / (ms * 1e-3) / 1e9
                rec.update(ms=round(ms, 4), algbw_gbs=round(algbw, 2),
                           busbw_gbs=round(algbw * 2.0 * (n - 1) / n, 2))
                tot_ms += ms
            tot_bytes += d["bytes"]
            steps = max(steps, d["n"])
            out.append(rec)
        if reset:
            self._stats = []
            self._held = 0
        res = {"world": n, "steps": steps, "buckets": out,
               "mb_per_step": round(tot_bytes / 2**20, 2),
               "timed": any("ms" in r for r in out)}
        if res["timed"]:
            res["sum_ms_per_step"] = round(tot_ms, 4)
            res["busbw_gbs"] = round(tot_bytes / (tot_ms * 1e-3) / 1e9 * 2.0 * (n - 1) / n, 2)
        return res
