#!/usr/bin/env python
"""Headline benchmark: images/sec (whole node), ResNet-18 224x224 training, 1/2/4/8 MI355X.

    python bench.py --gpus N --steps K --warmup W
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Config (BASELINE.json): ResNet-18 with the reference's 64,500-class head (utils.py:39),
224x224 synthetic uint8 images (preprocessed on the GPU each step), random-init weights,
bf16 compute with fp32 master weights, Adam (lr 4e-4, the reference optimizer,
main.py:125), data-parallel over RCCL with per-GPU batch fixed (weak scaling).

Timing: W untimed warmup steps, then EXACTLY K steps bracketed by barrier +
torch.cuda.synchronize() on both sides; the max over ranks is reported.  The timed region
includes the data path (ring acquire, H2D, preprocess kernel), forward, backward, the
gradient all-reduce and the optimizer step.  Rank 0 prints one JSON line.

Failure handling (the reference aborts the whole job on any rank's error,
/root/reference/README.md:38; its blocking per-tensor Allreduce loop, mpi_tools.py:30-37,
hangs forever on a lost peer):
  * the process group has a bounded timeout (--pg-timeout) and the self-spawned job a wall
    clock limit (--job-timeout), both well inside a driver's 600 s command limit;
  * warm-up and timed steps run under the device-completion watchdog (--watchdog seconds,
    parallel/watchdog.py): a rank whose GPU stops completing steps dumps its stacks and exits
    75 with a rank-tagged message, and the launcher tears the job down;
  * the headline record is built AND PRINTED (flushed) right after the timed steps, before
    any optional extra runs.  The extras after it (multi-GPU decision variants, the
    small-batch pass) each run in try/except, all under one wall-clock budget
    (--extras-budget); when they finish, rank 0 prints a second, complete record (the same
    headline fields plus the extras).  An extra's exception is recorded in that record
    ("error" fields); a hang ends every rank with 0 after the budget (the headline is
    already out); a native abort or GPU fault inside an extra ends the job non-zero with
    the launcher naming the rank, and the headline line is still on stdout.  A backstop
    that needs no Python thread (faulthandler.dump_traceback_later) ends a rank stuck in a
    native call that holds the GIL, where neither the watchdog thread nor the budget timer
    can run: stacks on stderr, exit 1.
  Test hooks (tests/test_launch_cpu.py): MPA_BENCH_INJECT=variant_raise | extras_hang |
  hang_rank=R | extras_abort=R (rank R dies with os._exit(134) inside the extras).
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import os
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_IMG_S = 8.06  # reference FLOP-equivalent img/s at 224^2 (best, 4 ranks)


def _emulate_comm(model, step, spec, dev, reserve=0):
    """bench.py --emulate-comm: see the flag's help.  ``reserve`` > 0 mimics the comm-aware
    persistent grids of an overlapped bucket (parallel/ddp.py): the conv kernels enqueued
    between the emulated collective's launch and the optimizer size their grids to the CUs
    it leaves free."""
    from mpi_pytorch_amd.ops import _ext
    parts = [float(v) for v in spec.split(":")]
    blocks, us = int(parts[0]), parts[1]
    lds = int(parts[2]) if len(parts) > 2 else 37664  # RCCL generic kernel's static LDS
    side = torch.cuda.Stream(device=dev)
    sink = torch.zeros(max(blocks, 1), device=dev)
    head = model.fc.weight if hasattr(model, "fc") else None

    def on_grad(p):
        if p is head:
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                _ext.ext().comm_emulator(blocks, 512, lds, us, sink)
            if reserve > 0:
                _ext.ext().set_comm_reserve(reserve)

    model._mpa_arena.add_listener(on_grad)
    fin = step.bucketer.finish

    def finish():
        fin()
        torch.cuda.current_stream(dev).wait_stream(side)
        if reserve > 0:
            _ext.ext().set_comm_reserve(0)

    step.bucketer.finish = finish


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1,
                   help="ranks (one per GPU).  Without a launcher environment (WORLD_SIZE unset) "
                        "bench.py spawns them itself through mpi_pytorch_amd.launch")
    p.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                   help="cpu: plumbing check of the same code path on host ops (gloo for N>1)")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=2048,
                   help="per-GPU batch (profiles/batch_sweep_r6.txt, one MI355X, same box: 1024 -> "
                        "53.3k, 1536 -> 54.9k, 2048 -> 54.7-55.5k img/s; ~57 GB of the 288 GB "
                        "HBM, and the all-reduce's share of a data-parallel step halves again)")
    p.add_argument("--model", default="resnet18")
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--classes", type=int, default=64500)
    p.add_argument("--optimizer", default="adam")
    p.add_argument("--lr", type=float, default=4e-4)
    p.add_argument("--graph", default="auto", choices=["auto", "on", "off"])
    # A/B switches usable under rocprofv3 (which must exec bench.py directly, no env wrapper)
    p.add_argument("--res-mask", type=int, default=None, choices=[0, 1],
                   help="identity shortcut gradient read by conv1's dgrad (MPA_RES_MASK)")
    p.add_argument("--wgrad-stream", type=int, default=None, choices=[0, 1],
                   help="conv weight gradients on a side stream (MPA_WGRAD_STREAM)")
    p.add_argument("--bucket-mb", type=float, default=16.0)
    p.add_argument("--comm-dtype", default="fp32")
    p.add_argument("--comm-ctas", type=int, default=None,
                   help="CTA cap of the overlapped buckets' RCCL communicator and the CUs the "
                        "persistent conv grids leave it (0 off; default MPA_COMM_CTAS)")
    p.add_argument("--comm-reserve", type=int, default=0,
                   help="diagnostics, with --emulate-comm: CUs the persistent conv grids leave "
                        "to the emulated collective while it is in flight")
    p.add_argument("--profile-steps", type=int, default=0)
    p.add_argument("--small-batch", type=int, default=128,
                   help="after the headline measurement, also time --steps steps at this "
                        "per-GPU batch (the reference's utils.py:40 BATCH_SIZE), eager and - "
                        "on one GPU - HIP-graph replayed; reported as 'small_batch' (0: off)")
    p.add_argument("--print-losses", action="store_true", help="debug: sync + print each loss")
    p.add_argument("--timers", default="auto", choices=["auto", "on", "off"],
                   help="per-phase HIP-event times of the timed steps (data / forward / backward "
                        "/ comm_wait / optimizer) as 'phases_ms' in the JSON line; auto: on for "
                        "more than one GPU (where comm_wait shows the exposed all-reduce)")
    p.add_argument("--static-data", action="store_true",
                   help="debug: reuse one device batch (no data pipeline in the loop)")
    p.add_argument("--emulate-comm", default="",
                   help="diagnostics, BLOCKS:US[:LDS]: when the classifier gradient lands, occupy "
                        "BLOCKS CUs for US microseconds on a side stream (a stand-in for the "
                        "data-parallel all-reduce overlapping backward); the optimizer waits "
                        "for it like for the real collective")
    p.add_argument("--decisions", type=int, default=1,
                   help="more than one GPU: after the headline, also time the capped-communicator "
                        "+ reservation and bf16-wire variants and probe the all-reduce bandwidth "
                        "('multi_gpu' in the JSON; 0: off)")
    p.add_argument("--pg-timeout", type=float, default=240.0,
                   help="process-group timeout in seconds (rendezvous and every collective)")
    p.add_argument("--job-timeout", type=float, default=560.0,
                   help="self-spawned multi-GPU job: wall-clock limit of the whole job (0 off)")
    p.add_argument("--watchdog", type=float, default=180.0,
                   help="seconds without a completed step (device events) before a rank "
                        "dumps its stacks and exits 75 (0 off)")
    p.add_argument("--data-threads", type=int, default=4,
                   help="C++ producer threads of the synthetic input ring")
    p.add_argument("--data-lookahead", type=int, default=1,
                   help="1: issue batch i+1's H2D copy + preprocess on the copy stream during "
                        "step i (DevicePrefetcher lookahead); 0: at the head of step i+1")
    p.add_argument("--reserve-gib", type=float,
                   default=float(os.environ.get("MPA_RESERVE_GIB", "160")),
                   help="grow the caching allocator by one segment of this size (capped at "
                        "90%% of free device memory) before building the model (0: off; "
                        "engine.reserve_device_memory)")
    p.add_argument("--extras-budget", type=float, default=150.0,
                   help="wall-clock budget of everything after the headline measurement "
                        "(multi-GPU decisions, small-batch pass); on expiry the headline line "
                        "is printed anyway")
    args = p.parse_args(argv)
    return args


def _cpu_stat() -> dict:
    """cgroup CPU-throttling counters of this container (cgroup v2 / v1 cpu.stat; empty if
    unreadable): a cgroup over its CPU quota is frozen for the rest of the period, the host
    stops enqueueing and the GPU idles - recorded so a slow run can be told apart."""
    for f in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat",
              "/sys/fs/cgroup/cpu,cpuacct/cpu.stat"):
        try:
            out = {}
            with open(f) as fh:
                for line in fh:
                    k, v = line.split()
                    out[k] = int(v)
            return out
        except (OSError, ValueError):
            continue
    return {}


def _hbm_probe(dev, gib: int = 16, reps: int = 3):
    """Streaming-write bandwidth (GB/s) of a fresh ``gib`` GiB buffer, ``reps`` times."""
    t = torch.empty(gib << 29, dtype=torch.bfloat16, device=dev)
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        t.fill_(1.0)
        b.record()
        b.synchronize()
        out.append(round((gib << 30) / a.elapsed_time(b) / 1e6, 1))
    del t
    torch.cuda.empty_cache()
    return out


def _gpu_busy():
    """Per card of the host (amdgpu sysfs): gpu_busy_percent and the current shader clock
    level (pp_dpm_sclk's starred line), or None."""
    import glob
    vals = []
    for d in sorted(glob.glob("/sys/class/drm/card*/device")):
        try:
            busy = int(open(d + "/gpu_busy_percent").read().strip())
        except (OSError, ValueError):
            continue
        clk = None
        try:
            for line in open(d + "/pp_dpm_sclk"):
                if "*" in line:
                    clk = line.split(":", 1)[1].replace("*", "").strip()
        except OSError:
            pass
        vals.append([d.split("/")[-2], busy, clk])
    return vals or None


def _inject() -> str:
    return os.environ.get("MPA_BENCH_INJECT", "")


class _Emitter:
    """Rank 0's JSON lines: the headline record as soon as it is built, then - once the
    extras are done - one complete record (headline fields + extras).  The final record is
    printed at most once, from the main thread or not at all (the extras deadline)."""

    def __init__(self, rank: int):
        self.rank = rank
        self._lock = threading.Lock()
        self.done = False

    def _print(self, rec: dict) -> None:
        if self.rank == 0:
            print(json.dumps(rec), flush=True)

    def headline(self, rec: dict) -> None:
        with self._lock:
            self._print(dict(rec))

    def final(self, rec: dict) -> bool:
        with self._lock:
            if self.done:
                return False
            self.done = True
            self._print(dict(rec))
            return True

    def expire(self) -> bool:
        """The extras budget ran out: no final record (the headline is already out)."""
        with self._lock:
            if self.done:
                return False
            self.done = True
            return True


def _deadline(seconds: float, emitter: _Emitter, rank: int):
    """Arm the extras budget: on expiry every rank exits 0 - the headline measurement is
    complete, valid and already printed; only the optional extras after it are lost.  A
    faulthandler backstop (no Python thread, no GIL) ends a rank whose main thread is stuck
    inside a native call 30 s later."""
    def fire():
        try:
            if emitter.expire():
                sys.stderr.write("bench.py rank %d: timeout: extras exceeded %.0f s; headline "
                                 "kept\n" % (rank, seconds))
                sys.stderr.flush()
        finally:
            os._exit(0)
    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    faulthandler.dump_traceback_later(seconds + 30.0, exit=True)
    return t


def _guarded(name: str, fn):
    """Run one optional extra; an exception becomes {"error": ...} in the record."""
    try:
        return fn()
    except Exception as e:  # noqa: BLE001 - any failure of an extra must not lose the headline
        sys.stderr.write("bench.py: extra %r failed: %r\n" % (name, e))
        return {"error": "%s: %s" % (type(e).__name__, str(e)[:300])}


def _launcher_env() -> bool:
    """True when a launcher (torchrun, our launch.py, an MPI launcher) already made us a
    rank of an N-process job."""
    return any(os.environ.get(k) for k in ("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE"))


def spawn(argv, nprocs: int) -> int:
    """``python bench.py --gpus N`` outside a launcher: start N rank processes of this very
    script (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR=127.0.0.1 set by
    ``mpi_pytorch_amd.launch``), fail fast if one dies, and return the job's exit code.
    Nothing here touches the GPU: the parent only waits for its children."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "_mpa_launch", os.path.join(ROOT, "mpi_pytorch_amd", "launch.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    a = parse_args(argv)
    return mod.launch(nprocs, [sys.executable, os.path.abspath(__file__)] + list(argv),
                      timeout=a.job_timeout)


def _timed(step, data, args, world, sync) -> float:
    """Whole-job img/s of ``args.steps`` steps after ``args.warmup`` warm-up steps, bracketed
    like the headline measurement (barrier + device sync, max time over ranks)."""
    from mpi_pytorch_amd.parallel import barrier
    from mpi_pytorch_amd.engine import steps_without_gc
    for _ in range(max(args.warmup, 2)):
        x, y = data.next()
        step(x, y)
    # the training driver's loop policy: cyclic GC at the boundaries, not mid-step
    with steps_without_gc():
        sync()
        barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            x, y = data.next()
            step(x, y)
        sync()
        barrier()
        sync()
        t1 = time.perf_counter()
    t = torch.tensor([t1 - t0], dtype=torch.float64, device=world.device)
    if world.world_size > 1:
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return args.steps * data.batch * world.world_size / float(t.item())


def _variant(step, data, args, world, sync, configure, restore) -> dict:
    """Re-time the headline step under another communication setting (``configure()``
    applies it on every rank, ``restore()`` undoes it): img/s over ``args.steps`` steps
    bracketed like the headline, with the per-bucket comm stats and - on GPUs - the phase
    times (``comm_wait`` is the exposed all-reduce).  Decision data for the multi-GPU
    defaults, recorded beside the headline rather than instead of it."""
    from mpi_pytorch_amd.parallel import barrier
    from mpi_pytorch_amd.engine import steps_without_gc
    info = configure() or {}
    try:
        if _inject() == "variant_raise":
            raise RuntimeError("injected variant failure")
        for _ in range(max(min(args.warmup, 3), 1)):
            x, y = data.next()
            step(x, y)
        if step.timer is not None:
            step.timer.summary()  # (drop the warm-up steps)
        step.bucketer.enable_comm_stats()
        with steps_without_gc():
            sync()
            barrier()
            sync()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                x, y = data.next()
                step(x, y)
            sync()
            barrier()
            sync()
            dt = time.perf_counter() - t0
        t = torch.tensor([dt], dtype=torch.float64, device=world.device)
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        out = dict(info)
        out.update(img_per_s=round(args.steps * data.batch * world.world_size / dt, 2),
                   ms_per_step=round(dt * 1000.0 / args.steps, 3))
        if step.timer is not None:
            out["phases_ms"] = step.timer.summary()
        comm = step.bucketer.comm_stats()
        if comm is not None:
            out["comm"] = comm
        return out
    finally:
        restore()


def _allreduce_probe(world, mb: float = 126.0, iters: int = 10, group=None) -> dict:
    """Standalone all-reduce of one ``mb`` MiB fp32 buffer (ResNet-18's 126 MiB classifier
    bucket) outside the training step: mean time over ``iters`` back-to-back collectives
    (max over ranks), algorithm bandwidth and ring bus bandwidth (algbw * 2(n-1)/n, the
    per-link figure nccl-tests reports; xGMI: ~153 GB/s per link)."""
    import torch.distributed as dist
    from mpi_pytorch_amd.parallel import barrier
    dev = world.device
    n = max(int(mb * 2**20) // 4, 1)
    buf = torch.ones(n, dtype=torch.float32, device=dev)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for _ in range(3):
        dist.all_reduce(buf, group=group)
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(buf, group=group)
    sync()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms = float(t.item()) * 1e3 / iters
    algbw = n * 4 / (ms * 1e-3) / 1e9
    ws = world.world_size
    del buf
    return {"mb": round(n * 4 / 2**20, 2), "iters": iters, "ms": round(ms, 4),
            "algbw_gbs": round(algbw, 2), "busbw_gbs": round(algbw * 2.0 * (ws - 1) / ws, 2)}


def _multi_gpu_decisions(step, data, args, world, sync) -> dict:
    """world_size > 1: the headline's communication alternatives, each timed like it - a
    CTA-capped communicator for the overlapped buckets plus the persistent-grid
    reservation (parallel/ddp.py ``comm_ctas``), and the bf16 wire format - and the raw
    all-reduce bandwidth of the default (and capped) communicator."""
    b = step.bucketer
    res = {}
    orig_ctas, orig_dtype = b.comm_ctas, b.comm_dtype
    probe = {"default": _guarded("allreduce_probe", lambda: _allreduce_probe(world))}

    def capped_on():
        ok = b.set_comm_ctas(8 if orig_ctas == 0 else 0)
        if ok and b.overlap_group is not None:
            probe["capped"] = _allreduce_probe(world, group=b.overlap_group)
        return {"comm_ctas": b.comm_ctas, "capped_communicator": bool(ok)}

    res["comm_ctas8" if orig_ctas == 0 else "comm_ctas0"] = _guarded("comm_ctas", lambda: _variant(
        step, data, args, world, sync, capped_on, lambda: b.set_comm_ctas(orig_ctas)))

    def bf16_on():
        b.comm_dtype = "bf16" if orig_dtype != "bf16" else "fp32"
        return {"comm_dtype": b.comm_dtype, "wire_mb": b.wire_mb()}

    def bf16_off():
        b.comm_dtype = orig_dtype

    res["comm_bf16" if orig_dtype != "bf16" else "comm_fp32"] = _guarded("comm_dtype", lambda: _variant(
        step, data, args, world, sync, bf16_on, bf16_off))
    def wgs_on():
        step.wgrad_stream_ddp = not orig_wgs
        return {"wgrad_stream_ddp": step.wgrad_stream_ddp}

    orig_wgs = step.wgrad_stream_ddp
    res["wgrad_stream_on" if not orig_wgs else "wgrad_stream_off"] = _guarded(
        "wgrad_stream", lambda: _variant(step, data, args, world, sync, wgs_on,
                                         lambda: setattr(step, "wgrad_stream_ddp", orig_wgs)))
    res["allreduce_probe"] = probe
    return res


def run(args) -> None:
    from mpi_pytorch_amd.parallel import init_world, barrier
    from mpi_pytorch_amd.engine import build_training
    from mpi_pytorch_amd.engine.step import markers
    from mpi_pytorch_amd.data import DevicePrefetcher
    from mpi_pytorch_amd.models import input_spec

    cuda = args.device == "cuda"
    timers = args.timers == "on" or (args.timers == "auto" and args.gpus > 1)
    world = init_world(args.device, timeout_s=args.pg_timeout, comm_timing=timers and cuda)
    if world.world_size != args.gpus:
        raise SystemExit("bench.py: --gpus {} but this job has {} ranks".format(
            args.gpus, world.world_size))
    torch.manual_seed(0)
    dev = world.device
    # device memory free at start (a previous process's memory still being released shows
    # here; see docs/NOTES.md "Slow processes")
    mem0 = [round(v / 2**30, 1) for v in torch.cuda.mem_get_info(dev)] if cuda else None
    bw0 = _hbm_probe(dev) if cuda else None
    from mpi_pytorch_amd.engine import reserve_device_memory
    share = max(1, -(-world.world_size // max(torch.cuda.device_count(), 1))) if cuda else 1
    reserved = reserve_device_memory(dev, args.reserve_gib / share)  # (ranks per GPU share it)

    def sync():
        if cuda:
            torch.cuda.synchronize()

    hw = (args.image_size, args.image_size)
    model, opt, step, _ = build_training(args.model, args.classes, dev, world, args.lr,
                                         args.optimizer, bucket_mb=args.bucket_mb,
                                         comm_dtype=args.comm_dtype, comm_ctas=args.comm_ctas)
    spec = input_spec(model, hw)  # the stem's image layout, written by the preprocess kernel
    data = DevicePrefetcher(dev, args.batch, hw, hw, args.classes, seed=1234, rank=world.rank,
                            world=world.world_size, depth=6, threads=args.data_threads,
                            cpad=spec["cpad"], pad=spec["pad"],
                            lookahead=bool(args.data_lookahead))

    if args.static_data:
        xs, ys = data.next()
        data.next = lambda: (xs, ys)
    if args.emulate_comm:
        _emulate_comm(model, step, args.emulate_comm, dev, args.comm_reserve)
    # progress watchdog over warm-up and the timed steps: a rank whose device stops
    # completing steps (a peer lost inside a collective) exits 75 instead of hanging
    from mpi_pytorch_amd.parallel.watchdog import Watchdog
    wd = Watchdog(args.watchdog, rank=world.rank, name="bench").start()
    if args.watchdog > 0:  # (no Python thread: fires even with the GIL held by a native call)
        faulthandler.dump_traceback_later(args.watchdog + 60.0, exit=True)
    inject = _inject()
    hang_rank = int(inject.split("=", 1)[1]) if inject.startswith("hang_rank=") else -1
    nbeat = [0]

    def beat():
        nbeat[0] += 1
        if args.watchdog > 0:  # re-arm the GIL-free backstop: it measures time since a beat
            faulthandler.dump_traceback_later(args.watchdog + 60.0, exit=True)
        if cuda:
            ev = torch.cuda.Event()
            ev.record()
            wd.beat_on(nbeat[0], ev)
        else:
            wd.beat(nbeat[0])

    # eager by default: the step is GPU-bound (host runs ahead), graph replay buys nothing
    # measurable and needs a per-step sync for correctness (engine/step.py)
    use_graph = args.graph == "on" and cuda
    if use_graph:
        x, y = data.next()
        use_graph = step.capture(x, y)
    for _ in range(args.warmup):
        x, y = data.next()
        loss = step(x, y)
        beat()
        if args.print_losses and world.rank == 0:
            print("warmup loss %.4f" % float(loss), file=sys.stderr)
    if args.print_losses:
        for i in range(args.steps):
            x, y = data.next()
            print("step %d loss %.4f" % (i, float(step(x, y))), file=sys.stderr)
        lazy = []
        for i in range(args.steps):
            x, y = data.next()
            lazy.append(step(x, y).clone())
        print("lazy losses:", " ".join("%.3f" % float(v) for v in lazy), file=sys.stderr)
        print("loss_sum/steps: %.4f" % step.mean_loss(), file=sys.stderr)
    if timers and not use_graph:
        step.enable_timers()
    if timers:
        step.bucketer.enable_comm_stats()
    mk = step.markers
    step.mean_loss()  # the reported loss is the timed steps' mean
    data_stats = getattr(data, "ring_stats", lambda reset=True: None)
    data_stats(True)  # starvation counters of the timed steps only
    sync()
    barrier()
    sync()
    cs0, cpu0 = _cpu_stat(), time.process_time()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i == 1 and world.rank == hang_rank:
            time.sleep(1e6)  # test hook: a rank that never reaches its next collective
        if mk is not None:
            mk.range_push("data")
        x, y = data.next()
        if mk is not None:
            mk.range_pop()
        step(x, y)
        beat()
    # (sampled while the device still runs the last queued steps; host side only;
    # MPA_BENCH_CARDS=1: every card of the host, a diagnostic of the slow-process study)
    cards = _gpu_busy() if cuda and os.environ.get("MPA_BENCH_CARDS") == "1" else None
    sync()
    barrier()
    sync()
    dt = time.perf_counter() - t0
    cs1, cpu1 = _cpu_stat(), time.process_time()
    wd.stop()
    faulthandler.cancel_dump_traceback_later()
    loss = step.mean_loss()
    phases = step.timer.summary() if step.timer is not None else None
    comm = step.bucketer.comm_stats()
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world.world_size > 1:
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    imgs = args.steps * args.batch * world.world_size
    value = imgs / dt
    ring = data_stats(True)

    # ---- the headline record, complete before any optional extra runs
    metric = "images/sec (whole node) ResNet-18 224x224 training at 1/2/4/8 MI355X"
    if args.model != "resnet18" or args.image_size != 224:  # a zoo run, not the headline
        metric = "images/sec (whole node) {} {}x{} training on {} MI355X".format(
            args.model, args.image_size, args.image_size, world.world_size)
    rec = {
        "metric": metric,
        "value": round(value, 2),
        "unit": "images/sec",
        "n_gpus": world.world_size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt * 1000.0 / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / BASELINE_IMG_S, 2),
        "dtype": "bf16" if cuda else "fp32",
        "data": "synthetic",
        "config": {
            "model": args.model,
            "global_batch": args.batch * world.world_size,
            "per_gpu_batch": args.batch,
            "seq_len": None,
            "image_size": args.image_size,
            "num_classes": args.classes,
            "optimizer": args.optimizer,
            "parallelism": "dp{}".format(world.world_size),
            "device": args.device,
            "backend": world.backend,
            "hip_graph": bool(use_graph),
            "mean_loss": round(loss, 4),
        },
    }
    if phases is not None:
        rec["phases_ms"] = phases
    if world.world_size > 1:
        rec["grad_allreduce_mb"] = step.bucketer.wire_mb()
        rec["comm_ctas"] = step.bucketer.comm_ctas if step.bucketer.overlap_group else 0
    if comm is not None:
        rec["comm"] = comm
    if ring is not None:
        rec["data_ring"] = ring
    host = {"process_cpu_s": round(cpu1 - cpu0, 3)}
    if "throttled_usec" in cs1:
        host["cgroup_throttled_ms"] = round((cs1["throttled_usec"] -
                                             cs0.get("throttled_usec", 0)) / 1e3, 1)
        host["cgroup_nr_throttled"] = cs1.get("nr_throttled", 0) - cs0.get("nr_throttled", 0)
    if mem0 is not None:
        host["device_free_total_gib_at_start"] = mem0
        host["hbm_probe_at_start_gbps"] = bw0
        host["reserved_gib"] = reserved
        if cards is not None:
            host["cards_busy_sclk"] = cards
    rec["host"] = host
    from mpi_pytorch_amd.parallel.dist import affinity
    if affinity() is not None:
        rec["host_affinity"] = affinity()

    # ---- the headline line goes out now: nothing after this point can lose it
    emitter = _Emitter(world.rank)
    emitter.headline(rec)
    # ---- optional extras, each guarded, all under one wall-clock budget
    timer = _deadline(args.extras_budget, emitter, world.rank)
    if inject == "extras_hang":
        time.sleep(1e6)
    if inject == "extras_gil_hang":  # test hook: a native call that blocks holding the GIL
        import ctypes
        ctypes.PyDLL(None).sleep(1000000)
    if inject.startswith("extras_abort=") and world.rank == int(inject.split("=", 1)[1]):
        os._exit(134)  # test hook: a native abort inside an extra
    if world.world_size > 1 and not args.emulate_comm and args.decisions:
        rec["multi_gpu"] = _guarded("multi_gpu", lambda: _multi_gpu_decisions(
            step, data, args, world, sync))
    if args.small_batch and args.small_batch != args.batch and cuda and not args.emulate_comm:
        def small_pass():
            nonlocal data
            step.timer = None
            step.bucketer._stats = None
            data.close()
            data = DevicePrefetcher(dev, args.small_batch, hw, hw, args.classes, seed=4321,
                                    rank=world.rank, world=world.world_size, depth=6,
                                    threads=2, cpad=spec["cpad"], pad=spec["pad"])
            small = {"per_gpu_batch": args.small_batch,
                     "eager_img_per_s": round(_timed(step, data, args, world, sync), 1)}
            if world.world_size == 1:
                x, y = data.next()
                if step.capture(x, y):
                    small["graph_img_per_s"] = round(_timed(step, data, args, world, sync), 1)
            step.mean_loss()
            return small
        rec["small_batch"] = _guarded("small_batch", small_pass)
    timer.cancel()
    faulthandler.cancel_dump_traceback_later()
    if "multi_gpu" in rec or "small_batch" in rec:
        emitter.final(rec)
    data.close()
    from mpi_pytorch_amd.parallel import shutdown
    shutdown()


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.gpus > 1 and not _launcher_env():
        sys.exit(spawn(argv, args.gpus))
    from mpi_pytorch_amd.ops import functional as Fn
    if args.res_mask is not None:
        Fn._RES_MASK = bool(args.res_mask)
    if args.wgrad_stream is not None:
        Fn._WGRAD_STREAM = bool(args.wgrad_stream)
    run(args)


if __name__ == "__main__":
    main()
