"""Pipelined inference: read -> resize -> normalize -> predict as HIP-stream stages.

Reference (``/root/reference/evaluation_pipeline.py:44-199``): an MPMD job with one MPI
rank per stage - rank 0 decodes images and sends pickled PIL images (~2 MB each) to rank
1, which resizes (PIL bicubic+antialias, :89) and sends to rank 2, which runs
ToTensor+Normalize (:116-122) and sends 3x128x128 fp32 tensors to one of the predictor
ranks 3..N-1 chosen uniformly at random per image (:178); predictors run batch-1 forward
passes from the checkpoint (:132-159); the per-predictor ``corrects / dataset_size`` are
SUM-reduced to rank 0 (:196) which logs ``Accuracy is ...`` (:199).  Needs >= 4 ranks.

Here, on one MI355X:
  stage 0  read/decode   the native ``BatchRing`` (csrc/runtime): C++ threads copy each
                         manifest row's synthetic image (a texture window,
                         ``SyntheticImages``) into pinned slots, or PIL decode threads write
                         real JPEGs into a slot (each image at its own extent inside the
                         slot pitch); slots come back to the consumer in batch order;
  stage 1  transfer      pinned slot -> HBM copy on a copy stream (event-ordered); the slot
                         returns to the ring once its copy event has completed;
  stage 2  resize+norm   the PIL-exact preprocess kernels (mode 1, bit-exact with PIL's
                         uint8 resize, per-image extents) on a preprocess stream;
  stage 3  predict       ``lanes`` predictor lanes, each a HIP stream running a *batched*
                         eval forward + fused argmax/correct-count; each batch goes to a
                         lane chosen at random (reference behaviour) or round-robin.
Stages overlap through events; ring depth bounds the in-flight batches (the end-of-stream
sentinel is the ring's batch count).  Accuracy = sum over lanes of correct_lane /
dataset_size, like the reference's reduce.  With several GPUs each rank takes an
``array_split`` shard and the per-rank partial accuracies are SUM-reduced (RCCL) -
predictor fan-out across GPUs.  The CPU path runs the same stages without streams.
"""
from __future__ import annotations

import os
import time
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..config import Config
from ..checkpoint import read_checkpoint
from ..data.loader import IMAGENET_MEAN, IMAGENET_STD
from ..data.manifest import SyntheticImages, FolderImages, images_available, synthetic_manifest
from ..models import initialize_model, input_spec
from ..ops import functional as Fn
from ..parallel import init_world, reduce_scalar, shard_dataframe, broadcast_object, ParamArena
from ..utils.logging import init_logger


def load_predictor(cfg: Config, device, ckpt_path: Optional[str] = None):
    """``initialize_model(..., use_pretrained=False)`` + checkpoint ``state_dict``
    (evaluation_pipeline.py:138-147)."""
    model, _ = initialize_model(cfg.MODEL_NAME, cfg.NUM_CLASSES, False, use_pretrained=False)
    model = model.to(device)
    model._mpa_arena = ParamArena(model, device)
    path = ckpt_path or os.path.join(cfg.CHECKPOINT_DIR, "checkpoint_{}.pt".format(cfg.MODEL_NAME))
    if os.path.exists(path):
        sd = read_checkpoint(path)["state_dict"]
        model.load_state_dict(sd)
        model._mpa_arena.sync_shadow()
    model.eval()
    return model


class StreamPipeline:
    def __init__(self, model, device, out_hw, lanes: int = 1, depth: int = 4,
                 assign: str = "random", seed: int = 0, mode: int = 1, cpad=None, pad=None):
        self.model = model
        if cpad is None:  # the model stem's input layout (models.input_spec)
            spec = input_spec(model, out_hw)
            cpad, pad = spec["cpad"], spec["pad"]
        self.pad = pad
        self.device = torch.device(device)
        self.out_hw = out_hw
        self.lanes = max(1, lanes)
        self.depth = max(2, depth)
        self.assign = assign
        self.rng = np.random.default_rng(seed)
        self.mode = mode
        self.cpad = cpad
        self.cuda = self.device.type == "cuda"
        if self.cuda:
            self.copy_stream = torch.cuda.Stream(self.device)
            self.prep_stream = torch.cuda.Stream(self.device)
            self.lane_streams = [torch.cuda.Stream(self.device) for _ in range(self.lanes)]
        self.counts = [torch.zeros(1, dtype=torch.int64, device=self.device)
                       for _ in range(self.lanes)]
        self.seen = [0] * self.lanes
        self._pinned = {}
        self._last_slot = None

    def _lane_for(self, i: int) -> int:
        if self.assign == "roundrobin":
            return i % self.lanes
        return int(self.rng.integers(0, self.lanes))

    def _staging(self, g: torch.Tensor) -> torch.Tensor:
        """Copy a host batch into a reusable pinned buffer (a ring of ``depth + 2``
        slots; a slot is reused only after the copy that read it has completed)."""
        key = (tuple(g.shape), g.dtype)
        ring = self._pinned.setdefault(key, [])
        for slot in ring:
            if slot[1] is None or slot[1].query():
                buf = slot[0]
                break
        else:
            if len(ring) >= self.depth + 2:
                ring[0][1].synchronize()
                buf = ring[0][0]
                slot = ring[0]
            else:
                buf = torch.empty(g.shape, dtype=g.dtype).pin_memory()
                slot = [buf, None]
                ring.append(slot)
        buf.copy_(g)
        self._last_slot = slot
        return buf

    def _preprocess(self, imgs):
        ext = None
        if not isinstance(imgs, np.ndarray):  # decoded images of different sizes: one
            imgs, ext = pad_batch(imgs)        # padded batch + extents, ONE preprocess
        g = torch.from_numpy(imgs)
        if not self.cuda:
            return Fn.preprocess(g, self.out_hw, IMAGENET_MEAN, IMAGENET_STD, self.mode,
                                 self.cpad, out_dtype=torch.float32, pad=self.pad,
                                 extents=ext), None
        g = self._staging(g)
        with torch.cuda.stream(self.copy_stream):
            gd = g.to(self.device, non_blocking=True)
            copied = torch.cuda.Event()
            copied.record(self.copy_stream)
        self._last_slot[1] = copied  # pinned slot free once this copy is done
        self.prep_stream.wait_stream(self.copy_stream)
        with torch.cuda.stream(self.prep_stream):
            gd.record_stream(self.prep_stream)
            x = Fn.preprocess(gd, self.out_hw, IMAGENET_MEAN, IMAGENET_STD, self.mode,
                              self.cpad, pad=self.pad, extents=ext)
            ev = torch.cuda.Event()
            ev.record(self.prep_stream)
        return x, ev

    @torch.no_grad()
    def run(self, batches) -> List[int]:
        """``batches`` yields (uint8 images, int64 labels); returns per-lane correct counts."""
        inflight = []
        for i, (imgs, labels) in enumerate(batches):
            x, ev = self._preprocess(imgs)
            lane = self._lane_for(i)
            if self.cuda:
                s = self.lane_streams[lane]
                s.wait_event(ev)
                with torch.cuda.stream(s):
                    x.record_stream(s)
                    y = labels.pin_memory().to(self.device, non_blocking=True)
                    out = self.model(x)
                    Fn.count_correct(out, y, self.counts[lane])
                    done = torch.cuda.Event()
                    done.record(s)
                inflight.append(done)
                if len(inflight) >= self.depth:
                    inflight.pop(0).synchronize()
            else:
                out = self.model(x)
                Fn.count_correct(out, labels, self.counts[lane])
            self.seen[lane] += int(labels.shape[0])
        if self.cuda:
            for s in self.lane_streams:
                s.synchronize()
        return [int(c.item()) for c in self.counts]



    @torch.no_grad()
    def run_ring(self, ring, nbatches: int) -> List[int]:
        """GPU stages fed by a native ``BatchRing``: no per-batch host copy, pinning or
        Python image work on the consumer thread.  Returns per-lane correct counts."""
        pending = []   # (slot, copy event): the slot returns to the ring once copied
        inflight = []  # lane completion events (bounds the batches in flight)
        depth = ring.depth()
        for i in range(nbatches):
            keep = []
            for k, (slot, ev) in enumerate(pending):
                if ev.query() or len(pending) - k >= depth - 1:
                    ev.synchronize()
                    ring.release(slot)
                else:
                    keep.append((slot, ev))
            pending = keep
            slot, img_h, lab_h, _bidx = ring.acquire()
            n, ext_h = ring.info(slot)
            ext = ext_h[:n].numpy().copy()
            uniform = bool((ext[:, 0] == img_h.shape[1]).all() and (ext[:, 1] == img_h.shape[2]).all())
            with torch.cuda.stream(self.copy_stream):
                img_d = img_h[:n].to(self.device, non_blocking=True)
                lab_d = lab_h[:n].to(self.device, non_blocking=True)
                copied = torch.cuda.Event()
                copied.record(self.copy_stream)
            pending.append((slot, copied))
            self.prep_stream.wait_event(copied)
            with torch.cuda.stream(self.prep_stream):
                img_d.record_stream(self.prep_stream)
                x = Fn.preprocess(img_d, self.out_hw, IMAGENET_MEAN, IMAGENET_STD, self.mode,
                                  self.cpad, pad=self.pad, extents=None if uniform else ext)
                prepped = torch.cuda.Event()
                prepped.record(self.prep_stream)
            lane = self._lane_for(i)
            s = self.lane_streams[lane]
            s.wait_event(prepped)
            with torch.cuda.stream(s):
                x.record_stream(s)
                lab_d.record_stream(s)
                out = self.model(x)
                Fn.count_correct(out, lab_d, self.counts[lane])
                done = torch.cuda.Event()
                done.record(s)
            inflight.append(done)
            if len(inflight) >= self.depth:
                inflight.pop(0).synchronize()
            self.seen[lane] += n
        for slot, ev in pending:
            ev.synchronize()
            ring.release(slot)
        for s in self.lane_streams:
            s.synchronize()
        return [int(c.item()) for c in self.counts]


def pad_batch(imgs):
    """A list of uint8 HWC images of different sizes -> one zero-padded [B, Hmax, Wmax, 3]
    batch and the per-image extents [B, 2] (each image at the top-left of its slot)."""
    H = max(a.shape[0] for a in imgs)
    W = max(a.shape[1] for a in imgs)
    buf = np.zeros((len(imgs), H, W, 3), dtype=np.uint8)
    for b, a in enumerate(imgs):
        buf[b, :a.shape[0], :a.shape[1]] = a
    return buf, np.array([a.shape[:2] for a in imgs], dtype=np.int64)


def make_ring(names: Sequence[str], labels: Sequence[int], batch: int, source, num_classes: int,
              depth: int = 8, threads: int = 4, pitch=None):
    """Stage 0 on the native ring for one manifest shard.  ``SyntheticImages``: window mode
    (C++ threads, bitwise ``source.load``).  ``FolderImages``: PIL decode threads write each
    image into its slot at its own extent (``pitch`` = the largest image, from the
    manifest's height/width columns when given).  Returns (ring, number of batches)."""
    from ..ops import _ext
    nb = (len(names) + batch - 1) // batch
    if isinstance(source, SyntheticImages):
        H, W = source.hw
        ring = _ext.ext().BatchRing(batch, H, W, num_classes, depth, threads, 0, 0, 1, False)
        offs = torch.tensor([source._offset(n) for n in names], dtype=torch.int64).view(-1, 2)
        ring.set_window_source(torch.from_numpy(source.tex), offs,
                               torch.as_tensor(np.asarray(labels, dtype=np.int64)))
        return ring, nb
    if pitch is None:
        raise ValueError("make_ring: real images need the slot pitch (max height, width)")
    ring = _ext.ext().BatchRing(batch, int(pitch[0]), int(pitch[1]), num_classes, depth, threads,
                                0, 0, 1, False)
    _feed_external(ring, list(names), np.asarray(labels, dtype=np.int64), batch, source, threads)
    return ring, nb


_FEED_ERRORS = {}  # id(ring) -> decode exceptions of its feeder threads


def feed_error(ring):
    """The first exception a decode thread of ``ring`` hit (it then stopped the ring), or
    None."""
    errs = _FEED_ERRORS.get(id(ring))
    return errs[0] if errs else None


def _feed_external(ring, names, labels, batch, source, threads: int) -> None:
    """PIL decode threads for real images: each takes an empty slot, THEN the next batch
    index, decodes its images straight into the slot (top-left, extent recorded) and
    commits it.  The ring hands batches to the consumer in index order, so a thread must
    own a slot before it owns an index: otherwise later indices could fill every free slot
    while the thread holding the next one waits for a slot forever.  A decode error stops
    the ring (the consumer's acquire raises instead of hanging; ``feed_error`` has it)."""
    nb = (len(names) + batch - 1) // batch
    lock = threading.Lock()
    nxt = [0]
    errors = _FEED_ERRORS.setdefault(id(ring), [])

    def worker():
        from PIL import Image
        while True:
            try:
                slot, img, lab, ext = ring.acquire_empty()
            except RuntimeError:  # ring stopped
                return
            with lock:
                bi = nxt[0]
                nxt[0] += 1
            if bi >= nb:
                ring.release(slot)
                return
            try:
                a = img.numpy()
                e = ext.numpy()
                lo, hi = bi * batch, min((bi + 1) * batch, len(names))
                for b, j in enumerate(range(lo, hi)):
                    with Image.open(os.path.join(source.root, names[j])) as im:
                        arr = np.asarray(im.convert("RGB"))
                    h, w = min(arr.shape[0], a.shape[1]), min(arr.shape[1], a.shape[2])
                    a[b, :h, :w] = arr[:h, :w]
                    e[b] = (h, w)
                    lab.numpy()[b] = labels[j]
            except Exception as ex:  # noqa: BLE001 - reported through feed_error
                errors.append(ex)
                ring.stop()
                return
            ring.commit(slot, bi, hi - lo)

    for _ in range(max(1, threads)):
        threading.Thread(target=worker, name="mpa-decode", daemon=True).start()


def _batches(names, labels, batch: int, source, prefetch: int = 2):
    """Stage 0: host read/decode in a worker pool, ``prefetch`` batches ahead."""
    pool = ThreadPoolExecutor(max_workers=2)
    idx = [np.arange(i, min(i + batch, len(names))) for i in range(0, len(names), batch)]
    futs = [pool.submit(source.load, [names[j] for j in ix]) for ix in idx[:prefetch]]
    for k, ix in enumerate(idx):
        imgs = futs[k].result()
        if k + prefetch < len(idx):
            futs.append(pool.submit(source.load, [names[j] for j in idx[k + prefetch]]))
        yield imgs, torch.as_tensor(np.asarray([labels[j] for j in ix], dtype=np.int64))
    pool.shutdown()


def run_pipeline(cfg: Config, ckpt_path: Optional[str] = None, max_images: int = 0) -> float:
    world = init_world(cfg.device, cfg.timeout_s)
    log = init_logger(world.rank, cfg.log_file or "evaluation.log", cfg.log_per_rank_files)
    df = None
    if world.rank == 0:
        log.info("Logger Initialized")
        if os.path.exists(cfg.TEST_CSV) and cfg.synthetic_images <= 0:
            import pandas as pd
            df = pd.read_csv(cfg.TEST_CSV)
        else:
            df = synthetic_manifest(cfg.synthetic_images or 256, cfg.NUM_CLASSES, cfg.seed)
        if max_images:
            df = df.iloc[:max_images]
    df = broadcast_object(df)
    dataset_size = len(df)
    shard = shard_dataframe(df, world.world_size)[world.rank]
    out_hw = cfg.input_hw if cfg.MODEL_NAME != "inception" else (299, 299)
    names = list(shard["file_name"].values)
    labels = list(shard["category_id"].values)
    if not cfg.synthetic and images_available(cfg.TRAIN_DIR, names):
        source = FolderImages(cfg.TRAIN_DIR, cfg.num_workers)  # reads TRAIN_DIR like :59
    else:
        # synthetic sources at the model's input size by default (eval_src > 0: that side):
        # the resize stage still runs (PIL-exact bicubic), but stage 0 copies and the H2D
        # link carries 150 KB per 224^2 image instead of the 600 KB of a 448^2 source,
        # which capped the pipeline near PCIe's ~50 GB/s / 600 KB = 83k img/s
        side = cfg.eval_src
        source = SyntheticImages((side, side) if side > 0 else tuple(out_hw))
    model = load_predictor(cfg, world.device, ckpt_path)
    pipe = StreamPipeline(model, world.device, out_hw, cfg.eval_lanes, assign=cfg.eval_assign,
                          seed=cfg.seed + world.rank)
    t0 = time.perf_counter()
    if world.device.type == "cuda":
        pitch = None
        if isinstance(source, FolderImages):
            pitch = (int(shard["height"].max()), int(shard["width"].max())) \
                if {"height", "width"} <= set(shard.columns) else (1024, 1024)
        ring, nb = make_ring(names, labels, cfg.eval_batch, source, cfg.NUM_CLASSES,
                             threads=max(2, cfg.num_workers), pitch=pitch)
        try:
            counts = pipe.run_ring(ring, nb)
        except RuntimeError as e:
            fe = feed_error(ring)
            if fe is not None:
                raise RuntimeError("eval pipeline: image decode failed: %r" % (fe,)) from e
            raise
        finally:
            ring.stop()
            _FEED_ERRORS.pop(id(ring), None)
    else:
        counts = pipe.run(_batches(names, labels, cfg.eval_batch, source))
    dt = time.perf_counter() - t0
    acc_local = 0.0
    for lane, c in enumerate(counts):
        a = c / max(dataset_size, 1)
        acc_local += a
        log.info("Finished node {}, acc {}".format(world.rank * pipe.lanes + lane + 3, a))
    total = reduce_scalar(acc_local, root=0)
    if world.rank == 0:
        log.info("Accuracy is {}".format(total))
        # the source extent is part of the number: a synthetic source at the model's input
        # size skips the downscale real ~1000x677 herbarium JPEGs need (cfg.eval_src)
        src = "real images" if isinstance(source, FolderImages) else \
            "synthetic {}x{} source".format(*source.hw)
        log.info("_Throughput: {:.1f} img/s ({} images, {} lanes x {} ranks, {})".format(
            dataset_size / dt if dt > 0 else 0.0, dataset_size, pipe.lanes, world.world_size,
            src))
    return float(total) if total is not None else acc_local


@torch.no_grad()
def plain_eval(model, names, labels, batch, source, device, out_hw, mode=1) -> int:
    """Non-pipelined batched evaluation (oracle for the pipeline tests): host batches,
    one preprocess call per batch in the model's input layout (images of different sizes
    padded into one batch with extents), forward, correct count."""
    spec = input_spec(model, out_hw)
    correct = torch.zeros(1, dtype=torch.int64, device=device)
    for imgs, lab in _batches(names, labels, batch, source):
        ext = None
        if not isinstance(imgs, np.ndarray):
            imgs, ext = pad_batch(imgs)
        g = torch.from_numpy(imgs).to(device)
        x = Fn.preprocess(g, out_hw, IMAGENET_MEAN, IMAGENET_STD, mode, spec["cpad"],
                          out_dtype=torch.float32, pad=spec["pad"], extents=ext)
        Fn.count_correct(model(x), lab.to(device), correct)
    return int(correct.item())
