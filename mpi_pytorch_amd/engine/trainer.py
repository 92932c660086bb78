"""Data-parallel training driver: the reference ``main.py::main()`` workflow
(``/root/reference/main.py:49-185``) on the MI355X engine.

Workflow parity (and the reference lines it mirrors):
  * logger + ``Logger Initialized`` on rank 0 (main.py:22-46)
  * rank 0 reads/samples/splits the manifest (main.py:73-82); shards with
    ``np.array_split`` semantics and scatters them (main.py:84,91) -> ``_Files Received``
  * train loader over the shard (bs=BATCH_SIZE, shuffle) and, on rank 0, a validation
    loader over ``train_sample`` (main.py:99-112)
  * ``initialize_model`` + Adam(lr=LR) (main.py:121-126); optional resume (main.py:127-130)
  * broadcast of rank-0 parameters (main.py:131)
  * epochs: train, per-rank ``_Epoch: e | Train Loss: l | Time: t`` (main.py:142-160);
    rank-0 checkpoint every epoch (main.py:162-171) and validation accuracy
    (main.py:173-185)

Engine differences (MI355X-first): NHWC/bf16 fused MFMA kernels, flat-arena bucketed RCCL
all-reduce overlapped with backward, fused optimizer, GPU preprocessing, a prefetch
thread for the host image work, device-side loss accumulation (one host sync per epoch
instead of one per step), equal step counts on every rank (the reference can deadlock
when shard batch counts differ), resume honours the saved epoch.
"""
from __future__ import annotations

import math
import os
import time
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..config import Config
from ..checkpoint import save_checkpoint, load_checkpoint, build_state, checkpoint_path
from ..parallel.watchdog import Watchdog
from ..data.manifest import (read_manifests, synthetic_manifest, SyntheticImages, FolderImages,
                             images_available)
from ..data.loader import IMAGENET_MEAN, IMAGENET_STD
from ..ops import functional as Fn
from ..parallel import (init_world, get_world, barrier, scatter_object, broadcast_object,
                        all_gather_object,
                        shard_dataframe, array_split_sizes, replica_checksum)
from ..parallel.sharding import equal_step_count
from ..utils.logging import init_logger, MetricsWriter, log_rank_lines
from .step import build_training, steps_without_gc
from ..models import input_spec


class ManifestBatches:
    """Batches of a manifest shard -> model-ready NHWC tensors on ``device``.

    Host work (synthetic generation or PIL decode) for batch i+1 runs in a worker thread
    while the GPU trains on batch i; images are copied pinned/non-blocking and
    normalised by the GPU preprocess kernel (bilinear resize, no antialias - the
    reference's ToTensor -> Resize -> Normalize on tensors, main.py:62-65)."""

    def __init__(self, names: Sequence[str], labels: Sequence[int], batch: int, out_hw,
                 device, source, shuffle: bool, seed: int = 0, mode: int = 0, cpad: int = 8,
                 pad=None):
        self.names = list(names)
        self.labels = np.asarray(labels, dtype=np.int64)
        self.batch = batch
        self.out_hw = out_hw
        self.device = torch.device(device)
        self.source = source
        self.shuffle = shuffle
        self.seed = seed
        self.mode = mode
        self.cpad = cpad
        self.pad = pad
        self.pool = ThreadPoolExecutor(max_workers=1)

    def set_layout(self, spec: dict) -> None:
        """Produce the model stem's input layout (``models.input_spec``)."""
        self.cpad = spec["cpad"]
        self.pad = spec["pad"]

    def __len__(self):
        return (len(self.names) + self.batch - 1) // self.batch

    def _host(self, idx):
        names = [self.names[i] for i in idx]
        if self._device_synth:  # images are gathered on the GPU in _to_device
            return names, torch.from_numpy(self.labels[idx])
        return self.source.load(names), torch.from_numpy(self.labels[idx])

    @property
    def _device_synth(self) -> bool:
        return self.device.type == "cuda" and isinstance(self.source, SyntheticImages)

    def _to_device(self, imgs, labels):
        cuda = self.device.type == "cuda"
        if self._device_synth:
            imgs = self.source.load_device(imgs, self.device)
            x = Fn.preprocess(imgs, self.out_hw, IMAGENET_MEAN, IMAGENET_STD, self.mode,
                              self.cpad, out_dtype=torch.float32, pad=self.pad)
            return x, labels.to(self.device, non_blocking=True)
        ext = None
        if not isinstance(imgs, np.ndarray):
            # decoded JPEGs of different sizes: one padded batch with per-image extents,
            # so ONE pinned H2D copy and ONE preprocess launch per batch
            from .eval_pipeline import pad_batch
            imgs, ext = pad_batch(imgs)
        g = torch.from_numpy(imgs)
        if cuda:
            g = g.pin_memory().to(self.device, non_blocking=True)
        x = Fn.preprocess(g, self.out_hw, IMAGENET_MEAN, IMAGENET_STD, self.mode, self.cpad,
                          out_dtype=torch.float32, pad=self.pad, extents=ext)
        y = labels.to(self.device, non_blocking=cuda)
        return x, y

    def epoch(self, e: int, steps: Optional[int] = None):
        order = np.arange(len(self.names))
        if self.shuffle:
            np.random.default_rng(self.seed * 7919 + e).shuffle(order)
        n = len(self)
        if steps is not None:
            n = min(n, steps)
        chunks = [order[i * self.batch:(i + 1) * self.batch] for i in range(n)]
        fut = self.pool.submit(self._host, chunks[0]) if chunks else None
        for i in range(len(chunks)):
            imgs, labels = fut.result()
            if i + 1 < len(chunks):
                fut = self.pool.submit(self._host, chunks[i + 1])
            yield self._to_device(imgs, labels)


def _image_source(cfg: Config, names: Sequence[str], src_hw):
    if not cfg.synthetic and images_available(cfg.TRAIN_DIR, names):
        return FolderImages(cfg.TRAIN_DIR, cfg.num_workers)
    return SyntheticImages(src_hw)


def run_training(cfg: Config) -> dict:
    world = init_world(cfg.device, cfg.timeout_s, comm_timing=cfg.step_timers)
    rank, size = world.rank, world.world_size
    log = init_logger(rank, cfg.log_file, cfg.log_per_rank_files)
    metrics = MetricsWriter(cfg.metrics_jsonl, rank)
    torch.manual_seed(cfg.seed)
    if rank == 0:
        log.info("Logger Initialized")

    # ---------------------------------------------------------------- manifests
    shards = None
    train_sample = None
    if rank == 0:
        log.info("Reading Training & Testing samples")
        if cfg.synthetic_images > 0 or not os.path.exists(cfg.TEST_CSV):
            n = cfg.synthetic_images or 800
            train_sample = synthetic_manifest(n, cfg.NUM_CLASSES, cfg.seed)
        else:
            train_sample, _test = read_manifests(cfg)
        shards = shard_dataframe(train_sample, size)
    my = scatter_object(shards, root=0)
    log.info("_Files Received: {}".format(len(my)))
    n_total = int(broadcast_object(len(train_sample) if rank == 0 else None))
    steps_per_epoch = equal_step_count(array_split_sizes(n_total, size), cfg.BATCH_SIZE)
    if cfg.max_steps:
        steps_per_epoch = min(steps_per_epoch, cfg.max_steps)

    out_hw = cfg.input_hw
    if cfg.MODEL_NAME == "inception" and min(out_hw) < 299:
        out_hw = (299, 299)  # aux head needs 17x17 Mixed_6e maps
    src_hw = (max(out_hw[0], 2 * out_hw[0]), max(out_hw[1], 2 * out_hw[1]))
    source = _image_source(cfg, list(my["file_name"].values), src_hw)
    dev = world.device
    train_loader = ManifestBatches(my["file_name"].values, my["category_id"].values,
                                   cfg.BATCH_SIZE, out_hw, dev, source, True, cfg.seed + rank)
    log.info("_Training Dataset Object Created")
    log.info("_Training Loader Created")
    val_loader = None
    if rank == 0 and cfg.VALIDATE:
        # reference validates on train_sample (main.py:108), not the test split
        val_loader = ManifestBatches(train_sample["file_name"].values,
                                     train_sample["category_id"].values, cfg.BATCH_SIZE,
                                     out_hw, dev, source, False)
        log.info("_Validation Dataset Object Created")
        log.info("_Validation Loader Created")

    # ------------------------------------------------------------------- model
    if cfg.reserve_gib > 0:
        from .step import reserve_device_memory
        log.debug("reserved {} GiB of device memory".format(
            reserve_device_memory(dev, cfg.reserve_gib)))
    model, opt, step, _input_size = build_training(
        cfg.MODEL_NAME, cfg.NUM_CLASSES, dev, world, cfg.LR, cfg.optimizer, cfg.momentum,
        cfg.weight_decay, cfg.FEATURE_EXTRACT, cfg.bucket_mb, cfg.overlap_comm,
        cfg.grad_comm_dtype, None if cfg.grad_comm_ctas < 0 else cfg.grad_comm_ctas)
    log.info("_Model Created: {}".format(cfg.MODEL_NAME))
    spec = input_spec(model, out_hw)
    for ld in (train_loader, val_loader):
        if ld is not None:
            ld.set_layout(spec)
    log.info("_Optimizer Created")
    start_epoch = 0
    ckpt = os.path.join(cfg.CHECKPOINT_DIR, cfg.CHECKPOINT_NAME)
    if cfg.FROM_CHECKPOINT:
        log.info("_Loading Checkpoint")
        _m, _o, saved_epoch = load_checkpoint(ckpt, model, opt, map_location="cpu")
        start_epoch = saved_epoch + 1 if cfg.resume_epoch else 0
        log.info("_Checkpoint loaded")
    from ..parallel import sync_params
    sync_params(model)
    # the reference's exact string (main.py:133 logs "CPU" whatever the device); the
    # actual compute device goes on a line of its own
    log.info("_Model loaded to CPU")
    log.debug("_Compute device: %s", dev)  # (no such line in the reference)
    log.info("_Entering training Loop")

    if cfg.step_timers:
        step.enable_timers()
        step.bucketer.enable_comm_stats()
    history = []
    use_graph = (cfg.graph == "on" and size == 1 and dev.type == "cuda"
                 and not cfg.step_timers)
    # fail fast on a stalled rank (e.g. a peer died inside a collective): SURVEY.md §5.3
    dog = Watchdog(cfg.watchdog_s, rank=rank).start()
    gstep = 0
    for epoch in range(start_epoch, cfg.NUM_EPOCHS):
        model.train()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        nimg = 0
        with steps_without_gc():  # cyclic GC at the epoch boundary, not mid-step
            for x, y in train_loader.epoch(epoch, steps_per_epoch):
                if use_graph and step._graph is None and x.shape[0] == cfg.BATCH_SIZE:
                    # graph = "on", one GPU: capture the whole step once, replay it after
                    step.capture(x, y)
                step(x, y)
                nimg += x.shape[0]
                gstep += 1
                if dev.type == "cuda":
                    # progress = the step's kernels COMPLETED on the device, not enqueued
                    ev = torch.cuda.Event()
                    ev.record()
                    dog.beat_on(gstep, ev)
                else:
                    dog.beat(gstep)
        tr_loss = step.mean_loss()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dog.beat(gstep)
        dt = time.perf_counter() - t0
        log_rank_lines(log, "_Epoch: {} | Train Loss: {} | Time: {}".format(epoch, tr_loss, dt),
                       rank, size, all_gather_object, cfg.log_per_rank_files)
        rec = {"epoch": epoch, "train_loss": tr_loss, "time_s": dt,
               "img_per_s_rank": nimg / dt if dt > 0 else 0.0,
               "img_per_s_global": nimg * size / dt if dt > 0 else 0.0}
        if step.timer is not None:
            rec["phases_ms"] = step.timer.summary()
        if size > 1:
            rec["grad_allreduce_mb"] = step.bucketer.wire_mb()
            cs = step.bucketer.comm_stats()
            if cs is not None:
                rec["comm"] = cs
        if cfg.checksum_every and size > 1:
            rec["replicas_consistent"] = replica_checksum(model)
        # rank 0 checkpoints and validates while the others wait at the next collective:
        # no rank's deadline runs until everyone is past the epoch-end work
        dog.pause()
        if rank == 0:
            log.info("_Creating a checkpoint at epoch {}".format(epoch))
            save_checkpoint(build_state(epoch, model, opt, tr_loss), epoch, cfg.MODEL_NAME,
                            cfg.CHECKPOINT_DIR, cfg.MODELS_DIR)
            log.info("_Checkpoint saved")
            if val_loader is not None:
                log.info("_Evaluating model")
                acc = evaluate(model, val_loader)
                rec["acc"] = acc
                log.info("_Epoch: {} | Acc: {}".format(epoch, acc))
        metrics.write(**rec)
        history.append(rec)
        if size > 1:
            barrier()
        dog.resume()
    dog.stop()
    return {"history": history, "checkpoint": ckpt}


@torch.no_grad()
def evaluate(model, loader: ManifestBatches) -> float:
    """Rank-0 accuracy over a loader (main.py:173-185)."""
    model.eval()
    dev = loader.device
    count = torch.zeros(1, dtype=torch.int64, device=dev)
    n = 0
    for x, y in loader.epoch(0):
        out = model(x)
        Fn.count_correct(out, y, count)
        n += x.shape[0]
    model.train()
    return float(count.item()) / max(n, 1)
