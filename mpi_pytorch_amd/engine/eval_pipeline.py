"""Pipelined inference: read -> resize -> normalize -> predict as HIP-stream stages.

Reference (``/root/reference/evaluation_pipeline.py:44-199``): an MPMD job with one MPI
rank per stage - rank 0 decodes images and sends pickled PIL images (~2 MB each) to rank
1, which resizes (PIL bicubic+antialias, :89) and sends to rank 2, which runs
ToTensor+Normalize (:116-122) and sends 3x128x128 fp32 tensors to one of the predictor
ranks 3..N-1 chosen uniformly at random per image (:178); predictors run batch-1 forward
passes from the checkpoint (:132-159); the per-predictor ``corrects / dataset_size`` are
SUM-reduced to rank 0 (:196) which logs ``Accuracy is ...`` (:199).  Needs >= 4 ranks.

Here, on one MI355X:
  stage 0  read/decode   host threads (PIL decode, or deterministic synthetic pixels) fill
                         batches of uint8 images;
  stage 1  transfer      pinned host -> HBM copy on a copy stream (event-ordered);
  stage 2  resize+norm   the preprocess kernel (bicubic+antialias, mode 1, exactly the
                         eval transform) on a preprocess stream, waiting on stage 1's event;
  stage 3  predict       ``lanes`` predictor lanes, each a HIP stream running a *batched*
                         eval forward + fused argmax/correct-count; each batch goes to a
                         lane chosen at random (reference behaviour) or round-robin.
Stages overlap through events; ring depth bounds the in-flight batches (the end-of-stream
sentinel is simply the end of the batch list).  Accuracy = sum over lanes of
correct_lane / dataset_size, like the reference's reduce.  With several GPUs each rank
takes an ``array_split`` shard and the per-rank partial accuracies are SUM-reduced
(RCCL) - predictor fan-out across GPUs.
"""
from __future__ import annotations

import os
import time
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional

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
        if isinstance(imgs, np.ndarray):
            groups = [torch.from_numpy(imgs)]
        else:
            groups = [torch.from_numpy(np.ascontiguousarray(a))[None] for a in imgs]
        outs = []
        for g in groups:
            if self.cuda:
                g = self._staging(g)
                with torch.cuda.stream(self.copy_stream):
                    gd = g.to(self.device, non_blocking=True)
                    copied = torch.cuda.Event()
                    copied.record(self.copy_stream)
                self._last_slot[1] = copied  # pinned slot free once this copy is done
                self.prep_stream.wait_stream(self.copy_stream)
                with torch.cuda.stream(self.prep_stream):
                    gd.record_stream(self.prep_stream)
                    outs.append(Fn.preprocess(gd, self.out_hw, IMAGENET_MEAN, IMAGENET_STD,
                                              self.mode, self.cpad, pad=self.pad))
            else:
                outs.append(Fn.preprocess(g, self.out_hw, IMAGENET_MEAN, IMAGENET_STD,
                                          self.mode, self.cpad, out_dtype=torch.float32,
                                          pad=self.pad))
        if self.cuda:
            with torch.cuda.stream(self.prep_stream):
                x = outs[0] if len(outs) == 1 else torch.cat(outs, 0)
                ev = torch.cuda.Event()
                ev.record(self.prep_stream)
            return x, ev
        return (outs[0] if len(outs) == 1 else torch.cat(outs, 0)), None

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
        source = SyntheticImages((2 * out_hw[0], 2 * out_hw[1]))
    model = load_predictor(cfg, world.device, ckpt_path)
    pipe = StreamPipeline(model, world.device, out_hw, cfg.eval_lanes, assign=cfg.eval_assign,
                          seed=cfg.seed + world.rank)
    t0 = time.perf_counter()
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
        log.info("_Throughput: {:.1f} img/s ({} images, {} lanes x {} ranks)".format(
            dataset_size / dt if dt > 0 else 0.0, dataset_size, pipe.lanes, world.world_size))
    return float(total) if total is not None else acc_local


@torch.no_grad()
def plain_eval(model, names, labels, batch, source, device, out_hw, mode=1) -> int:
    """Non-pipelined batched evaluation (oracle for the pipeline tests)."""
    correct = torch.zeros(1, dtype=torch.int64, device=device)
    for imgs, lab in _batches(names, labels, batch, source):
        if isinstance(imgs, np.ndarray):
            g = torch.from_numpy(imgs).to(device)
            x = Fn.preprocess(g, out_hw, IMAGENET_MEAN, IMAGENET_STD, mode, 8,
                              out_dtype=torch.float32)
        else:
            x = torch.cat([Fn.preprocess(torch.from_numpy(a)[None].to(device), out_hw,
                                         IMAGENET_MEAN, IMAGENET_STD, mode, 8,
                                         out_dtype=torch.float32) for a in imgs], 0)
        Fn.count_correct(model(x), lab.to(device), correct)
    return int(correct.item())
