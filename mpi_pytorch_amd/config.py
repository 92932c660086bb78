"""Typed run configuration.

The reference keeps every tunable as a hand-edited module constant in ``utils.py``
(``/root/reference/utils.py:4-45``) with no CLI or environment overrides.  This module
keeps the *same field names* (so ``cfg.MODEL_NAME``, ``cfg.BATCH_SIZE`` ... read exactly
like the reference) and adds:

* CLI overrides (``--MODEL_NAME resnet34`` or ``--model-name resnet34``),
* environment overrides (``MPA_MODEL_NAME=resnet34``),
* MI355X fields the reference does not have: ``dtype``, ``bucket_mb``, ``synthetic``,
  ``image_size``, ``optimizer``, ``momentum``, ``per_gpu_batch``, ``backend`` ...

Precedence: defaults < environment < explicit kwargs/CLI.
"""
from __future__ import annotations

import argparse
import dataclasses
import os
from dataclasses import dataclass, field, fields
from typing import Any, Dict, List, Optional

MODEL_NAMES = ("resnet18", "resnet34", "alexnet", "vgg", "vgg16", "squeezenet",
               "densenet", "inception")

_ENV_PREFIX = "MPA_"


@dataclass
class Config:
    # ---- reference fields (utils.py:4-45) -------------------------------------------
    MODEL_NAME: str = "resnet18"           # utils.py:4
    FROM_CHECKPOINT: bool = False          # utils.py:5
    VALIDATE: bool = True                  # utils.py:6
    CHECKPOINT_NAME: str = ""              # utils.py:7 (derived from MODEL_NAME if empty)
    DEBUG: bool = True                     # utils.py:13
    N_IMAGES: int = 50000                  # utils.py:14
    TRAIN_DIR: str = "./data/train/"       # utils.py:22
    TRAIN_FILE: str = "metadata.json"      # utils.py:23
    TEST_DIR: str = "./data/test/"         # utils.py:24
    CHECKPOINT_DIR: str = "./checkpoints/"  # utils.py:26
    MODELS_DIR: str = "./models/"          # utils.py:27
    WIDTH: int = 128                       # utils.py:33
    HEIGHT: int = 128                      # utils.py:34
    NUM_CLASSES: int = 64500               # utils.py:39
    BATCH_SIZE: int = 128                  # utils.py:40 (per rank)
    LR: float = 4e-4                       # utils.py:41
    NUM_EPOCHS: int = 10                   # utils.py:42
    FEATURE_EXTRACT: bool = False          # utils.py:43
    USE_PRETRAINED: bool = False           # utils.py:45 (no hub download offline)

    # ---- manifest paths (hard-coded in the reference: main.py:77,81-82) ----------------
    TRAIN_CSV: str = "./data/train_sample.csv"
    TEST_CSV: str = "./data/test_sample.csv"
    DEBUG_SAMPLE: int = 1000               # main.py:78 sample(1000, random_state=0)

    # ---- new fields --------------------------------------------------------------------
    device: str = "auto"                   # auto | cuda | cpu
    dtype: str = "bf16"                    # compute dtype on GPU (bf16); CPU always fp32
    synthetic: bool = True                 # synthetic images (no Herbarium data offline)
    synthetic_images: int = 0              # images per epoch in synthetic mode (0 => 800 like DEBUG)
    image_size: int = 0                    # 0 => use WIDTH/HEIGHT
    optimizer: str = "adam"                # adam | sgd
    momentum: float = 0.9
    weight_decay: float = 0.0
    bucket_mb: float = 16.0                # gradient all-reduce bucket size (MiB)
    grad_comm_dtype: str = "fp32"          # fp32 | bf16 (wire dtype of the gradient all-reduce)
    overlap_comm: bool = True              # launch bucket all-reduce during backward
    grad_comm_ctas: int = -1               # >0: overlapped buckets on a CTA-capped RCCL
                                           # communicator + comm-aware persistent conv grids
                                           # (0 off; -1: MPA_COMM_CTAS or the default)
    resume_epoch: bool = True              # honour saved epoch (reference restarts at 0: main.py:142)
    graph: str = "auto"                    # auto | on | off : HIP-graph capture of the train step
    seed: int = 0
    log_file: str = "training.log"
    log_per_rank_files: bool = False       # reference appends all ranks to one file (main.py:32)
    metrics_jsonl: str = ""                # machine-readable per-epoch metrics
    step_timers: bool = False              # per-phase HIP-event step times in the metrics
    num_workers: int = 2                   # native decode/prefetch threads
    eval_lanes: int = 1                    # predictor lanes in the eval pipeline
    eval_batch: int = 64
    eval_assign: str = "random"            # random (reference) | roundrobin
    eval_src: int = 0                      # synthetic eval source side (0: the model input size)
    max_steps: int = 0                     # stop an epoch early (0 = full epoch)
    checksum_every: int = 0                # cross-rank replica checksum period (steps, 0=off)
    timeout_s: float = 1800.0              # rendezvous/collective timeout
    watchdog_s: float = 900.0              # abort a rank with no step progress (0: off)
    reserve_gib: float = 0.0               # grow the allocator by one segment up front
                                           # (engine.reserve_device_memory; NOTES "Slow processes")

    def __post_init__(self) -> None:
        if not self.CHECKPOINT_NAME:
            self.CHECKPOINT_NAME = "checkpoint_{}.pt".format(self.MODEL_NAME)
        if self.MODEL_NAME not in MODEL_NAMES:
            raise ValueError("Invalid model name {!r}; expected one of {}".format(
                self.MODEL_NAME, MODEL_NAMES))
        if self.optimizer not in ("adam", "sgd"):
            raise ValueError("optimizer must be adam|sgd")

    # -----------------------------------------------------------------------------------
    @property
    def input_hw(self):
        if self.image_size:
            return (self.image_size, self.image_size)
        return (self.HEIGHT, self.WIDTH)

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    @classmethod
    def from_env(cls, **overrides) -> "Config":
        kw: Dict[str, Any] = {}
        for f in fields(cls):
            for key in (_ENV_PREFIX + f.name, _ENV_PREFIX + f.name.upper()):
                if key in os.environ:
                    kw[f.name] = _coerce(f.type, os.environ[key])
                    break
        kw.update(overrides)
        return cls(**kw)

    @classmethod
    def add_arguments(cls, p: argparse.ArgumentParser) -> None:
        for f in fields(cls):
            names = ["--" + f.name]
            alt = "--" + f.name.lower().replace("_", "-")
            if alt != names[0]:
                names.append(alt)
            p.add_argument(*names, dest=f.name, default=None, type=str,
                           help="(default: {})".format(f.default))

    @classmethod
    def from_args(cls, argv: Optional[List[str]] = None, **defaults) -> "Config":
        """Config from command-line flags; ``defaults`` are entry-point defaults (e.g.
        ``log_file="evaluation.log"``) that explicit flags override."""
        p = argparse.ArgumentParser(add_help=True)
        cls.add_arguments(p)
        ns, _unknown = p.parse_known_args(argv)
        kw = {}
        types = {f.name: f.type for f in fields(cls)}
        for k, v in vars(ns).items():
            if v is not None:
                kw[k] = _coerce(types[k], v)
        for k, v in defaults.items():
            kw.setdefault(k, v)
        return cls.from_env(**kw)


def _coerce(tp: Any, value: Any) -> Any:
    if not isinstance(value, str):
        return value
    t = tp if isinstance(tp, str) else getattr(tp, "__name__", str(tp))
    if t == "bool":
        return value.strip().lower() in ("1", "true", "yes", "on", "y")
    if t == "int":
        return int(float(value))
    if t == "float":
        return float(value)
    return value
