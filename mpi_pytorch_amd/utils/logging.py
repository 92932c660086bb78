"""Rank-tagged logger with the reference's exact record format.

Reference: ``init_logger`` in ``/root/reference/main.py:22-41`` (and the copy in
``evaluation_pipeline.py:19-41``): logger name ``Herbarium``, format
``'%(levelname)s:%(name)s_R{rank}:%(message)s'``, a stream handler plus an
append-mode ``FileHandler``.  The reference lets every rank append to the same file,
which tears lines; here only the requested ranks write the shared file
and ``per_rank_files=True`` gives each rank its own ``<log>.r<rank>`` file instead.

Every rank's ``_Epoch | Train Loss | Time`` line still reaches the shared file
(``main.py:159-160`` logs it per rank): :func:`log_rank_lines` gathers the lines to rank 0,
which writes each one tagged with its own rank (``INFO:Herbarium_R2:...``), so the per-rank
time skew of SURVEY §3.2 stays visible without torn lines.
"""
from __future__ import annotations

import json
import logging
import os
import time
from typing import Any, Dict, Optional

LOGGER_NAME = "Herbarium"


def init_logger(rank: int = 0, log_file: Optional[str] = "training.log",
                per_rank_files: bool = False, file_ranks=(0,),
                stream: bool = True) -> logging.Logger:
    fmt = logging.Formatter("%(levelname)s:%(name)s_R%(mpa_rank)s:%(message)s")
    logger = logging.getLogger(LOGGER_NAME)
    for f in list(logger.filters):
        logger.removeFilter(f)
    logger.addFilter(_RankTag(rank))
    logger.setLevel(logging.DEBUG)
    logger.propagate = False
    for h in list(logger.handlers):
        logger.removeHandler(h)
        try:
            h.close()
        except Exception:
            pass
    if stream:
        sh = logging.StreamHandler()
        sh.setLevel(logging.DEBUG)
        sh.setFormatter(fmt)
        logger.addHandler(sh)
    if log_file:
        path = None
        if per_rank_files:
            path = "{}.r{}".format(log_file, rank)
        elif file_ranks is None or rank in file_ranks:
            path = log_file
        if path:
            d = os.path.dirname(path)
            if d:
                os.makedirs(d, exist_ok=True)
            fh = logging.FileHandler(path, mode="a")
            fh.setFormatter(fmt)
            logger.addHandler(fh)
    return logger


class _RankTag(logging.Filter):
    """Tags records with this process's rank unless the caller passed ``extra=
    {"mpa_rank": r}`` (a line gathered from rank r)."""

    def __init__(self, rank: int):
        super().__init__()
        self.rank = rank

    def filter(self, record: logging.LogRecord) -> bool:
        if not hasattr(record, "mpa_rank"):
            record.mpa_rank = self.rank
        return True


def log_rank_lines(logger: logging.Logger, msg: str, rank: int, world_size: int,
                   gather=None, per_rank_files: bool = False) -> None:
    """Log ``msg`` for every rank.  Per-rank files: each rank writes its own.  Shared file:
    ``gather(obj) -> list`` (an all-gather over ranks) brings every rank's line to rank 0,
    which logs them in rank order, each with its own rank tag; the other ranks print
    their own line to their stream only (they have no file handler)."""
    if world_size == 1 or per_rank_files or gather is None:
        logger.info(msg)
        return
    lines = gather(msg)
    if rank != 0:
        logger.info(msg)
        return
    for r, m in enumerate(lines):
        logger.info(m, extra={"mpa_rank": r})


def get_logger() -> logging.Logger:
    return logging.getLogger(LOGGER_NAME)


class MetricsWriter:
    """Append-only JSONL metrics stream (one object per line, rank-tagged)."""

    def __init__(self, path: str, rank: int = 0):
        self.path = path
        self.rank = rank
        if path:
            d = os.path.dirname(path)
            if d:
                os.makedirs(d, exist_ok=True)

    def write(self, **rec: Any) -> None:
        if not self.path:
            return
        rec = dict(rec)
        rec.setdefault("ts", time.time())
        rec.setdefault("rank", self.rank)
        with open(self.path, "a") as f:
            f.write(json.dumps(rec, default=float) + "\n")
