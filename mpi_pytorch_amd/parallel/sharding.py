"""Data sharding with ``numpy.array_split`` semantics.

The reference splits the manifest on rank 0 with ``np.array_split(train_sample, size)``
and scatters the pickled shards (``/root/reference/main.py:84,91``).  Shards are
contiguous and differ in size by at most one row (the first ``n % size`` shards get the
extra row).  Because the split is deterministic, ranks can also compute their own bounds
locally from a broadcast row count instead of receiving pickled DataFrames.
"""
from __future__ import annotations

from typing import List, Tuple


def array_split_sizes(n: int, parts: int) -> List[int]:
    q, r = divmod(n, parts)
    return [q + 1 if i < r else q for i in range(parts)]


def shard_bounds(n: int, parts: int, index: int) -> Tuple[int, int]:
    sizes = array_split_sizes(n, parts)
    start = sum(sizes[:index])
    return start, start + sizes[index]


def shard_dataframe(df, parts: int):
    """Same result as ``np.array_split(df, parts)`` without the pandas deprecation path."""
    out = []
    for i in range(parts):
        s, e = shard_bounds(len(df), parts, i)
        out.append(df.iloc[s:e])
    return out


def equal_step_count(n_local: List[int], batch: int) -> int:
    """Steps per epoch every rank can run so collective counts always match.

    The reference can deadlock when shards straddle a multiple of the batch size
    (different batch counts => mismatched Allreduce counts).  All ranks run
    ``min(ceil(n_i / batch))`` steps instead.
    """
    return min((n + batch - 1) // batch for n in n_local) if n_local else 0
