"""Process-group bring-up: one process per GPU, RCCL (torch backend ``nccl``) over xGMI.

The reference gets its world from ``mpi4py`` at import time (``/root/reference/main.py:1,16-18``,
``mpi_tools.py:1``).  MPI is not available on the MI355X image, so ranks come from the
environment set by our launcher (``python -m mpi_pytorch_amd.launch``), by
``torch.distributed.run`` (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*), or by an MPI launcher
(OMPI_COMM_WORLD_* / PMI_*).  World size 1 needs no process group at all, mirroring the
reference's ``num_processes() == 1`` short-circuits (``mpi_tools.py:32-33,49-50``).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class World:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def is_dist(self) -> bool:
        return self.world_size > 1

    @property
    def is_root(self) -> bool:
        return self.rank == 0


_WORLD: Optional[World] = None


def _env_int(*names: str, default: int = -1) -> int:
    for n in names:
        v = os.environ.get(n)
        if v is not None and v != "":
            return int(v)
    return default


def env_rank_info():
    rank = _env_int("RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "SLURM_PROCID", default=0)
    world = _env_int("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "SLURM_NTASKS", default=1)
    local = _env_int("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID",
                     "SLURM_LOCALID", default=-1)
    if local < 0:
        local = rank
    return rank, world, local


def init_world(device: str = "auto", timeout_s: float = 1800.0,
               backend: Optional[str] = None, comm_timing: bool = False) -> World:
    """Initialise (idempotently) the process group and pick this rank's device.

    ``comm_timing``: have ProcessGroupNCCL record start/end events around every
    collective (``TORCH_NCCL_ENABLE_TIMING``), read back by ``GradBucketer.comm_stats``."""
    if comm_timing:
        os.environ.setdefault("TORCH_NCCL_ENABLE_TIMING", "1")
    global _WORLD
    if _WORLD is not None:
        return _WORLD
    rank, world, local = env_rank_info()
    use_cuda = (device == "cuda") or (device == "auto" and torch.cuda.is_available())
    if use_cuda:
        ndev = torch.cuda.device_count()
        dev = torch.device("cuda", local % max(ndev, 1))
        torch.cuda.set_device(dev)
        if world > 1:
            pin_host_to_gpu(dev)
    else:
        dev = torch.device("cpu")
    be = "none"
    if world > 1:
        be = backend or os.environ.get("MPA_DIST_BACKEND") or ("nccl" if use_cuda else "gloo")
        # RCCL communicator errors / timeouts raise in the rank that sees them (and tear the
        # communicator down) instead of leaving the job hung; see parallel/watchdog.py
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        if not dist.is_initialized():
            kw = dict(backend=be, rank=rank, world_size=world,
                      timeout=datetime.timedelta(seconds=timeout_s))
            if be == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(**kw)
        if use_cuda:
            # the GEMM tuner then syncs only its own stream: a device drain would also wait
            # for the first step's overlapped all-reduces (csrc/kernels/igemm.hip)
            from ..ops import _ext
            if _ext.available():
                _ext.ext().igemm_set_tune_drain(0)
    _WORLD = World(rank=rank, world_size=world, local_rank=local, device=dev, backend=be)
    return _WORLD


_AFFINITY: Optional[dict] = None


def _pci_addr(dev: torch.device) -> Optional[str]:
    """PCI address ("dddd:bb:dd.f") of a HIP device, or None if torch does not report it."""
    try:
        pr = torch.cuda.get_device_properties(dev)
        dom = int(getattr(pr, "pci_domain_id", 0))
        bus = int(getattr(pr, "pci_bus_id"))
        slot = int(getattr(pr, "pci_device_id"))
    except Exception:
        return None
    return "%04x:%02x:%02x.0" % (dom, bus, slot)


def parse_cpulist(text: str) -> set:
    """Linux cpulist ("0-3,8,10-11") -> {0,1,2,3,8,10,11}."""
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            cpus.update(range(int(a), int(b) + 1))
        else:
            cpus.add(int(part))
    return cpus


def pin_host_to_gpu(dev: torch.device, sysfs: str = "/sys/bus/pci/devices",
                    addr: Optional[str] = None) -> Optional[dict]:
    """Restrict this rank's host threads (the caller and every thread started afterwards:
    batch producers, copy hand-off) to the CPUs of its GPU's NUMA node, read from the
    device's PCI ``local_cpulist``.  One process per GPU on a two-socket node otherwise lets
    the scheduler place a rank's producers on the far socket, so its pinned ring slots and
    H2D copies cross the inter-socket link.  Kept within the CPUs the process may already
    use (container / cgroup limits); a no-op when sysfs does not say.  Opt-in (MPA_NUMA_PIN=1)
    until an 8-GPU run measures it: several ranks share a node's CPUs, and each torch
    intra-op pool is still sized for the whole machine (the pool is capped below).
    Returns {"pci", "numa_node", "cpus"} or None."""
    global _AFFINITY
    if os.environ.get("MPA_NUMA_PIN", "0") != "1" or not hasattr(os, "sched_setaffinity"):
        return None
    addr = addr or _pci_addr(dev)
    if addr is None:
        return None
    base = os.path.join(sysfs, addr)
    try:
        with open(os.path.join(base, "local_cpulist")) as f:
            local = parse_cpulist(f.read())
        node = -1
        try:
            with open(os.path.join(base, "numa_node")) as f:
                node = int(f.read().strip())
        except OSError:
            pass
        allowed = os.sched_getaffinity(0)
    except (OSError, ValueError):
        return None
    cpus = local & allowed
    if not cpus or cpus == allowed:
        return None
    try:
        os.sched_setaffinity(0, cpus)
    except OSError:
        return None
    # the ranks of this node that share the pinned CPUs split them: cap the intra-op pool
    sharing = max(_env_int("LOCAL_WORLD_SIZE", default=1), 1)
    threads = max(len(cpus) // sharing, 1)
    if torch.get_num_threads() > threads:
        torch.set_num_threads(threads)
    _AFFINITY = {"pci": addr, "numa_node": node, "cpus": len(cpus), "threads": threads}
    return _AFFINITY


def affinity() -> Optional[dict]:
    """What :func:`pin_host_to_gpu` did for this rank (None: not pinned)."""
    return _AFFINITY


def get_world() -> World:
    return _WORLD if _WORLD is not None else init_world()


def shutdown() -> None:
    global _WORLD
    if dist.is_available() and dist.is_initialized():
        try:
            dist.barrier()
        except Exception:
            pass
        dist.destroy_process_group()
    _WORLD = None


def barrier() -> None:
    w = get_world()
    if w.is_dist:
        if w.backend == "nccl":
            dist.barrier(device_ids=[w.device.index])
        else:
            dist.barrier()
