"""Data-parallel semantics on CPU with the gloo backend (world size 2, spawned processes).

Checks the reference's DP contract:
* shard sizes follow ``np.array_split`` (main.py:84);
* ``sync_params`` makes replicas identical (mpi_tools.py:47-53);
* averaged gradients over N ranks with B/N images each == single-process gradient over the
  same B images (mpi_tools.py:36) - checked on a BN-free model so per-rank batch
  statistics do not enter;
* the overlapped bucketed all-reduce gives the same result as the post-backward path.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from mpi_pytorch_amd.parallel import array_split_sizes, shard_bounds
from mpi_pytorch_amd.parallel.sharding import equal_step_count, shard_dataframe


def test_array_split_semantics():
    for n in (0, 1, 7, 800, 801, 40000):
        for p in (1, 2, 3, 4, 6, 8):
            ref = [len(a) for a in np.array_split(np.arange(n), p)]
            assert array_split_sizes(n, p) == ref
            b = [shard_bounds(n, p, i) for i in range(p)]
            assert b[0][0] == 0 and b[-1][1] == n
    assert equal_step_count([400, 400], 128) == 4
    assert equal_step_count([267, 267, 266], 128) == 3


def test_shard_dataframe_matches_numpy():
    import pandas as pd
    df = pd.DataFrame({"a": np.arange(803)})
    for p in (2, 3, 4):
        ours = shard_dataframe(df, p)
        ref = np.array_split(df["a"].values, p)
        for s, r in zip(ours, ref):
            assert np.array_equal(s["a"].values, r)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# DenseNet at 64 px: at 32 px its last block runs at 1x1 with BN over 4 samples, where even
# the CPU thread count moves the fp32 gradient by 1 % (shattered gradients, NOTES.md)
_HW = {"alexnet": 95, "densenet": 64, "resnet18": 32}


def _worker(rank, world, port, out_dir, overlap, model="alexnet"):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from mpi_pytorch_amd.parallel import init_world, sync_params, shutdown
    from mpi_pytorch_amd.engine import build_model, loss_fn
    from mpi_pytorch_amd.optim import build_optimizer
    import mpi_pytorch_amd.parallel.dist as D
    D._WORLD = None
    w = init_world("cpu")
    torch.manual_seed(100 + rank)  # different init per rank: sync_params must fix it
    m, _ = build_model(model, 10, False, torch.device("cpu"), w, bucket_mb=8.0,
                       overlap=overlap)
    for mod in m.modules():
        if type(mod).__name__ == "Dropout":
            mod.p = 0.0
    sync_params(m)
    opt = build_optimizer("sgd", m, 0.01, momentum=0.9)
    opt.grad_scale = 1.0 / world
    g = torch.Generator().manual_seed(7)
    X = torch.randn(8, _HW[model], _HW[model], 3, generator=g)
    Y = torch.randint(0, 10, (8,), generator=g)
    per = 8 // world
    xs, ys = X[rank * per:(rank + 1) * per], Y[rank * per:(rank + 1) * per]
    init = m._mpa_arena.master.clone()
    for _ in range(2):
        m._mpa_arena.zero_grad()
        loss_fn(m(xs), ys).backward()
        m._mpa_bucketer.finish()
        grad = m._mpa_arena.grad.clone() * (1.0 / world)
        opt.step()
    torch.save({"init": init, "grad": grad, "final": m._mpa_arena.master.clone()},
               os.path.join(out_dir, "r%d.pt" % rank))
    shutdown()


def _single(out_dir, model="alexnet"):
    from mpi_pytorch_amd.engine import build_model, loss_fn
    from mpi_pytorch_amd.optim import build_optimizer
    from mpi_pytorch_amd.parallel import World
    init = torch.load(os.path.join(out_dir, "r0.pt"))["init"]
    threads = torch.get_num_threads()
    torch.set_num_threads(1)  # the ranks' reduction order
    m, _ = build_model(model, 10, False, torch.device("cpu"), World())
    for mod in m.modules():
        if type(mod).__name__ == "Dropout":
            mod.p = 0.0
    m._mpa_arena.master.copy_(init)
    opt = build_optimizer("sgd", m, 0.01, momentum=0.9)
    g = torch.Generator().manual_seed(7)
    X = torch.randn(8, _HW[model], _HW[model], 3, generator=g)
    Y = torch.randint(0, 10, (8,), generator=g)
    for _ in range(2):
        m._mpa_arena.zero_grad()
        # mean over 8 == average of the two per-rank means over 4
        l0 = loss_fn(m(X[:4]), Y[:4])
        l1 = loss_fn(m(X[4:]), Y[4:])
        ((l0 + l1) / 2).backward()
        grad = m._mpa_arena.grad.clone()
        opt.step()
    torch.set_num_threads(threads)
    return grad, m._mpa_arena.master.clone()


@pytest.mark.parametrize("world,overlap,model", [(2, True, "alexnet"), (2, False, "alexnet"),
                                                 (4, True, "alexnet"), (2, True, "densenet")])
def test_dp_equivalence_gloo(world, overlap, model):
    """DP over gloo == one process on the whole batch (mean of equal-size per-rank means is
    the global mean), with the bucketed overlapped all-reduce; world 4 rehearses more ranks
    than the one-GPU box can hold.  DenseNet: BN per rank (batch statistics of the rank's
    half, as in the reference) and the block-level gradient accumulator under bucketing."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d, overlap, model), nprocs=world,
                           join=True, start_method="spawn")
        rs = [torch.load(os.path.join(d, "r%d.pt" % r)) for r in range(world)]
        r0 = rs[0]
        # broadcast made replicas identical, and they stay identical
        for r in rs[1:]:
            assert torch.equal(r0["init"], r["init"])
            assert torch.equal(r0["final"], r["final"])
        grad, final = _single(d, model)
        assert torch.allclose(r0["grad"], grad, atol=1e-5, rtol=1e-4)
        assert torch.allclose(r0["final"], final, atol=1e-5, rtol=1e-4)


def test_watchdog_fires_on_stall_and_not_while_beating():
    import time
    from mpi_pytorch_amd.parallel.watchdog import Watchdog
    hits = []
    dog = Watchdog(0.3, rank=3, on_timeout=hits.append, poll_s=0.02).start()
    for i in range(10):  # steady progress: never fires
        time.sleep(0.05)
        dog.beat(i)
    assert not hits
    time.sleep(0.6)  # stall
    assert hits and "rank 3" in hits[0] and "last completed step 9" in hits[0]
    dog.stop()


def test_watchdog_exits_process_with_stall_code():
    """A stalled rank terminates with EXIT_STALLED and a stack dump (fail fast)."""
    import subprocess
    import sys
    code = ("import time\n"
            "from mpi_pytorch_amd.parallel.watchdog import Watchdog\n"
            "Watchdog(0.2, rank=1, poll_s=0.02).start()\n"
            "time.sleep(30)\n")
    root = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                       cwd=root)
    assert r.returncode == 75, (r.returncode, r.stderr[-500:])
    assert "rank 1: no train progress" in r.stderr and "Thread" in r.stderr


def test_bucket_layout_resnet18():
    """GradBucketer on ResNet-18 @64,500: the classifier is bucket 0 (produced first, reduced
    under the whole conv backward), buckets tile the gradient arena contiguously, and the
    stem's parameters (their gradients land last, after the pool / BN / stem-wgrad backward)
    form a tiny final bucket, so layer2..layer1 launch before that stem backward."""
    from mpi_pytorch_amd.engine import build_model
    from mpi_pytorch_amd.parallel import World
    from mpi_pytorch_amd.parallel.ddp import GradBucketer
    m, _ = build_model("resnet18", 64500, False, torch.device("cpu"), World())
    a = m._mpa_arena
    b = GradBucketer(a, 2, 16.0)
    names = [[a.names[id(p)] for p in ps] for ps in b.buckets]
    assert names[0] == ["fc.bias", "fc.weight"]
    assert names[-1] == ["bn1.bias", "bn1.weight", "conv1.weight"]
    assert b.describe()[-1]["bytes"] < 128 * 1024
    assert "layer1.0.conv1.weight" in names[-2]
    assert b.ranges[0][0] == 0 and b.ranges[-1][1] == a.n_train
    assert all(b.ranges[i][1] == b.ranges[i + 1][0] for i in range(len(b.ranges) - 1))
    assert sum(len(ps) for ps in b.buckets) == len(a.trainable)


def test_numa_pin_from_sysfs(tmp_path):
    """pin_host_to_gpu restricts the process to its GPU's local CPUs (sysfs local_cpulist),
    within the CPUs it may already use, and restores nothing else; unknown devices are a
    no-op."""
    import os as _os
    from mpi_pytorch_amd.parallel import dist as D
    assert D.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    allowed = _os.sched_getaffinity(0)
    if len(allowed) < 2:
        pytest.skip("needs two CPUs")
    keep = sorted(allowed)[: len(allowed) // 2]
    dev = tmp_path / "0000:c1:00.0"
    dev.mkdir()
    (dev / "local_cpulist").write_text(",".join(str(c) for c in keep) + "\n")
    (dev / "numa_node").write_text("1\n")
    import torch
    nthr = torch.get_num_threads()
    assert D.pin_host_to_gpu(None, sysfs=str(tmp_path), addr="0000:c1:00.0") is None  # opt-in
    _os.environ["MPA_NUMA_PIN"] = "1"
    try:
        info = D.pin_host_to_gpu(None, sysfs=str(tmp_path), addr="0000:c1:00.0")
        assert {k: info[k] for k in ("pci", "numa_node", "cpus")} == \
            {"pci": "0000:c1:00.0", "numa_node": 1, "cpus": len(keep)}
        assert torch.get_num_threads() <= max(len(keep), 1)
        assert _os.sched_getaffinity(0) == set(keep)
        assert D.pin_host_to_gpu(None, sysfs=str(tmp_path), addr="0000:c2:00.0") is None
    finally:
        _os.environ.pop("MPA_NUMA_PIN", None)
        _os.sched_setaffinity(0, allowed)
        torch.set_num_threads(nthr)


def _tune_worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from mpi_pytorch_amd.parallel import init_world, agree_tuned_tiles, shutdown
    init_world("cpu")
    # each rank "tuned" its own tiles for the same shapes (what timing noise does)
    table = {"rows M4096 N64 K576": "%dx128" % (64 * (rank + 1)),
             "wgrad K64 N576 P4096": "%dx256" % (128 if rank else 64)}
    state = {"t": "".join("%s -> %s\n" % kv for kv in sorted(table.items()))}

    def load(t):
        state["t"] = t
    agreed = agree_tuned_tiles(get=lambda: state["t"], load=load)
    with open(os.path.join(out_dir, "tiles%d.txt" % rank), "w") as f:
        f.write(state["t"])
    assert agreed == state["t"]
    shutdown()


def test_agree_tuned_tiles_two_ranks():
    """Data-parallel ranks adopt rank 0's autotuned GEMM tiles (parallel/comm.py
    agree_tuned_tiles, called by TrainStep after the first step of each batch shape), so
    every rank runs identical kernels."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_tune_worker, args=(2, _free_port(), d), nprocs=2, join=True,
                           start_method="spawn")
        t0 = open(os.path.join(d, "tiles0.txt")).read()
        t1 = open(os.path.join(d, "tiles1.txt")).read()
    assert t0 == t1 and "64x128" in t0 and "64x256" in t0
