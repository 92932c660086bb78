"""RCCL-side checks that fit one GPU: a 1-rank ``nccl`` process group in a child process
(the multi-rank data-parallel path is covered over gloo in test_parallel_cpu.py; RCCL
refuses two ranks on one GPU)."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_capped_rccl_group_and_bucketer():
    """capped_group builds a maxCTAs-capped RCCL communicator that all-reduces correctly,
    and a GradBucketer on it reserves CUs for its overlapped buckets and releases them in
    finish() (world size 1 here, so the bucketer is forced active)."""
    code = textwrap.dedent("""
        import sys, torch, torch.distributed as dist
        sys.path.insert(0, %r)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        from mpi_pytorch_amd.parallel.ddp import capped_group, GradBucketer
        from mpi_pytorch_amd.parallel import ParamArena
        from mpi_pytorch_amd.ops import _ext
        g = capped_group(8, dev)
        assert g is not None
        t = torch.arange(1 << 20, device=dev, dtype=torch.float32)
        dist.all_reduce(t, group=g)
        assert torch.equal(t, torch.arange(1 << 20, device=dev, dtype=torch.float32))
        m = torch.nn.Sequential(torch.nn.Linear(512, 4096), torch.nn.Linear(4096, 8))
        arena = ParamArena(m, dev)
        b = GradBucketer(arena, 2, bucket_mb=0.1, comm_ctas=8)
        assert b.overlap_group is not None and len(b.buckets) > 1
        arena.grad.fill_(1.0)
        for p in b.buckets[0]:
            arena.notify(p)
        seen = _ext.ext().comm_reserve()
        b.finish()
        torch.cuda.synchronize()
        assert seen == 8 and _ext.ext().comm_reserve() == 0, seen
        assert float(arena.grad.min()) == 1.0 and float(arena.grad.max()) == 1.0
        dist.destroy_process_group()
        print("CAPPED_OK")
    """ % ROOT)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=100)
    assert r.returncode == 0 and "CAPPED_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


def test_tuned_table_roundtrip():
    """The autotuner's table dump loads back (igemm_tuned_load): what a data-parallel rank
    adopts from rank 0 (parallel/comm.py agree_tuned_tiles) is what its lookups then use."""
    import torch
    sys.path.insert(0, ROOT)
    from mpi_pytorch_amd.ops import _ext
    k = _ext.ext()
    before = k.igemm_tuned_table()
    try:
        t = "rows test-key-A -> 64x128\nwgrad test key B -> 128x256\nbroken line\n"
        assert k.igemm_tuned_load(t, True) == 2
        assert k.igemm_tuned_table() == "rows test-key-A -> 64x128\nwgrad test key B -> 128x256\n"
        assert k.igemm_tuned_load("rows test-key-A -> 256x256\n", False) == 1
        assert "rows test-key-A -> 256x256" in k.igemm_tuned_table()
        assert "wgrad test key B -> 128x256" in k.igemm_tuned_table()
    finally:
        k.igemm_tuned_load(before, True)
    assert torch.cuda.is_available()
