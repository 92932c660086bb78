"""Two data-parallel ranks on the one-GPU box (gloo carries the gradient buckets between
them; the driver's 8-GPU runs use RCCL over xGMI).  Everything else is the real GPU path:
native kernels, the flat arena, bucketed all-reduce launched from backward, the fused
optimizer and bench.py's own rank spawning.

Reference: ``mpiexec -n 2 python -m mpi4py main.py`` (``/root/reference/README.md:38``)
with per-parameter gradient averaging (``mpi_tools.py:30-37``)."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env.update(MASTER_ADDR="127.0.0.1", MPA_DIST_BACKEND="gloo", PYTHONPATH=ROOT, **kw)
    return env


def test_bench_two_ranks_one_gpu(gpu, tmp_path):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch", "32",
           "--image-size", "64", "--classes", "1000", "--steps", "3", "--warmup", "1",
           "--small-batch", "0"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=_env(), capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    # the headline line, then the complete record with the multi-GPU decision extras
    assert len(lines) == 2, r.stdout
    head, rec = json.loads(lines[0]), json.loads(lines[1])
    assert head["value"] == rec["value"] and "multi_gpu" in rec
    assert rec["n_gpus"] == 2 and rec["config"]["backend"] == "gloo"
    assert rec["config"]["parallelism"] == "dp2" and rec["dtype"] == "bf16"
    assert rec["comm"]["timed"] and all(b["calls"] == 3 for b in rec["comm"]["buckets"])
    assert 0 < rec["config"]["mean_loss"] < 10
    assert rec["phases_ms"]["backward"] > 0


_WORKER = r'''
import os, sys, torch
sys.path.insert(0, os.environ["PYTHONPATH"])
from mpi_pytorch_amd.parallel import init_world, shutdown
from mpi_pytorch_amd.engine import build_training
from mpi_pytorch_amd.ops import _ext
_ext.ext().set_deterministic(1)
w = init_world("cuda")
torch.manual_seed(0)
model, opt, step, _ = build_training("resnet18", 100, w.device, w, 1e-2, "sgd")
g = torch.Generator().manual_seed(5)
X = (torch.randn(32, 64, 64, 8, generator=g) * (torch.arange(8) < 3)).to(torch.bfloat16)
Y = torch.randint(0, 100, (32,), generator=g)
n = 32 // w.world_size
x = X[w.rank * n:(w.rank + 1) * n].to(w.device)
y = Y[w.rank * n:(w.rank + 1) * n].to(w.device)
step(x, y)
torch.cuda.synchronize()
from mpi_pytorch_amd.ops import functional as Fn
if os.environ.get("MPA_WGRAD_STREAM_DDP") == "1":
    assert Fn._SIDE["stream"] is not None and step.bucketer._launch_stream is not None
if w.rank == 0:
    torch.save({"master": model._mpa_arena.master.cpu()}, sys.argv[1])
shutdown()
'''


@pytest.mark.parametrize("wgs", ["0", "1"])
def test_dp_two_ranks_equals_one_rank_on_gpu(gpu, tmp_path, wgs):
    """2 ranks x 16 images: BN takes per-rank batch statistics (as in the reference), so DP
    equals one process stepping on the AVERAGE of the two halves' gradients, computed here
    with the same kernels (two backward passes accumulating in the arena, grad_scale 1/2).
    One SGD step (Adam's first step is sign-like and would amplify rounding-level
    differences of near-zero gradients), deterministic mode.  wgs=1: the ranks' conv weight
    gradients on the side stream, each bucket's collective issued from a stream that waits
    for both (MPA_WGRAD_STREAM_DDP)."""
    script = tmp_path / "w.py"
    script.write_text(_WORKER)
    out = tmp_path / "dp.pt"
    cmd = [sys.executable, "-m", "mpi_pytorch_amd.launch", "-n", "2", "--timeout", "200",
           str(script), str(out)]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=_env(MPA_WGRAD_STREAM_DDP=wgs),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    dp = torch.load(str(out))["master"]
    # one process: gradients of the two halves summed in the arena (two backward passes,
    # the second accumulating), averaged by the optimizer's grad_scale, one SGD step
    from mpi_pytorch_amd.engine import build_training, loss_fn
    from mpi_pytorch_amd.parallel import World
    from mpi_pytorch_amd.ops import _ext
    _ext.ext().set_deterministic(1)
    try:
        torch.manual_seed(0)
        model, opt, step, _ = build_training("resnet18", 100, gpu, World(device=gpu), 1e-2,
                                             "sgd")
        g = torch.Generator().manual_seed(5)
        X = (torch.randn(32, 64, 64, 8, generator=g) * (torch.arange(8) < 3)).to(torch.bfloat16)
        Y = torch.randint(0, 100, (32,), generator=g)
        # each half's forward must see the BN running stats a rank sees (the initial ones):
        # the conv epilogues take the batch statistics around the running mean, and these
        # nets' gradients are shattered enough that a rounding-level change of the second
        # half's forward moves its gradient by ~1 % (docs/NOTES.md "Numerics")
        bn0 = {k: v.clone() for k, v in model.state_dict().items()
               if "running" in k or "num_batches" in k}
        model._mpa_arena.zero_grad()
        for h in range(2):
            model.load_state_dict(bn0, strict=False)
            loss_fn(model(X[16 * h:16 * (h + 1)].to(gpu)), Y[16 * h:16 * (h + 1)].to(gpu)).backward()
        opt.grad_scale = 0.5
        opt.step()
        torch.cuda.synchronize()
        ref = model._mpa_arena.master.cpu()
    finally:
        _ext.ext().set_deterministic(0)
    d = (dp - ref).abs()
    assert float(d.max()) < 1e-6 * max(1.0, float(ref.abs().max())) + 1e-7, float(d.max())
