"""Diagnostic: replay HIP graphs of (a) forward, (b) forward+backward, (c) full step of
ResNet-18 back-to-back with FIXED weights and input; every replay must give (nearly) the
same loss.  Reports min/max/NaN count per variant."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.engine import build_model, loss_fn
from mpi_pytorch_amd.parallel import World

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
R = int(sys.argv[2]) if len(sys.argv) > 2 else 40
gpu = torch.device("cuda", 0)
torch.manual_seed(0)
model, _ = build_model("resnet18", 64500, False, gpu, World())
x = (torch.randn(B, 224, 224, 8, device=gpu) * (torch.arange(8, device=gpu) < 3)).to(torch.bfloat16)
y = torch.randint(0, 64500, (B,), device=gpu)
arena = model._mpa_arena
bn_state = {k: v.clone() for k, v in model.state_dict().items() if "running" in k or "num_b" in k}


def restore():
    model.load_state_dict(bn_state, strict=False)


def fwd():
    return loss_fn(model(x), y).detach()


def fwdbwd():
    arena.zero_grad()
    loss = loss_fn(model(x), y)
    loss.backward()
    return loss.detach() + 0.0 * arena.grad[:1].sum()


for name, fn in (("fwd", fwd), ("fwdbwd", fwdbwd)):
    restore()
    eager = [float(fn()) for _ in range(3)]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    vals = torch.zeros(R, device=gpu)
    gn = torch.zeros(R, device=gpu)
    for i in range(R):
        g.replay()
        vals[i] = out
        if name == "fwdbwd":
            gn[i] = arena.grad.norm()
    torch.cuda.synchronize()
    v = vals.cpu()
    print("%-7s eager %s | graph min %.5f max %.5f nan %d | gradnorm min %.4g max %.4g" % (
        name, ["%.5f" % e for e in eager], float(v.min()), float(v.max()),
        int(torch.isnan(v).sum()), float(gn.min()), float(gn.max())), flush=True)
    del g
