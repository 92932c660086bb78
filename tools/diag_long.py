"""Diagnostic: long ResNet-18 training trajectory on one static batch (memorisation), eager
or HIP graph, printing every loss and flagging the first non-finite value together with
weight / gradient / BN-state magnitudes.  Usage: diag_long.py {eager|graph} steps batch"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.engine import build_training
from mpi_pytorch_amd.parallel import World

mode = sys.argv[1]
S = int(sys.argv[2])
B = int(sys.argv[3])
gpu = torch.device("cuda", 0)
torch.manual_seed(0)
model, opt, step, _ = build_training("resnet18", 64500, gpu, World(), 4e-4)
x = (torch.randn(B, 224, 224, 8, device=gpu) * (torch.arange(8, device=gpu) < 3)).to(torch.bfloat16)
y = torch.randint(0, 64500, (B,), device=gpu)
if mode == "graph":
    step.capture(x, y)
arena = model._mpa_arena
losses = []
for i in range(S):
    l = float(step(x, y))
    losses.append(l)
    if l != l or abs(l) > 100:
        g = arena.grad
        print("NON-FINITE/HUGE at step %d: loss %g |w|max %g |g|max %g nan_g %d" % (
            i, l, float(arena.master.abs().max()), float(g.abs().nan_to_num(0).max()),
            int(torch.isnan(g).sum())))
        for n, p in model.named_parameters():
            if not torch.isfinite(p).all() or not torch.isfinite(p.grad).all():
                print("   bad param", n)
                break
        for n, m in model.named_modules():
            if hasattr(m, "running_var") and not torch.isfinite(m.running_var).all():
                print("   bad running stats", n)
                break
        break
print(mode, "B=%d" % B, " ".join("%.3f" % v for v in losses))
