"""Diagnostic: ResNet-18 loss trajectory on fresh random batches (eager), printing per-step
loss and the BN running stats magnitude.  Usage: python tools/diag_traj.py [batch] [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.engine import build_training
from mpi_pytorch_amd.parallel import World

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
S = int(sys.argv[2]) if len(sys.argv) > 2 else 25
gpu = torch.device("cuda", 0)
torch.manual_seed(0)
model, opt, step, _ = build_training("resnet18", 64500, gpu, World(), 4e-4)
out = []
for i in range(S):
    x = (torch.randn(B, 224, 224, 8, device=gpu) * (torch.arange(8, device=gpu) < 3)).to(torch.bfloat16)
    y = torch.randint(0, 64500, (B,), device=gpu)
    loss = float(step(x, y))
    out.append(loss)
    if i in (0, 1, 2, 5, 10, S - 1):
        rm = max(float(m.running_mean.abs().max()) for m in model.modules() if hasattr(m, "running_mean"))
        rv = max(float(m.running_var.max()) for m in model.modules() if hasattr(m, "running_var"))
        print("step %d loss %.4f  max|running_mean| %.3g  max running_var %.3g" % (i, loss, rm, rv))
print("traj:", " ".join("%.2f" % v for v in out))
