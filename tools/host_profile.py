"""Host-side cost of an eager training step: cProfile over N steps of a model on one GPU
(synthetic bf16 NHWC batch already on the device, so only the Python dispatch of the step
itself is measured), plus the per-step host enqueue time against the GPU step time.

    python tools/host_profile.py densenet 224 256 [steps=5] [top=40]

If the host enqueue time per step is close to the synchronized step time, the step is
host-bound and kernel work cannot make it faster.
"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.engine import build_training
from mpi_pytorch_amd.parallel import World


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "densenet"
    hw = int(sys.argv[2]) if len(sys.argv) > 2 else 224
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    top = int(sys.argv[5]) if len(sys.argv) > 5 else 40
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model, opt, step, _ = build_training(name, 64500, dev, World(device=dev), 4e-4)
    x = (torch.randn(B, hw, hw, 8, device=dev) * (torch.arange(8, device=dev) < 3)).to(
        torch.bfloat16)
    y = torch.randint(0, 64500, (B,), device=dev)
    for _ in range(3):
        step(x, y)
    torch.cuda.synchronize()
    # enqueue time per step (the host may run ahead of the GPU by a few steps)
    t0 = time.perf_counter()
    host = []
    for _ in range(n):
        h0 = time.perf_counter()
        step(x, y)
        host.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n
    print(f"{name} {hw}px b{B}: synchronized step {wall * 1e3:.2f} ms, host enqueue "
          f"{sum(host) / n * 1e3:.2f} ms/step (min {min(host) * 1e3:.2f})", flush=True)
    # backward nodes normally run on autograd's device thread, which cProfile does not
    # see: run them on this thread for the profile
    torch.autograd.set_multithreading_enabled(False)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        step(x, y)
    torch.cuda.synchronize()
    pr.disable()
    torch.autograd.set_multithreading_enabled(True)
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(top)


if __name__ == "__main__":
    main()
