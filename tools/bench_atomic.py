"""Round-trip latency of device-scope atomics (the cost a dynamic work queue in the
persistent conv kernels would have to hide per tile) against a dependent load.

    python tools/bench_atomic.py [iters]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.ops import _ext

IT = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
C = _ext.ext()
dev = torch.device("cuda", 0)
q = torch.zeros((1 << 20) + 64, dtype=torch.int32, device=dev)
names = {0: "atomic, one counter", 1: "atomic, counter per XCD", 2: "atomic, counter per block",
         3: "dependent load"}
for mode in (0, 1, 2, 3):
    for blocks in (1, 8, 64, 256):
        C.atomic_latency(blocks, 50, mode, q)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        C.atomic_latency(blocks, IT, mode, q)
        e.record()
        torch.cuda.synchronize()
        print("%-26s blocks %3d: %7.3f us per round trip"
              % (names[mode], blocks, s.elapsed_time(e) * 1e3 / IT), flush=True)
