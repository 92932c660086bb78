"""Stem weight-gradient timing at the headline shape (pixel-pair canvas, batch B):
halo-staged stem kernel vs the GEMM plan (MPA_STEM_DIRECT=0 path via igemm_set_stem(0)).

    python tools/bench_stem_wgrad.py [batch] [iters]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.ops import _ext

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
IT = int(sys.argv[2]) if len(sys.argv) > 2 else 10
C = _ext.ext()
dev = torch.device("cuda", 0)
P = Q = 112
x = (torch.randn(B, 2 * (P - 1) + 7, Q + 3, 8, device=dev) * 0.5).to(torch.bfloat16)
dy = (torch.randn(B, P, Q, 64, device=dev) * 0.1).to(torch.bfloat16)
dw = torch.zeros(64, 7, 4, 8, device=dev)


def timeit(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(IT):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / IT * 1e3


fn = lambda: C.conv_wgrad(dy, x, dw, 2, 1, 0, 0)
t1 = timeit(fn)
C.igemm_set_stem(0)
t0 = timeit(fn)
C.igemm_set_stem(1)
gflop = 2.0 * B * P * Q * 64 * 224 / 1e9
print("stem wgrad batch %d: halo kernel %.1f us (%.0f TF)  GEMM plan %.1f us (%.0f TF)" % (
    B, t1, gflop / t1 * 1e3, t0, gflop / t0 * 1e3))
