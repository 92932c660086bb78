"""Tile / split sweep of the pixel-pair stem GEMMs (ResNet-18 7x7/s2 stem run as a stride-1
conv over 8-channel pixel pairs, see models/layers.py Conv2d) at the bench batch.

    python tools/stem_sweep.py [batch] [iters]

Prints the forward (with the BN-statistics epilogue, as training runs it) per forced rows
tile and the weight gradient per forced (tile, splits); `auto` is the planner's choice."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.ops import _ext

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
IT = int(sys.argv[2]) if len(sys.argv) > 2 else 10
C = _ext.ext()
dev = torch.device("cuda", 0)


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
    return s.elapsed_time(e) / IT * 1e3  # us


# canvas 230 x 230 x 4 channels = 230 x 115 pixel pairs x 8; weight [64][7][4][8]
x = (torch.randn(B, 230, 115, 8, device=dev) * 0.5).to(torch.bfloat16)
w = (torch.randn(64, 7, 4, 8, device=dev) * 0.05).to(torch.bfloat16)
e = torch.empty(0, device=dev)
stats = torch.empty(2, 64, device=dev)
shift = torch.zeros(64, device=dev)
y = C.conv_fwd(x, w, e, 2, 1, 0, 0, False, stats, shift)
assert tuple(y.shape) == (B, 112, 112, 64), y.shape
flop = 2.0 * y.numel() * 7 * 4 * 8
dy = (torch.randn_like(y.float()) * 0.1).to(torch.bfloat16)
dw = torch.zeros(64, 7, 4, 8, device=dev)
print("stem pixel-pair, batch %d: output %s, %.1f GFLOP per pass" % (B, tuple(y.shape), flop / 1e9))
for bm, bn in [(0, 0), (128, 64), (256, 64), (128, 32), (128, 128)]:
    C.igemm_force_tile(bm, bn, 0)
    t = timeit(lambda: C.conv_fwd(x, w, e, 2, 1, 0, 0, False, stats, shift))
    print("fwd   %-8s %7.1f us  %5.0f TF/s" % ("auto" if not bm else "%dx%d" % (bm, bn), t,
                                               flop / t * 1e-6))
C.igemm_force_tile(0, 0, 0)
t = timeit(lambda: C.conv_fwd(x, w, e, 2, 1, 0, 0, False, e, e))
print("fwd   auto, no BN-statistics epilogue  %7.1f us" % t)
t = timeit(lambda: y.zero_())
print("write-only reference: zero_() of the %.0f MB output  %7.1f us (%.2f TB/s)" % (
    y.numel() * 2 / 1e6, t, y.numel() * 2 / t * 1e-6))
for bm, bn, sp in [(0, 0, 0), (64, 256, 256), (64, 256, 1024), (64, 256, 2048), (64, 128, 0),
                   (64, 128, 512), (64, 128, 1024), (64, 128, 1536), (64, 128, 2048), (128, 256, 0)]:
    C.igemm_force_tile(bm, bn, sp)
    t = timeit(lambda: C.conv_wgrad(dy, x, dw, 2, 1, 0, 0))
    print("wgrad %-14s %7.1f us  %5.0f TF/s" % ("auto" if not bm else "%dx%d/s%d" % (bm, bn, sp),
                                                 t, flop / t * 1e-6))
C.igemm_force_tile(0, 0, 0)
t = timeit(lambda: C.conv_wgrad(dy, x, dw, 2, 1, 0, 0))
print("wgrad auto (again, after the forced tiles)  %7.1f us  %5.0f TF/s" % (t, flop / t * 1e-6))
