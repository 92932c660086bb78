"""Rows-GEMM tile sweep on zoo conv shapes (forward and dgrad of the LDS-DMA engine, every
tile forced in turn through igemm_force_tile), against the tile the autotuner picks.

    python tools/bench_tiles.py [set=inception|resnet|densenet] [batch] [iters]

Prints per shape: us (and achieved TF) for each tile, fwd and dgrad.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.ops import _ext

SET = sys.argv[1] if len(sys.argv) > 1 else "inception"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
IT = int(sys.argv[3]) if len(sys.argv) > 3 else 10
C = _ext.ext()
dev = torch.device("cuda", 0)

SHAPES = {  # H, W, Cin, Cout, R, S, stride, pad_h, pad_w
    "inception": [
        (17, 17, 768, 192, 1, 1, 1, 0, 0),
        (17, 17, 192, 192, 1, 7, 1, 0, 3),
        (17, 17, 192, 192, 7, 1, 1, 3, 0),
        (17, 17, 160, 160, 1, 7, 1, 0, 3),
        (35, 35, 288, 64, 1, 1, 1, 0, 0),
        (35, 35, 64, 96, 3, 3, 1, 1, 1),
        (8, 8, 384, 384, 1, 3, 1, 0, 1),
        (8, 8, 2048, 448, 1, 1, 1, 0, 0),
        (73, 73, 80, 192, 3, 3, 1, 0, 0),
    ],
    "resnet": [
        (56, 56, 64, 128, 3, 3, 2, 1, 1),
        (28, 28, 128, 256, 3, 3, 2, 1, 1),
        (14, 14, 256, 512, 3, 3, 2, 1, 1),
        (56, 56, 64, 128, 1, 1, 2, 0, 0),
    ],
    "densenet": [
        (56, 56, 256, 128, 1, 1, 1, 0, 0),
        (28, 28, 512, 128, 1, 1, 1, 0, 0),
        (14, 14, 1024, 128, 1, 1, 1, 0, 0),
        (7, 7, 1024, 128, 1, 1, 1, 0, 0),
    ],
}[SET]
TILES = [(128, 128), (256, 128), (128, 64), (256, 64), (256, 256), (128, 32)]


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


e = torch.empty(0, device=dev)
print("rows tile sweep (%s), batch %d: us [TF]; auto = the autotuned plan" % (SET, B))
for H, W, Ci, Co, R, S, st, ph, pw in SHAPES:
    x = torch.randn(B, H, W, Ci, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, R, S, Ci, device=dev) * 0.05).to(torch.bfloat16)
    wt = w.permute(3, 1, 2, 0).reshape(Ci, R * S, Co).contiguous()
    P = (H + 2 * ph - R) // st + 1
    Q = (W + 2 * pw - S) // st + 1
    dy = torch.randn(B, P, Q, Co, device=dev).to(torch.bfloat16)
    flop = 2.0 * B * P * Q * Co * R * S * Ci
    stats = torch.zeros(2, Co, device=dev)
    row_f, row_d = [], []
    for bm, bn in [(0, 0)] + TILES:
        C.igemm_force_tile(bm, bn, 0)
        try:
            tf = timeit(lambda: C.conv_fwd(x, w, e, st, st, ph, pw, False, stats, e))
            td = timeit(lambda: C.conv_dgrad(dy, w, H, W, st, st, ph, pw, wt))
        finally:
            C.igemm_force_tile(0, 0, 0)
        lab = "auto" if bm == 0 else "%dx%d" % (bm, bn)
        row_f.append("%s %6.1f [%4.0f]" % (lab, tf, flop / tf / 1e6))
        row_d.append("%s %6.1f [%4.0f]" % (lab, td, flop / td / 1e6))
    print("%3dx%-3d %4d->%-4d %dx%d s%d fwd  | %s" % (H, W, Ci, Co, R, S, st, " | ".join(row_f)))
    print("%27s dgrad| %s" % ("", " | ".join(row_d)))
    sys.stdout.flush()
