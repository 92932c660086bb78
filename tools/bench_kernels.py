"""Per-shape timing of the native conv kernels (fwd / dgrad / wgrad) on the ResNet-18 layer
shapes at a given batch, reported as TFLOP/s.  Usage:
    python tools/bench_kernels.py [batch] [iters]
Runs each shape on both staging engines (register-staged, LDS-DMA) in one process.
Set MPA_IGEMM_OCC=2|3|4 to compare occupancy targets of the register engine."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.ops import _ext

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
IT = int(sys.argv[2]) if len(sys.argv) > 2 else 10
C = _ext.ext()
dev = torch.device("cuda", 0)
SHAPES = [  # name, H, Cin, Cout, R, stride, pad
    ("stem7x7", 224, 8, 64, 7, 2, 3),
    ("l1.3x3", 56, 64, 64, 3, 1, 1),
    ("l2.3x3s2", 56, 64, 128, 3, 2, 1),
    ("l2.ds1x1", 56, 64, 128, 1, 2, 0),
    ("l2.3x3", 28, 128, 128, 3, 1, 1),
    ("l3.3x3s2", 28, 128, 256, 3, 2, 1),
    ("l3.3x3", 14, 256, 256, 3, 1, 1),
    ("l4.3x3s2", 14, 256, 512, 3, 2, 1),
    ("l4.3x3", 7, 512, 512, 3, 1, 1),
]


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
    return s.elapsed_time(e) / IT * 1e-3


ENGINES = [int(e) for e in os.environ.get("MPA_BENCH_ENGINES", "0,1").split(",")]
for eng in ENGINES:
    C.igemm_set_engine(eng)
    print("== engine %s" % ("dma" if eng else "reg"))
    print("occ=%s batch=%d" % (os.environ.get("MPA_IGEMM_OCC", "3"), B))
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    for name, H, Ci, Co, R, st, pd in SHAPES:
        x = torch.randn(B, H, H, Ci, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, R, R, Ci, device=dev) * 0.05).to(torch.bfloat16)
        P = (H + 2 * pd - R) // st + 1
        dy = torch.randn(B, P, P, Co, device=dev).to(torch.bfloat16)
        dw = torch.zeros(Co, R, R, Ci, device=dev)
        e = torch.empty(0, device=dev)
        stats = torch.empty(2, Co, device=dev)
        flop = 2.0 * B * P * P * Co * R * R * Ci
        tf = timeit(lambda: C.conv_fwd(x, w, e, st, st, pd, pd, False, stats, e))
        td = timeit(lambda: C.conv_dgrad(dy, w, H, H, st, st, pd, pd))
        tw = timeit(lambda: C.conv_wgrad(dy, x, dw, st, st, pd, pd))
        tot["fwd"] += tf
        tot["dgrad"] += td
        tot["wgrad"] += tw
        print("%-10s fwd %7.1f us %6.0f TF | dgrad %7.1f us %6.0f TF | wgrad %7.1f us %6.0f TF" % (
            name, tf * 1e6, flop / tf / 1e12, td * 1e6, flop / td / 1e12, tw * 1e6, flop / tw / 1e12))
    print("sum (one instance each): fwd %.0f us  dgrad %.0f us  wgrad %.0f us" % (
        tot["fwd"] * 1e6, tot["dgrad"] * 1e6, tot["wgrad"] * 1e6))
