"""Per-shape timing of the native conv kernels (fwd / dgrad / wgrad) on the ResNet-18 layer
shapes at a given batch, reported as TFLOP/s.

    python tools/bench_kernels.py [batch] [iters]          engines 0 (register) and 1/2 (DMA)
    python tools/bench_kernels.py [batch] [iters] sweep    every tile on the DMA engine
    (MPA_SWEEP_SHAPES=s2,ds: only the shapes whose name contains one of those)

MPA_BENCH_ENGINES=0,1,1h,2 selects engines ("1h": halo 3x3/s1 kernel on).  Sweep rows print each tile's time (us) with its split count forced to
auto; the `auto` column is what the planner picks."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.ops import _ext

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
IT = int(sys.argv[2]) if len(sys.argv) > 2 else 10
SWEEP = len(sys.argv) > 3 and sys.argv[3] == "sweep"
C = _ext.ext()
dev = torch.device("cuda", 0)
SHAPES = [  # name, H, Cin, Cout, R, stride, pad
    ("stem7x7", 224, 8, 64, 7, 2, 3),
    ("l1.3x3", 56, 64, 64, 3, 1, 1),
    ("l2.3x3s2", 56, 64, 128, 3, 2, 1),
    ("l2.ds1x1", 56, 64, 128, 1, 2, 0),
    ("l2.3x3", 28, 128, 128, 3, 1, 1),
    ("l3.3x3s2", 28, 128, 256, 3, 2, 1),
    ("l3.ds1x1", 28, 128, 256, 1, 2, 0),
    ("l3.3x3", 14, 256, 256, 3, 1, 1),
    ("l4.3x3s2", 14, 256, 512, 3, 2, 1),
    ("l4.ds1x1", 14, 256, 512, 1, 2, 0),
    ("l4.3x3", 7, 512, 512, 3, 1, 1),
]
ROWS_TILES = [(0, 0), (256, 128), (128, 128), (256, 64), (128, 64)]
WGRAD_TILES = [(0, 0), (256, 256), (128, 256), (128, 128), (64, 128)]


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


def tensors(H, Ci, Co, R, st, pd):
    x = torch.randn(B, H, H, Ci, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, R, R, Ci, device=dev) * 0.05).to(torch.bfloat16)
    P = (H + 2 * pd - R) // st + 1
    dy = torch.randn(B, P, P, Co, device=dev).to(torch.bfloat16)
    dw = torch.zeros(Co, R, R, Ci, device=dev)
    e = torch.empty(0, device=dev)
    stats = torch.empty(2, Co, device=dev)
    flop = 2.0 * B * P * P * Co * R * R * Ci
    # dgrad as training runs it: from the transposed weight copy [C][R*S][K] (arena shadow_t)
    wt = w.permute(3, 1, 2, 0).reshape(Ci, R * R, Co).contiguous() if Ci % 8 == 0 else None
    fns = (lambda: C.conv_fwd(x, w, e, st, st, pd, pd, False, stats, e),
           lambda: C.conv_dgrad(dy, w, H, H, st, st, pd, pd, wt),
           lambda: C.conv_wgrad(dy, x, dw, st, st, pd, pd))
    return flop, fns


if SWEEP:
    C.igemm_set_engine(2)
    print("tile sweep, DMA engine, batch %d (us; TF in brackets)" % B)
    only = os.environ.get("MPA_SWEEP_SHAPES")  # e.g. "s2,ds": names containing either
    for name, H, Ci, Co, R, st, pd in SHAPES:
        if only and not any(k in name for k in only.split(",")):
            continue
        flop, (f, d, w) = tensors(H, Ci, Co, R, st, pd)
        for label, fn, tiles in (("fwd", f, ROWS_TILES), ("dgrad", d, ROWS_TILES),
                                 ("wgrad", w, WGRAD_TILES)):
            cells = []
            for bm, bn in tiles:
                C.igemm_force_tile(bm, bn, 0)
                t = timeit(fn)
                cells.append("%s %6.1f(%4.0f)" % ("auto" if bm == 0 else "%dx%d" % (bm, bn),
                                                 t * 1e6, flop / t / 1e12))
            print("%-9s %-5s " % (name, label) + " | ".join(cells))
        C.igemm_force_tile(0, 0, 0)
    sys.exit(0)

# "1h": engine 1 with the halo-staged 3x3/s1 kernel (conv_halo.hip) on; plain numbers off
ENGINES = os.environ.get("MPA_BENCH_ENGINES", "0,1,1h,2").split(",")
for spec in ENGINES:
    eng = int(spec.rstrip("h"))
    C.igemm_set_engine(eng)
    C.igemm_set_halo(1 if spec.endswith("h") else 0)
    print("== engine %s (%s%s)" % (spec, ["register", "dma rows", "dma all"][eng],
                                   " + halo 3x3/s1" if spec.endswith("h") else ""))
    print("batch=%d" % B)
    tot = [0.0, 0.0, 0.0]
    for name, H, Ci, Co, R, st, pd in SHAPES:
        flop, fns = tensors(H, Ci, Co, R, st, pd)
        ts = [timeit(fn) for fn in fns]
        for i in range(3):
            tot[i] += ts[i]
        print("%-10s fwd %7.1f us %6.0f TF | dgrad %7.1f us %6.0f TF | wgrad %7.1f us %6.0f TF" % (
            name, ts[0] * 1e6, flop / ts[0] / 1e12, ts[1] * 1e6, flop / ts[1] / 1e12,
            ts[2] * 1e6, flop / ts[2] / 1e12))
    print("sum (one instance each): fwd %.0f us  dgrad %.0f us  wgrad %.0f us" % (
        tot[0] * 1e6, tot[1] * 1e6, tot[2] * 1e6))
