"""Timing of the classifier-head ops of the headline step (ResNet-18 @64,500 classes):
linear fwd / dgrad / wgrad at [batch, 512] x [64,512, 512], the fused CE fwd / bwd, and a
wgrad tile sweep (forced BM x BN, splits).

    python tools/bench_head.py [batch] [iters]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.ops import _ext

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
IT = int(sys.argv[2]) if len(sys.argv) > 2 else 20
C = _ext.ext()
dev = torch.device("cuda", 0)
NO, NI = 64512, 512


def timeit(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(IT):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / IT * 1e3  # us


x = torch.randn(B, NI, device=dev).to(torch.bfloat16)
w = (torch.randn(NO, NI, device=dev) * 0.05).to(torch.bfloat16)
wt = w.t().contiguous()
b = torch.randn(NO, device=dev)
dy = (torch.randn(B, NO, device=dev) * 0.01).to(torch.bfloat16)
dw = torch.zeros(NO, NI, device=dev)
labels = torch.randint(0, 64500, (B,), device=dev)
gflop = 2.0 * B * NO * NI / 1e9

rows = [("linear_fwd", lambda: C.linear_fwd(x, w, b, False)),
        ("linear_dgrad", lambda: C.linear_dgrad(dy, w, wt)),
        ("linear_wgrad", lambda: C.linear_wgrad(dy, x, dw)),
        ("wgrad_overwr", lambda: C.linear_wgrad(dy, x, dw, overwrite=True))]
for name, fn in rows:
    t = timeit(fn)
    print("%-14s %8.1f us  %6.0f TF" % (name, t, gflop / t * 1e3))
logits = C.linear_fwd(x, w, b, False)[:, :64500]
loss, lse = C.ce_fwd(logits, labels)
go = torch.ones(1, device=dev)
print("%-14s %8.1f us" % ("ce_fwd", timeit(lambda: C.ce_fwd(logits, labels))))
print("%-14s %8.1f us" % ("ce_bwd", timeit(lambda: C.ce_bwd(logits, labels, lse, go))))

print("wgrad sweep (BM x BN / splits): us")
for bm, bn in ((128, 256), (256, 256), (128, 128), (64, 128), (64, 256)):
    cells = []
    for sp in (1, 2, 4):
        C.igemm_force_tile(bm, bn, sp)
        cells.append("s%d %7.1f" % (sp, timeit(lambda: C.linear_wgrad(dy, x, dw))))
    print("%3dx%-3d " % (bm, bn) + " | ".join(cells))
C.igemm_force_tile(0, 0, 0)
print("fwd sweep (BM x BN / splits): us")
for bm, bn in ((128, 128), (256, 128), (256, 64), (128, 64), (256, 256)):
    cells = []
    for sp in (1, 2):
        C.igemm_force_tile(bm, bn, sp)
        cells.append("s%d %7.1f" % (sp, timeit(lambda: C.linear_fwd(x, w, b, False))))
    print("%3dx%-3d " % (bm, bn) + " | ".join(cells))
C.igemm_force_tile(0, 0, 0)

print("dgrad sweep (BM x BN / splits, transposed weight): us")
for bm, bn in ((128, 64), (128, 128), (256, 128), (256, 256), (256, 64)):
    cells = []
    for sp in (4, 8, 16, 32, 64):
        C.igemm_force_tile(bm, bn, sp)
        cells.append("s%d %6.1f" % (sp, timeit(lambda: C.linear_dgrad(dy, w, wt))))
    print("%3dx%-3d " % (bm, bn) + " | ".join(cells))
C.igemm_force_tile(0, 0, 0)
print("%-14s %8.1f us (auto)" % ("linear_dgrad", timeit(lambda: C.linear_dgrad(dy, w, wt))))
print("%-14s %8.1f us (auto, forward weight: transposing LDS reads, no [in][out] copy)" % (
    "linear_dgrad", timeit(lambda: C.linear_dgrad(dy, w))))

# vendor GEMMs (hipBLASLt through torch) on the same shapes, for comparison
print("vendor (torch / hipBLASLt):")
vrows = [("F.linear fwd", lambda: torch.nn.functional.linear(x, w, b.to(torch.bfloat16))),
         ("mm dgrad", lambda: torch.mm(dy, w))]
try:
    torch.mm(dy.t(), x, out_dtype=torch.float32)
    vrows.append(("mm wgrad fp32", lambda: torch.mm(dy.t(), x, out_dtype=torch.float32)))
except Exception as ex:  # no bf16 -> fp32 mm on this build
    print("  mm(out_dtype=float32) unavailable: %s" % str(ex)[:80])
vrows.append(("mm wgrad bf16", lambda: torch.mm(dy.t(), x)))
for name, fn in vrows:
    t = timeit(fn)
    print("%-14s %8.1f us  %6.0f TF" % (name, t, gflop / t * 1e3))
