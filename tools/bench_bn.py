"""BatchNorm kernel bandwidth at the ResNet-18 batch-256 shapes.  Knobs are read once per
process (grid and rows-in-flight are fixed in bn.hip since round 5).
    python tools/bench_bn.py [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.ops import _ext

IT = int(sys.argv[1]) if len(sys.argv) > 1 else 20
C_ = _ext.ext()
dev = torch.device("cuda", 0)
SHAPES = [(3211264, 64), (802816, 64), (200704, 128), (50176, 256), (12544, 512)]


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
    return s.elapsed_time(e) / IT * 1e-3



tot = 0.0
for M, C in SHAPES:
    x = torch.randn(M, C, device=dev).to(torch.bfloat16)
    r = torch.randn(M, C, device=dev).to(torch.bfloat16)
    dy = torch.randn(M, C, device=dev).to(torch.bfloat16)
    g = torch.ones(C, device=dev)
    b = torch.zeros(C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    st = torch.stack([x[:4096].float().mean(0), x[:4096].float().var(0)]).contiguous()
    e = torch.empty(0, device=dev)
    y, mean, rstd = C_.bn_fwd_train(x, st, g, b, rm, rv, 0.1, 1e-5, r, True)
    dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    nb = M * C * 2
    tf = timeit(lambda: C_.bn_fwd_train(x, st, g, b, rm, rv, 0.1, 1e-5, r, True))
    tb = timeit(lambda: C_.bn_bwd(dy, x, y, mean, rstd, g, dg, db, True, True))
    ts = timeit(lambda: C_.bn_fwd_train(x, e, g, b, rm, rv, 0.1, 1e-5, e, True))
    tot += tf + tb
    # bytes: fwd reads x,res writes y (3); bwd reduce reads dy,x,y (3) + apply reads dy,y,x
    # writes dx,g (5); stats-only fwd = stats pass (1) + apply (2)
    print("M=%8d C=%4d  fwd %7.1f us %5.2f TB/s | bwd %7.1f us %5.2f TB/s | stats+fwd %7.1f us %5.2f TB/s" % (
        M, C, tf * 1e6, 3 * nb / tf / 1e12, tb * 1e6, 8 * nb / tb / 1e12, ts * 1e6, 3 * nb / ts / 1e12))
print("sum fwd+bwd %.1f us" % (tot * 1e6))
