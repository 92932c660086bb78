"""Stem backward at batch B (ResNet-18: 7x7/s2 pixel-pair conv -> BN -> ReLU -> 3x3/s2/p1
max-pool, 112^2 x 64 conv output): the two-pass form (maxpool_bn_bwd writes the full-size
dz, conv_wgrad reads it) vs the fused form (pooled sums + stem_pool_wgrad, dz formed in the
weight gradient's staging).  HIP-event timed per kernel group.

    python tools/bench_stem_bwd.py [batch] [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.ops import _ext

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
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
    return s.elapsed_time(e) / IT * 1e3


torch.manual_seed(0)
P = Q = 112
x = (torch.randn(B, 2 * (P - 1) + 7, Q + 3, 8, device=dev) * 0.5).to(torch.bfloat16)
z = (torch.randn(B, P, Q, 64, device=dev) * 1.5 + 0.2).to(torch.bfloat16)
st = torch.stack([z.float().reshape(-1, 64).mean(0), z.float().reshape(-1, 64).var(0, unbiased=False)])
g = torch.rand(64, device=dev) + 0.5
b = torch.randn(64, device=dev) * 0.5
rm, rv = torch.zeros(64, device=dev), torch.ones(64, device=dev)
zsel = torch.empty(B, P // 2, Q // 2, 64, device=dev, dtype=torch.bfloat16)
y, idx, mean, rstd = C.bn_relu_maxpool_fwd(z, st, g, b, rm, rv, 0.1, 1e-5, 3, 3, 2, 2, 1, 1,
                                           False, zsel_out=zsel)
dp = torch.randn_like(y)
dg, db = torch.zeros(64, device=dev), torch.zeros(64, device=dev)
dw = torch.zeros(64, 7, 4, 8, device=dev)
holder = {}


def two_pass_bn():
    holder["dz"] = C.maxpool_bn_bwd(dp, idx, z, mean, rstd, g, b, dg, db, 3, 3, 2, 2, 1, 1,
                                    zsel=zsel)


two_pass_bn()
t_bn = timeit(two_pass_bn)
t_wg = timeit(lambda: C.conv_wgrad(holder["dz"], x, dw, 2, 1, 0, 0, True))
sums = C.maxpool_bn_bwd_sums(dp, zsel, mean, rstd, g, b, dg, db)
t_sums = timeit(lambda: C.maxpool_bn_bwd_sums(dp, zsel, mean, rstd, g, b, dg, db))
t_pool = timeit(lambda: C.stem_pool_wgrad(dp, idx, z, mean, rstd, g, b, sums, x, dw, 2, 1, 0, 0,
                                          True))
t_fwd = timeit(lambda: C.bn_relu_maxpool_fwd(z, st, g, b, rm, rv, 0.1, 1e-5, 3, 3, 2, 2, 1, 1,
                                             False, zsel_out=zsel))
print("batch %d: two-pass  maxpool_bn_bwd %.1f us + conv_wgrad %.1f us = %.1f us"
      % (B, t_bn, t_wg, t_bn + t_wg))
print("          fused     sums %.1f us + stem_pool_wgrad %.1f us = %.1f us"
      % (t_sums, t_pool, t_sums + t_pool))
print("          forward   bn_relu_maxpool_fwd %.1f us" % t_fwd)

# forward: conv + separate pool pass vs the pool fused into the conv kernel
w = (torch.randn(64, 7, 4, 8, device=dev) * 0.05).to(torch.bfloat16)
st = torch.empty(2, 64, device=dev)
sh = torch.zeros(64, device=dev)
e = torch.empty(0, device=dev)
zs = torch.empty(B, P // 2, Q // 2, 64, device=dev, dtype=torch.bfloat16)


def two_pass_fwd():
    zz = C.conv_fwd(x, w, e, 2, 1, 0, 0, False, st, sh)
    C.bn_relu_maxpool_fwd(zz, st, g, b, rm, rv, 0.1, 1e-5, 3, 3, 2, 2, 1, 1, False, zsel_out=zs)


t_conv = timeit(lambda: C.conv_fwd(x, w, e, 2, 1, 0, 0, False, st, sh))
t_two = timeit(two_pass_fwd)
t_fused = timeit(lambda: C.conv_stem_pool_fwd(x, w, 2, 1, 0, 0, st, sh, g, b, rm, rv, 0.1, 1e-5))
print("          forward   conv %.1f us; conv + pool pass %.1f us; fused conv+pool + apply %.1f us"
      % (t_conv, t_two, t_fused))
