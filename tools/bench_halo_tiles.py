"""A/B of the halo 3x3 kernel's tile height on ResNet-18 layer1 (56x56x64 -> 64, batch B):
256-pixel tiles (MI = 4) vs 448-pixel tiles of whole rows (MI = 7, MPA_HALO_MI7), forward
with BN statistics and the plain dgrad, HIP-event timed; prints us / TFLOP/s and checks the
two tilings give bitwise-equal outputs.

    python tools/bench_halo_tiles.py [batch] [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.ops import _ext

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
IT = int(sys.argv[2]) if len(sys.argv) > 2 else 20
C = _ext.ext()
dev = torch.device("cuda", 0)


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
    return s.elapsed_time(e) / IT * 1e3


torch.manual_seed(0)
H, Ci, Co = 56, 64, 64
x = torch.randn(B, H, H, Ci, device=dev).to(torch.bfloat16)
w = (torch.randn(Co, 3, 3, Ci, device=dev) * 0.05).to(torch.bfloat16)
dy = torch.randn(B, H, H, Co, device=dev).to(torch.bfloat16)
e = torch.empty(0, device=dev)
shift = torch.randn(Co, device=dev) * 0.1
flop = 2.0 * B * H * H * Co * 9 * Ci
res = {}
for mi7 in (0, 1):
    C.igemm_set_halo_mi7(mi7)
    st = torch.empty(2, Co, device=dev)
    y = C.conv_fwd(x, w, e, 1, 1, 1, 1, False, st, shift)
    dx = C.conv_dgrad(dy, w, H, H, 1, 1, 1, 1)
    acc = x.clone()
    dxa = C.conv_dgrad(dy, w, H, H, 1, 1, 1, 1, None, acc)
    tf = timeit(lambda: C.conv_fwd(x, w, e, 1, 1, 1, 1, False, st, shift))
    td = timeit(lambda: C.conv_dgrad(dy, w, H, H, 1, 1, 1, 1))
    res[mi7] = (y, st.clone(), dx, dxa)
    print("MI%d  fwd+stats %7.1f us %6.0f TF | dgrad %7.1f us %6.0f TF"
          % (7 if mi7 else 4, tf, flop / tf * 1e-6, td, flop / td * 1e-6), flush=True)
C.igemm_set_halo_mi7(1)
(y0, s0, d0, a0), (y1, s1, d1, a1) = res[0], res[1]
print("fwd bitwise equal:", torch.equal(y0, y1), " dgrad bitwise equal:", torch.equal(d0, d1),
      " accumulate bitwise equal:", torch.equal(a0, a1),
      " stats max rel diff: %.2e" % float(((s0 - s1).abs() / (s0.abs() + 1e-6)).max()))
