"""Per-layer conv kernel table for a zoo model: every Conv2d of the model (shapes taken from
one CPU forward at batch 1), grouped by unique shape, timed on the GPU through the native
fwd / dgrad / wgrad ops at the training batch, with achieved TF = 2*N*P*Q*K*R*S*C / time
and each shape's share of the model's conv time.  Shows which layers fall off the fast
kernels (odd channel counts, valid padding, 1xk / kx1 taps).

    python tools/bench_zoo_convs.py inception [batch=256] [iters=5]
    python tools/bench_zoo_convs.py densenet 256
"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.models import initialize_model

NAME = sys.argv[1] if len(sys.argv) > 1 else "inception"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
IT = int(sys.argv[3]) if len(sys.argv) > 3 else 5

model, size = initialize_model(NAME, 1000, False)
shapes = collections.OrderedDict()  # (H, W, Ci, Co, R, S, sh, sw, ph, pw) -> [count]

# record every conv the training forward issues (the fused ops call ops.ref on the CPU,
# grouped 1x1 heads included, as one GEMM per group)
from mpi_pytorch_amd.ops import ref  # noqa: E402

_conv_fwd = ref.conv_fwd


def _rec(x, w, bias, sh, sw, ph, pw, *a, **k):
    key = (x.shape[1], x.shape[2], x.shape[3], w.shape[0], w.shape[1], w.shape[2], sh, sw, ph, pw)
    e = shapes.setdefault(key, [0])
    e[0] += 1
    return _conv_fwd(x, w, bias, sh, sw, ph, pw, *a, **k)


ref.conv_fwd = _rec
model.train()
model(torch.randn(2, size, size, 3))
ref.conv_fwd = _conv_fwd

from mpi_pytorch_amd.ops import _ext  # noqa: E402

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
    return s.elapsed_time(e) / IT * 1e-3


rows = []
tot = 0.0
for key, (cnt,) in shapes.items():
    H, W, Ci, Co, R, S, sh, sw, ph, pw = key
    if Ci % 8:  # stems with 3 input channels run a padded-channel path; skip here
        continue
    if os.environ.get("ZOO_ONLY") and "%dx%d:%d->%d" % (H, W, Ci, Co) not in os.environ["ZOO_ONLY"]:
        continue  # e.g. ZOO_ONLY="7x7:128->32,14x14:128->32"
    P = (H + 2 * ph - R) // sh + 1
    Q = (W + 2 * pw - S) // sw + 1
    x = torch.randn(B, H, W, Ci, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, R, S, Ci, device=dev) * 0.05).to(torch.bfloat16)
    dy = torch.randn(B, P, Q, Co, device=dev).to(torch.bfloat16)
    dw = torch.zeros(Co, R, S, Ci, device=dev)
    e = torch.empty(0, device=dev)
    stats = torch.empty(2, Co, device=dev)
    wt = w.permute(3, 1, 2, 0).reshape(Ci, R * S, Co).contiguous()
    flop = 2.0 * B * P * Q * Co * R * S * Ci
    ts = [timeit(lambda: C.conv_fwd(x, w, e, sh, sw, ph, pw, False, stats, e)),
          timeit(lambda: C.conv_dgrad(dy, w, H, W, sh, sw, ph, pw, wt)),
          timeit(lambda: C.conv_wgrad(dy, x, dw, sh, sw, ph, pw))]
    t3 = sum(ts) * cnt
    tot += t3
    rows.append((t3, key, cnt, ts, flop))
    del x, w, dy, dw, wt
    torch.cuda.empty_cache()

print("# tools/bench_zoo_convs.py %s batch %d: per unique conv shape (x count), fwd / dgrad / "
      "wgrad us and TF, share of the model's conv time (%.2f ms per step incl. dgrad of the "
      "first layer)" % (NAME, B, tot * 1e3))
for t3, key, cnt, ts, flop in sorted(rows, key=lambda r: -r[0]):
    H, W, Ci, Co, R, S, sh, sw, ph, pw = key
    print("%5.1f%% x%-2d %3dx%-3d %4d->%-4d %dx%d s%d%s p%d,%d | fwd %7.1f us %5.0f TF | dgrad "
          "%7.1f us %5.0f TF | wgrad %7.1f us %5.0f TF " % (
              100 * t3 / tot, cnt, H, W, Ci, Co, R, S, sh, "" if sw == sh else ",%d" % sw, ph,
              pw, ts[0] * 1e6, flop / ts[0] / 1e12, ts[1] * 1e6, flop / ts[1] / 1e12,
              ts[2] * 1e6, flop / ts[2] / 1e12))
