"""Root-cause probe for HIP-graph replay divergence (docs/NOTES.md "HIP graph replay").

Deterministic mode makes a step a pure function of its inputs, so graph replays can be
compared BITWISE with eager steps.  For each separation between replays

    none  - back-to-back replay() calls (the failing pattern),
    event - an event recorded and waited on the same stream (no host sync),
    sync  - a host stream synchronize (the known-good pattern),

and for graphs of the forward only (no state change: every replay must equal the first),
forward+backward, and the full step, report the first replay whose loss / gradient /
weights differ from eager.

    python tools/graph_bisect.py [batch=32] [hw=64] [replays=60]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.engine import build_training, loss_fn
from mpi_pytorch_amd.ops import _ext
from mpi_pytorch_amd.parallel import World

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
HW = int(sys.argv[2]) if len(sys.argv) > 2 else 64
R = int(sys.argv[3]) if len(sys.argv) > 3 else 60
NC = int(os.environ.get("NC", "100"))
gpu = torch.device("cuda", 0)
_ext.ext().set_deterministic(int(os.environ.get("DET", "1")))
g = torch.Generator().manual_seed(1)
x = (torch.randn(B, HW, HW, 8, generator=g) * (torch.arange(8) < 3)).to(gpu, torch.bfloat16)
y = torch.randint(0, NC, (B,), generator=g).to(gpu)


def fresh():
    torch.manual_seed(0)
    return build_training(os.environ.get("MODEL", "resnet18"), NC, gpu, World(device=gpu),
                          1e-3)[:3]


def checksum(model):
    a = model._mpa_arena
    return torch.stack([a.grad.double().sum(), a.master.double().sum(),
                        a.grad.double().abs().sum()])


def eager_ref(n):
    model, opt, step = fresh()
    losses, sums = [], []
    for _ in range(n):
        losses.append(step(x, y).clone())
        sums.append(checksum(model))
    torch.cuda.synchronize()
    return torch.stack(losses), torch.stack(sums)


def run_step_graph(sep, n):
    model, opt, step = fresh()
    step.capture(x, y, warmup=2)
    losses, sums = [], []
    ev = torch.cuda.Event()
    for _ in range(n):
        losses.append(step(x, y).clone())
        sums.append(checksum(model))
        if sep == "event":
            ev.record()
            torch.cuda.current_stream().wait_event(ev)
        elif sep == "sync":
            torch.cuda.current_stream().synchronize()
    torch.cuda.synchronize()
    return torch.stack(losses), torch.stack(sums)


def first_diff(a, b):
    d = (a != b)
    if d.dim() > 1:
        d = d.any(dim=1)
    idx = d.nonzero()
    return -1 if idx.numel() == 0 else int(idx[0])


def run_fwd_graph(sep, n, with_bwd):
    model, opt, step = fresh()
    arena = model._mpa_arena

    def body():
        arena.zero_grad()
        loss = loss_fn(model(x), y)
        if with_bwd:
            loss.backward()
        return loss.detach()

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            body()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        out = body()
    vals, sums = [], []
    ev = torch.cuda.Event()
    for _ in range(n):
        gr.replay()
        vals.append(out.clone())
        sums.append(checksum(model))
        if sep == "event":
            ev.record()
            torch.cuda.current_stream().wait_event(ev)
        elif sep == "sync":
            torch.cuda.current_stream().synchronize()
    torch.cuda.synchronize()
    v, c = torch.stack(vals), torch.stack(sums)
    # the BN running mean drifts between replays and the conv epilogues take their
    # statistics around it (docs/NOTES.md "BN statistics without cancellation"), so replays
    # agree to rounding, not bitwise: report the spread
    return float((v - v[0]).abs().max()), float(((c - c[0]).abs() / c[0].abs()).max()), v


print("batch %d hw %d replays %d deterministic %d" % (B, HW, R, _ext.ext().deterministic()),
      flush=True)
for with_bwd in (False, True):
    for sep in ("none", "event", "sync"):
        fl, fc, v = run_fwd_graph(sep, R, with_bwd)
        print("%-7s sep=%-5s spread over replays: loss %.3g  grad/weights (rel) %.3g   "
              "(loss[0] %.6f, nan %d)" % ("fwdbwd" if with_bwd else "fwd", sep, fl, fc,
                                          float(v[0]), int(torch.isnan(v).sum())), flush=True)
ref_l, ref_c = eager_ref(R + 2)
ref_l, ref_c = ref_l[2:], ref_c[2:]
for sep in ("none", "event", "sync"):
    l, c = run_step_graph(sep, R)
    print("step    sep=%-5s first replay != eager: loss %d  grad/weights %d   (max |dloss| %.3g, "
          "nan %d)" % (sep, first_diff(l, ref_l), first_diff(c, ref_c),
                       float((l - ref_l).abs().nan_to_num(1e30).max()), int(torch.isnan(l).sum())),
          flush=True)
