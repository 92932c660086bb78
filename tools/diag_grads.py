"""Diagnostic: per-parameter gradient agreement GPU (bf16 native) vs CPU (fp32 ref), and a
short training-loss trajectory eager vs HIP graph.  Not part of the test suite."""
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.engine import build_model, loss_fn, TrainStep
from mpi_pytorch_amd.parallel import World
from mpi_pytorch_amd.optim import build_optimizer


def per_param(name, hw, B, nc=40):
    gpu = torch.device("cuda", 0)
    torch.manual_seed(0)
    w = World()
    mc, _ = build_model(name, nc, False, torch.device("cpu"), w)
    mg, _ = build_model(name, nc, False, gpu, w)
    mg.load_state_dict(mc.state_dict())
    mg._mpa_arena.sync_shadow()
    for m in (mc, mg):
        for mod in m.modules():
            if type(mod).__name__ == "Dropout":
                mod.p = 0.0
    torch.manual_seed(1)
    x = torch.randn(B, hw, hw, 3) * 0.5
    y = torch.randint(0, nc, (B,))
    lc = loss_fn(mc(x), y)
    lc.backward()
    lg = loss_fn(mg(x.to(gpu).to(torch.bfloat16)), y.to(gpu))
    lg.backward()
    torch.cuda.synchronize()
    print("== %s hw=%d B=%d loss cpu %.5f gpu %.5f" % (name, hw, B, float(lc), float(lg)))
    pc = dict(mc.named_parameters())
    rows = []
    for n, p in mg.named_parameters():
        a = pc[n].grad.reshape(-1)
        b = p.grad.reshape(-1).cpu()
        cos = float(torch.nn.functional.cosine_similarity(a, b, dim=0))
        ratio = float(b.norm() / (a.norm() + 1e-12))
        rows.append((n, cos, ratio, float(a.norm())))
    for n, cos, ratio, nrm in rows:
        flag = " <<<" if cos < 0.98 else ""
        print("  %-45s cos %.4f  |g| ratio %.3f  |g| %.3e%s" % (n, cos, ratio, nrm, flag))


def traj(graph):
    gpu = torch.device("cuda", 0)
    torch.manual_seed(0)
    w = World()
    m, _ = build_model("resnet18", 64500, False, gpu, w)
    opt = build_optimizer("adam", m, 4e-4)
    st = TrainStep(m, opt, w)
    x = (torch.randn(64, 224, 224, 3, device=gpu)).to(torch.bfloat16)
    y = torch.randint(0, 64500, (64,), device=gpu)
    if graph:
        st.capture(x, y)
    out = []
    for i in range(15):
        out.append(float(st(x, y)))
    print("traj graph=%s:" % graph, " ".join("%.3f" % v for v in out))




def native_vs_refbf16(name, hw, B, nc=40):
    """Same GPU, same bf16 rounding points: native kernels vs ops/ref.py on bf16 tensors."""
    import mpi_pytorch_amd.ops.functional as Fn
    from mpi_pytorch_amd.ops import ref
    gpu = torch.device("cuda", 0)
    torch.manual_seed(0)
    w = World()
    ma, _ = build_model(name, nc, False, gpu, w)
    mb, _ = build_model(name, nc, False, gpu, w)
    mb.load_state_dict(ma.state_dict())
    for m in (ma, mb):
        m._mpa_arena.sync_shadow()
        for mod in m.modules():
            if type(mod).__name__ == "Dropout":
                mod.p = 0.0
    torch.manual_seed(1)
    x = (torch.randn(B, hw, hw, 3, device=gpu) * 0.5).to(torch.bfloat16)
    y = torch.randint(0, nc, (B,), device=gpu)
    la = loss_fn(ma(x), y)
    la.backward()
    orig = Fn.K
    Fn.K = lambda t: ref
    try:
        lb = loss_fn(mb(x), y)
        lb.backward()
    finally:
        Fn.K = orig
    torch.cuda.synchronize()
    ga, gb = ma._mpa_arena.grad, mb._mpa_arena.grad
    cos = float(torch.nn.functional.cosine_similarity(ga, gb, dim=0))
    print("== native vs ref-bf16 %s B=%d: loss %.5f %.5f  grad cos %.5f" % (name, B, float(la),
                                                                           float(lb), cos))
    pb = dict(mb.named_parameters())
    worst = []
    for n, p in ma.named_parameters():
        c = float(torch.nn.functional.cosine_similarity(p.grad.reshape(-1), pb[n].grad.reshape(-1), dim=0))
        worst.append((c, n))
    worst.sort()
    for c, n in worst[:8]:
        print("   worst %-45s cos %.4f" % (n, c))


if __name__ == "__main__" and len(sys.argv) == 1:
    for nm, hw, B in (("resnet18", 96, 8), ("inception", 299, 8), ("densenet", 96, 8),
                      ("vgg", 64, 8)):
        native_vs_refbf16(nm, hw, B)


def native_twice(name, hw, B, nc=40):
    """Run-to-run agreement of the native path (fp32 atomics => summation order varies)."""
    gpu = torch.device("cuda", 0)
    torch.manual_seed(0)
    w = World()
    m, _ = build_model(name, nc, False, gpu, w)
    for mod in m.modules():
        if type(mod).__name__ == "Dropout":
            mod.p = 0.0
    torch.manual_seed(1)
    x = (torch.randn(B, hw, hw, 3, device=gpu) * 0.5).to(torch.bfloat16)
    y = torch.randint(0, nc, (B,), device=gpu)
    gs = []
    for _ in range(2):
        m._mpa_arena.zero_grad()
        sd = {k: v.clone() for k, v in m.state_dict().items() if "running" in k or "num_b" in k}
        loss_fn(m(x), y).backward()
        m.load_state_dict(sd, strict=False)
        gs.append(m._mpa_arena.grad.clone())
    cos = float(torch.nn.functional.cosine_similarity(gs[0], gs[1], dim=0))
    print("== native run-to-run %s: grad cos %.6f  bitwise equal %s" % (name, cos,
                                                                        bool(torch.equal(*gs))))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "twice":
    for nm, hw, B in (("resnet18", 96, 8), ("inception", 299, 8), ("densenet", 96, 8)):
        native_twice(nm, hw, B)
