"""Gradient agreement of a model's native GPU path against the fp32 CPU path, per GEMM
staging engine, plus native-vs-native repeat agreement (the run-to-run floor set by
summation-order differences).  Usage: python tools/diag_engines.py [model] [hw] [batch]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.engine import build_model, loss_fn
from mpi_pytorch_amd.ops import _ext
from mpi_pytorch_amd.parallel import World

name = sys.argv[1] if len(sys.argv) > 1 else "inception"
hw = int(sys.argv[2]) if len(sys.argv) > 2 else 299
B = int(sys.argv[3]) if len(sys.argv) > 3 else 4
gpu = torch.device("cuda", 0)
torch.manual_seed(0)
mc, _ = build_model(name, 40, False, torch.device("cpu"), World())
mg, _ = build_model(name, 40, False, gpu, World())
mg.load_state_dict(mc.state_dict())
mg._mpa_arena.sync_shadow()
for m in (mc, mg):
    for mod in m.modules():
        if type(mod).__name__ == "Dropout":
            mod.p = 0.0
torch.manual_seed(1)
x = torch.randn(B, hw, hw, 3) * 0.5
y = torch.randint(0, 40, (B,))
lc = loss_fn(mc(x), y)
lc.backward()
gc = mc._mpa_arena.grad.clone()
C = _ext.ext()


def native():
    mg._mpa_arena.grad.zero_()
    for mod in mg.modules():  # identical BN running stats each run (stats shift input)
        if hasattr(mod, "running_mean") and mod.running_mean is not None:
            mod.running_mean.zero_()
            mod.running_var.fill_(1.0)
    lg = loss_fn(mg(x.to(gpu).to(torch.bfloat16)), y.to(gpu))
    lg.backward()
    torch.cuda.synchronize()
    return float(lg), mg._mpa_arena.grad.cpu().clone()


cos = lambda a, b: float(torch.nn.functional.cosine_similarity(a, b, dim=0))
print("%s hw=%d B=%d  cpu loss %.5f" % (name, hw, B, float(lc)))
res = {}
for eng in (0, 1, 2):
    C.igemm_set_engine(eng)
    l1, g1 = native()
    l2, g2 = native()
    res[eng] = g1
    print("engine %d: loss %.5f  cos(cpu)=%.4f ratio=%.4f  cos(repeat)=%.4f  equal(repeat)=%s" % (
        eng, l1, cos(gc, g1), float(g1.norm() / gc.norm()), cos(g1, g2), torch.equal(g1, g2)))
print("cos(engine0, engine1)=%.4f cos(engine0, engine2)=%.4f" % (cos(res[0], res[1]), cos(res[0], res[2])))
# per-parameter breakdown for the default engine
C.igemm_set_engine(1)
_, g1 = native()
off = 0
worst = []
for n_, p in mg.named_parameters():
    k = p.numel()
    a, b = gc[off:off + k], g1[off:off + k]
    off += k
    if float(a.norm()) > 0:
        worst.append((cos(a, b), n_, float(b.norm() / a.norm())))
worst.sort()
for c_, n_, r_ in worst[:12]:
    print("  %-50s cos %.4f ratio %.3f" % (n_, c_, r_))
