"""Print the teacher-forced unit parity table (utils/parity.py) of the zoo models:
per unit the cosines / norm ratios of output, input gradient and parameter gradients,
native bf16 GPU vs fp32 CPU.  python tools/unit_parity.py [model ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.engine import build_model, loss_fn
from mpi_pytorch_amd.parallel import World
from mpi_pytorch_amd.utils.parity import unit_parity

SIZES = {"resnet18": 64, "resnet34": 64, "vgg": 64, "alexnet": 127, "squeezenet": 96,
         "densenet": 64, "inception": 299, "vgg16": 64}
gpu = torch.device("cuda", 0)
for name in sys.argv[1:] or list(SIZES):
    hw = SIZES[name]
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
    x = (torch.randn(8, hw, hw, 3) * 0.5).to(gpu).to(torch.bfloat16)
    y = torch.randint(0, 40, (8,)).to(gpu)
    rows = unit_parity(mg, mc, x, y, loss_fn)
    worst = lambda k: min((r[k] for r in rows if k in r), default=float("nan"))
    print("== %s @%d, batch 8: %d units, min y_cos %.5f  min dx_cos %.5f  min dw_cos %.5f" % (
        name, hw, len(rows), worst("y_cos"), worst("dx_cos"), worst("dw_cos")), flush=True)
    for r in rows:
        print("  %-42s %-14s y %.5f/%.4f  dx %s  dw %s" % (
            r["unit"][:42], r["type"][:14], r["y_cos"], r["y_ratio"],
            "%.5f/%.4f" % (r["dx_cos"], r["dx_ratio"]) if "dx_cos" in r else "-",
            "%.5f/%.4f" % (r["dw_cos"], r["dw_ratio"]) if "dw_cos" in r else "-"))
