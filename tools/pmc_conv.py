"""Run a few ResNet-18 conv GEMMs (fwd / dgrad / wgrad) a handful of times each, for
hardware-counter collection:
    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES ... --kernel-trace --output-format csv \\
        -d out -- python tools/pmc_conv.py [batch] [shape,shape,...]
Shapes (default l1.3x3,l3.3x3): the names of tools/bench_kernels.py SHAPES, e.g.
l2.3x3s2,l2.ds1x1.  Summarise with tools/pmc_summary.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_pytorch_amd.ops import _ext

C = _ext.ext()
dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
TABLE = {  # name: H, Cin, Cout, R, stride, pad
    "l1.3x3": (56, 64, 64, 3, 1, 1), "l2.3x3s2": (56, 64, 128, 3, 2, 1),
    "l2.ds1x1": (56, 64, 128, 1, 2, 0), "l2.3x3": (28, 128, 128, 3, 1, 1),
    "l3.3x3s2": (28, 128, 256, 3, 2, 1), "l3.3x3": (14, 256, 256, 3, 1, 1),
    "l4.3x3s2": (14, 256, 512, 3, 2, 1), "l4.3x3": (7, 512, 512, 3, 1, 1),
}
names = (sys.argv[2] if len(sys.argv) > 2 else "l1.3x3,l3.3x3").split(",")
for name in names:
    H, Ci, Co, R, st, pd = TABLE[name]
    x = torch.randn(B, H, H, Ci, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, R, R, Ci, device=dev) * 0.05).to(torch.bfloat16)
    P = (H + 2 * pd - R) // st + 1
    dy = torch.randn(B, P, P, Co, device=dev).to(torch.bfloat16)
    dw = torch.zeros(Co, R, R, Ci, device=dev)
    e = torch.empty(0, device=dev)
    stats = torch.empty(2, Co, device=dev)
    wt = w.permute(3, 1, 2, 0).reshape(Ci, R * R, Co).contiguous()  # as training runs dgrad
    for _ in range(3):
        C.conv_fwd(x, w, e, st, st, pd, pd, False, stats, e)
        C.conv_dgrad(dy, w, H, H, st, st, pd, pd, wt)
        C.conv_wgrad(dy, x, dw, st, st, pd, pd)
    torch.cuda.synchronize()
print("done")
