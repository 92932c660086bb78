"""Preprocess-kernel timing at the headline shape (512 x 224 x 224 RGB u8 -> pixel-pair
canvas bf16), against a plain device fill of the same output bytes as a write-bandwidth
yardstick.

    python tools/bench_pre.py [batch] [iters]
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
mean, std = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]


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


img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev)
for cpad, pad in ((4, [3, 3, 3, 5]), (8, []), (4, [])):
    out = C.preprocess(img, 224, 224, mean, std, 0, cpad, pad)
    nbytes = out.numel() * 2
    t = timeit(lambda: C.preprocess(img, 224, 224, mean, std, 0, cpad, pad))
    buf = torch.empty_like(out)
    tf = timeit(lambda: buf.fill_(0))
    print("cpad %d pad %-14s out %6.1f MB  preprocess %7.1f us (%5.2f TB/s)  fill %7.1f us (%5.2f TB/s)"
          % (cpad, pad, nbytes / 1e6, t, (nbytes + img.numel()) / t / 1e6, tf, nbytes / tf / 1e6))
