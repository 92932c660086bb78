"""Vendor-library yardstick for the native kernels: the same ResNet-18 work run through
PyTorch-ROCm's own paths (MIOpen convolutions, hipBLASLt GEMMs, ATen BN/pool/CE, fused
torch Adam), on the same GPU, same dtype, same batch.

    python tools/bench_vendor.py layers [batch] [iters]   per-layer MIOpen conv fwd/dgrad/wgrad
                                                          + hipBLASLt GEMM of the im2col shape
    python tools/bench_vendor.py model  [batch] [steps]   whole ResNet-18 @64,500 training step
                                                          (channels_last, bf16 autocast, fp32
                                                          master weights, fused Adam)

This is a measurement tool only: nothing in the framework falls back to these paths.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn as nn
import torch.nn.functional as F

MODE = sys.argv[1] if len(sys.argv) > 1 else "layers"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
IT = int(sys.argv[3]) if len(sys.argv) > 3 else 10
dev = torch.device("cuda", 0)

SHAPES = [  # name, H, Cin, Cout, R, stride, pad  (tools/bench_kernels.py)
    ("stem7x7", 224, 3, 64, 7, 2, 3),
    ("l1.3x3", 56, 64, 64, 3, 1, 1),
    ("l2.3x3s2", 56, 64, 128, 3, 2, 1),
    ("l2.ds1x1", 56, 64, 128, 1, 2, 0),
    ("l2.3x3", 28, 128, 128, 3, 1, 1),
    ("l3.3x3s2", 28, 128, 256, 3, 2, 1),
    ("l3.3x3", 14, 256, 256, 3, 1, 1),
    ("l4.3x3s2", 14, 256, 512, 3, 2, 1),
    ("l4.3x3", 7, 512, 512, 3, 1, 1),
]


def timeit(fn, it=IT):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e-3


def layers():
    print("vendor per-layer, batch %d (MIOpen conv channels_last bf16; hipBLASLt GEMM)" % B)
    tot = [0.0, 0.0, 0.0]
    for name, H, Ci, Co, R, st, pd in SHAPES:
        x = torch.randn(B, Ci, H, H, device=dev, dtype=torch.bfloat16).to(
            memory_format=torch.channels_last)
        w = (torch.randn(Co, Ci, R, R, device=dev) * 0.05).to(torch.bfloat16).to(
            memory_format=torch.channels_last)
        P = (H + 2 * pd - R) // st + 1
        dy = torch.randn(B, Co, P, P, device=dev, dtype=torch.bfloat16).to(
            memory_format=torch.channels_last)
        flop = 2.0 * B * P * P * Co * R * R * Ci
        tf = timeit(lambda: F.conv2d(x, w, stride=st, padding=pd))
        td = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [st, st], [pd, pd], [1, 1], False, [0, 0], 1, [True, False, False]))
        tw = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [st, st], [pd, pd], [1, 1], False, [0, 0], 1, [False, True, False]))
        M, N, K = B * P * P, Co, R * R * Ci
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
        tg = timeit(lambda: a @ b)
        for i, t in enumerate((tf, td, tw)):
            tot[i] += t
        print("%-9s fwd %8.1f us %5.0f TF | dgrad %8.1f us %5.0f TF | wgrad %8.1f us %5.0f TF"
              " | gemm(%d,%d,%d) %7.1f us %5.0f TF" % (
                  name, tf * 1e6, flop / tf / 1e12, td * 1e6, flop / td / 1e12, tw * 1e6,
                  flop / tw / 1e12, M, N, K, tg * 1e6, flop / tg / 1e12), flush=True)
        del x, w, dy, a, b
    print("sum (one instance each): fwd %.0f us  dgrad %.0f us  wgrad %.0f us" %
          tuple(t * 1e6 for t in tot))


class Block(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False),
                                      nn.BatchNorm2d(cout))

    def forward(self, x):
        o = F.relu(self.bn1(self.conv1(x)))
        o = self.bn2(self.conv2(o))
        return F.relu(o + (x if self.down is None else self.down(x)))


class ResNet18(nn.Module):
    def __init__(self, nc):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        cfg = [(64, 64, 1), (64, 64, 1), (64, 128, 2), (128, 128, 1), (128, 256, 2),
               (256, 256, 1), (256, 512, 2), (512, 512, 1)]
        self.blocks = nn.Sequential(*[Block(*c) for c in cfg])
        self.fc = nn.Linear(512, nc)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.bn1(self.conv1(x))), 3, 2, 1)
        x = self.blocks(x)
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def model():
    torch.backends.cudnn.benchmark = True
    m = ResNet18(64500).to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.Adam(m.parameters(), lr=4e-4, fused=True)
    x = torch.randn(B, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 64500, (B,), device=dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    for i in range(5):
        step()
        torch.cuda.synchronize()
        print("warmup step %d done" % i, flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(IT):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / IT
    print("vendor ResNet-18 @64500 train step, batch %d, bf16 autocast + fused Adam, "
          "static data: %.2f ms/step, %.0f img/s" % (B, dt * 1e3, B / dt), flush=True)


if __name__ == "__main__":
    {"layers": layers, "model": model}[MODE]()
