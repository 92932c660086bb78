"""Time the fused Adam kernel in isolation (warm and after a 4 GiB cache-evicting write)
at ResNet-18 / ResNet-50-ish / VGG-16 parameter counts, and report achieved HBM bandwidth
(30 bytes per parameter: fp32 master/m/v read+write, fp32 grad read, bf16 shadow write).

    python tools/adam_probe.py
"""
import torch

from mpi_pytorch_amd.ops import _ext


def main():
    k = _ext.load()
    dev = torch.device("cuda:0")
    flush = torch.empty(1 << 30, dtype=torch.float32, device=dev)
    for n in (11_689_512, 44_549_160, 138_357_544):
        n = (n + 7) // 8 * 8
        p = torch.randn(n, device=dev)
        g = torch.randn(n, device=dev) * 1e-2
        m = torch.zeros(n, device=dev)
        v = torch.zeros(n, device=dev)
        sh = torch.empty(n, dtype=torch.bfloat16, device=dev)
        st = torch.zeros(1, device=dev)
        for cold in (False, True):
            ts = []
            for it in range(12):
                if cold:
                    flush.fill_(float(it))
                e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
                e0.record()
                k.adam_step(p, g, m, v, sh, st, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1.0)
                e1.record()
                torch.cuda.synchronize()
                if it >= 2:
                    ts.append(e0.elapsed_time(e1) * 1e3)
            ts.sort()
            us = ts[len(ts) // 2]
            print(f"adam n={n / 1e6:7.2f}M {'cold' if cold else 'warm'}: {us:8.1f} us  "
                  f"{30 * n / us / 1e6:6.2f} TB/s", flush=True)
        del p, g, m, v, sh


if __name__ == "__main__":
    main()
