"""Multi-rank check of the data-parallel path on GPU tensors with the native kernels.
Launch with N ranks (they may share one GPU when the backend is gloo):

    MPA_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 \
        --master-addr 127.0.0.1 tools/dp_check.py

Checks, printed as one line per check on rank 0 and exit code 1 on failure:
1. ``sync_params`` makes differently-initialised replicas identical;
2. the bucketed all-reduce issued from backward (overlap) equals a plain post-backward
   all-reduce of the same local gradients (the reference's ``mpi_avg_grads`` semantics);
3. after several optimizer steps on different data, replicas are still identical.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist

from mpi_pytorch_amd.engine import build_training, loss_fn
from mpi_pytorch_amd.parallel import init_world, replica_checksum, sync_params, shutdown


def main():
    world = init_world("cuda")
    rank, n = world.rank, world.world_size
    dev = world.device
    torch.manual_seed(1234 + rank)  # different init per rank
    # AlexNet without dropout: no BatchNorm, so two backward passes over the same batch
    # differ only by fp32 summation order (BN nets at init amplify that chaotically)
    model, opt, step, _ = build_training("alexnet", 100, dev, world, 1e-4, bucket_mb=16.0)
    for mod in model.modules():
        if type(mod).__name__ == "Dropout":
            mod.p = 0.0
    ok = True

    def report(name, cond, extra=""):
        nonlocal ok
        ok &= bool(cond)
        if rank == 0:
            print("%-46s %s %s" % (name, "OK" if cond else "FAIL", extra), flush=True)

    sync_params(model)
    report("params identical after sync_params", replica_checksum(model))

    gen = torch.Generator().manual_seed(99 + rank)  # different data per rank
    x = torch.randn(8, 64, 64, 3, generator=gen).to(dev).to(torch.bfloat16)
    y = torch.randint(0, 100, (8,), generator=gen).to(dev)
    arena = model._mpa_arena
    bk = model._mpa_bucketer

    # (a) overlapped bucketed all-reduce from backward
    arena.zero_grad()
    loss_fn(model(x), y).backward()
    bk.finish()
    g_overlap = arena.grad.clone()
    # (b) local gradient only, then one plain all-reduce after backward
    bk.active = False
    arena.zero_grad()
    loss_fn(model(x), y).backward()
    bk.active = True
    g_local = arena.grad.clone()
    dist.all_reduce(g_local)
    torch.cuda.synchronize()
    rel = float((g_overlap - g_local).abs().max() / (g_local.abs().max() + 1e-12))
    cos = float(torch.nn.functional.cosine_similarity(g_overlap, g_local, dim=0))
    report("bucketed overlap == post-backward all-reduce", rel < 2e-2 and cos > 0.999,
           "(rel %.2e, cos %.6f, %d buckets)" % (rel, cos, len(bk.buckets)))

    # (c) replicas stay identical through optimizer steps on different data
    for _ in range(3):
        step(x, y)
    torch.cuda.synchronize()
    report("replicas identical after 3 steps", replica_checksum(model),
           "(loss %.4f)" % float(step.mean_loss()))
    shutdown()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
