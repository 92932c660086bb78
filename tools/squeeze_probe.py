"""SqueezeNet-1.0 slow-mode probe (round-5 review, weak item 7).

Some processes run SqueezeNet-1.0 at batch 512 2.5-4x slower than others for their whole
life (profiles/squeezenet_slow_runs_r5.txt), never under rocprofv3.  This probe times ONE
process with HIP events only (no profiler):

  * per-phase step times (StepTimer: forward / backward / optimizer);
  * per-module forward times of one step (forward pre / post hooks on the leaf modules);
  * HBM bandwidth of a streaming write over freshly allocated buffers of the head's
    activation size (11.2 GB), twice, and over a small (256 MB) buffer.

Run it in several processes one after another and compare a slow process with a fast one:

    python tools/squeeze_probe.py [batch] [steps] [model] [static]

(model: squeezenet (default) or any zoo name, e.g. resnet18; static = 1 reuses one batch)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def _ev():
    return torch.cuda.Event(enable_timing=True)


def bw_probe(nbytes: int, reps: int = 2):
    t = torch.empty(nbytes // 2, dtype=torch.bfloat16, device="cuda")
    out = []
    for _ in range(reps):
        a, b = _ev(), _ev()
        a.record()
        t.fill_(1.0)
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b)
        out.append(round(nbytes / ms / 1e6, 1))  # GB/s
    del t
    return out


def cpu_stat():
    """cgroup CPU throttling counters (cgroup v2 cpu.stat, or v1 cpu.stat) - a process whose
    cgroup exceeds its CPU quota is frozen for the rest of the period, and the GPU idles."""
    for f in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat",
              "/sys/fs/cgroup/cpu,cpuacct/cpu.stat"):
        try:
            out = {}
            for line in open(f):
                k, v = line.split()
                out[k] = int(v)
            return out
        except (OSError, ValueError):
            continue
    return {}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    name = sys.argv[3] if len(sys.argv) > 3 else "squeezenet"
    static = len(sys.argv) > 4 and sys.argv[4] == "1"
    from mpi_pytorch_amd.parallel import init_world
    from mpi_pytorch_amd.engine import build_training
    from mpi_pytorch_amd.data import DevicePrefetcher
    from mpi_pytorch_amd.models import input_spec

    t0 = time.time()
    world = init_world("cuda")
    torch.manual_seed(0)
    dev = world.device
    model, opt, step, _ = build_training(name, 64500, dev, world, 4e-4, "adam")
    hw = (224, 224)
    spec = input_spec(model, hw)
    data = DevicePrefetcher(dev, B, hw, hw, 64500, seed=1234, rank=0, world=1, depth=4,
                            threads=4, cpad=spec["cpad"], pad=spec["pad"])
    if static:
        xs, ys = data.next()
        data.next = lambda: (xs, ys)
    for _ in range(3):
        x, y = data.next()
        step(x, y)
    torch.cuda.synchronize()
    timer = step.enable_timers()
    keys = ("num_alloc_retries", "num_device_alloc", "num_device_free", "num_sync_all_streams")
    st0 = torch.cuda.memory_stats()
    cs0 = cpu_stat()
    host_ms = []
    a, b = _ev(), _ev()
    a.record()
    for _ in range(steps):
        h0 = time.perf_counter()
        x, y = data.next()
        step(x, y)
        host_ms.append(round((time.perf_counter() - h0) * 1e3, 2))
    b.record()
    b.synchronize()
    st1 = torch.cuda.memory_stats()
    cs1 = cpu_stat()
    cpu_delta = {k: cs1[k] - cs0.get(k, 0) for k in cs1}
    alloc_delta = {k: st1.get(k, 0) - st0.get(k, 0) for k in keys}
    ms_step = a.elapsed_time(b) / steps
    phases = timer.summary()

    # per-module forward times of one more step
    recs = []
    leaves = [(n, m) for n, m in model.named_modules() if not list(m.children())]

    def pre(mod, inp):
        e = _ev()
        e.record()
        mod._probe_t0 = e

    def post(mod, inp, out):
        e = _ev()
        e.record()
        recs.append((mod._probe_name, mod._probe_t0, e))

    hooks = []
    for n, m in leaves:
        m._probe_name = n
        hooks.append(m.register_forward_pre_hook(pre))
        hooks.append(m.register_forward_hook(post))
    # ... and per autograd node of its backward (node pre / post hooks: compute-stream time
    # between a node's start and end; side-stream weight gradients are not in it)
    brecs = []
    orig_backward = torch.Tensor.backward

    def backward_hooked(self, *a, **k):
        seen, todo, idx = set(), [self.grad_fn], 0
        while todo:
            node = todo.pop()
            if node is None or node in seen:
                continue
            seen.add(node)
            idx += 1
            tag = "%s#%d" % (type(node).__name__, idx)

            def npre(go, tag=tag):
                e = _ev()
                e.record()
                brecs.append([tag, e, None])

            def npost(gi, go, tag=tag):
                e = _ev()
                e.record()
                for r in reversed(brecs):
                    if r[0] == tag:
                        r[2] = e
                        break

            node.register_prehook(npre)
            node.register_hook(npost)
            todo.extend(f for f, _ in node.next_functions)
        return orig_backward(self, *a, **k)

    torch.Tensor.backward = backward_hooked
    try:
        x, y = data.next()
        step(x, y)
        torch.cuda.synchronize()
    finally:
        torch.Tensor.backward = orig_backward
    for h in hooks:
        h.remove()
    mods = sorted(((round(s.elapsed_time(e), 3), n) for n, s, e in recs), reverse=True)[:10]
    bnodes = sorted(((round(s.elapsed_time(e), 3), n) for n, s, e in brecs if e is not None),
                    reverse=True)[:10]

    st = torch.cuda.memory_stats()
    rec = {
        "model": name, "static": static, "batch": B, "ms_per_step": round(ms_step, 3), "img_per_s": round(B / ms_step * 1e3, 1),
        "phases_ms": {k: phases[k] for k in ("forward", "backward", "optimizer")},
        "host_enqueue_ms": host_ms,
        "allocator_delta": alloc_delta,
        "cgroup_cpu_delta": cpu_delta,
        "threads": len(os.listdir("/proc/self/task")),
        "cpus_allowed": len(os.sched_getaffinity(0)),
        "top_forward_modules_ms": mods,
        "top_backward_nodes_ms": bnodes,
        "alloc_gb": round(st.get("allocated_bytes.all.peak", 0) / 1e9, 2),
        "segments": st.get("segment.all.current", 0),
        "bw_fresh_11gb_GBps": bw_probe(11_200_000_000),
        "bw_fresh_256mb_GBps": bw_probe(256 << 20),
        "tune": os.environ.get("MPA_TUNE", "1"),
        "wall_s": round(time.time() - t0, 1),
    }
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
