"""Evaluation-pipeline throughput (reference: evaluation_pipeline.py's read -> resize ->
normalize -> predict stages; ResNet-18, 64,500 classes, 128x128 inputs, utils.py:33-39).

    python tools/bench_eval.py [images=40000] [batch=256] [lanes=1,2,4] [src=256]

Synthetic manifest rows -> native ring (window mode, C++ copy threads) -> H2D copy stream ->
PIL-exact bicubic preprocess (src x src -> 128 x 128) -> predictor lanes.  Prints one JSON
line per lane count: images/s over the whole pipeline (first pass excluded: warm-up)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from mpi_pytorch_amd.data.manifest import SyntheticImages
from mpi_pytorch_amd.engine import build_training
from mpi_pytorch_amd.engine.eval_pipeline import StreamPipeline, make_ring
from mpi_pytorch_amd.parallel import World

N = int(sys.argv[1]) if len(sys.argv) > 1 else 40000
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
LANES = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "1,2,4").split(",")]
SRC = int(sys.argv[4]) if len(sys.argv) > 4 else 256
MODEL = os.environ.get("MODEL", "resnet18")
HW = int(os.environ.get("HW", "128"))
NC = 64500
gpu = torch.device("cuda", 0)
torch.manual_seed(0)
model = build_training(MODEL, NC, gpu, World(device=gpu), 1e-3)[0]
model.eval()
names = ["synthetic/%07d.jpg" % i for i in range(N)]
labels = np.random.default_rng(0).integers(0, NC, size=N)
src = SyntheticImages((SRC, SRC))
threads = int(os.environ.get("THREADS", "8"))
for lanes in [LANES[0]] + LANES:  # first run: warm-up (tuning, allocator)
    ring, nb = make_ring(names, labels, B, src, NC, depth=8, threads=threads)
    pipe = StreamPipeline(model, gpu, (HW, HW), lanes=lanes, assign="roundrobin")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    counts = pipe.run_ring(ring, nb)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ring.stop()
    print(json.dumps({"metric": "eval pipeline images/s", "model": MODEL, "image": HW,
                      "src": SRC, "batch": B, "lanes": lanes, "images": N,
                      "img_per_s": round(N / dt, 1), "seconds": round(dt, 3),
                      "correct": int(sum(counts)), "ring_threads": threads}), flush=True)
