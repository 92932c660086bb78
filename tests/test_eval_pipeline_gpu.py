"""The HIP-stream evaluation pipeline on the GPU (reference: the 4-stage MPMD pipeline of
``/root/reference/evaluation_pipeline.py:44-199``).

Stage 0 is the native ``BatchRing`` (window mode: C++ threads copy each manifest row's
synthetic image into pinned slots; external mode: PIL decode threads write JPEGs into a
slot at their own extents), then copy stream -> preprocess stream (PIL-exact kernels) ->
predictor lanes.  For every lane count and assignment policy the correct count must equal
a plain, non-pipelined batched evaluation of the same images EXACTLY."""
import os

import numpy as np
import pytest
import torch

from mpi_pytorch_amd.data.manifest import SyntheticImages, FolderImages
from mpi_pytorch_amd.engine import build_training
from mpi_pytorch_amd.engine.eval_pipeline import StreamPipeline, plain_eval, make_ring, _batches
from mpi_pytorch_amd.parallel import World

pytestmark = pytest.mark.gpu
NC = 10


@pytest.fixture(scope="module")
def model(gpu):
    torch.manual_seed(0)
    m, _opt, _step, _ = build_training("resnet18", NC, gpu, World(device=gpu), 1e-3)
    m.eval()
    return m


def _manifest(n, seed=0):
    names = ["synthetic/%05d.jpg" % i for i in range(n)]
    labels = list(np.random.default_rng(seed).integers(0, NC, size=n))
    return names, labels


@pytest.mark.parametrize("lanes,assign", [(1, "random"), (3, "random"), (3, "roundrobin")])
def test_ring_pipeline_equals_plain_eval(gpu, model, lanes, assign):
    names, labels = _manifest(203)  # a short last batch
    src = SyntheticImages((96, 80))
    ref = plain_eval(model, names, labels, 16, src, gpu, (64, 64))
    ring, nb = make_ring(names, labels, 16, src, NC, depth=4, threads=3)
    try:
        pipe = StreamPipeline(model, gpu, (64, 64), lanes=lanes, assign=assign)
        counts = pipe.run_ring(ring, nb)
    finally:
        ring.stop()
    assert sum(counts) == ref
    assert sum(pipe.seen) == len(names)
    assert ref > 0  # a non-trivial comparison (random labels over 10 classes)


def test_host_batches_pipeline_equals_plain_eval(gpu, model):
    names, labels = _manifest(70, seed=1)
    src = SyntheticImages((64, 64))
    ref = plain_eval(model, names, labels, 16, src, gpu, (64, 64))
    pipe = StreamPipeline(model, gpu, (64, 64), lanes=2, assign="roundrobin")
    assert sum(pipe.run(_batches(names, labels, 16, src))) == ref


def test_ring_orders_batches_and_short_tail(gpu):
    """Window mode: batches arrive in index order whatever thread filled them, with the
    manifest's labels, the texture windows of SyntheticImages bit for bit, a short last
    batch and full extents."""
    names, labels = _manifest(50, seed=2)
    src = SyntheticImages((24, 40))
    ring, nb = make_ring(names, labels, 8, src, NC, depth=3, threads=4)
    try:
        assert nb == 7
        for bi in range(nb):
            slot, img, lab, idx = ring.acquire()
            n, ext = ring.info(slot)
            lo = bi * 8
            assert idx == bi and n == min(8, 50 - lo)
            assert np.array_equal(img.numpy()[:n], src.load(names[lo:lo + n]))
            assert lab.numpy()[:n].tolist() == [int(v) for v in labels[lo:lo + n]]
            assert (ext.numpy()[:n] == [24, 40]).all()
            ring.release(slot)
    finally:
        ring.stop()


def test_real_jpeg_ring_pipeline(gpu, model, tmp_path):
    """External mode: PIL decode threads write JPEGs of different sizes into padded slots;
    the pipeline's accuracy equals the plain evaluation of the same files."""
    from PIL import Image
    rng = np.random.default_rng(3)
    names, labels = [], []
    for i in range(37):
        h, w = int(rng.integers(40, 120)), int(rng.integers(40, 120))
        arr = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        name = "img%03d.jpg" % i
        Image.fromarray(arr).save(os.path.join(tmp_path, name), quality=90)
        names.append(name)
        labels.append(int(rng.integers(0, NC)))
    src = FolderImages(str(tmp_path), 2)
    ref = plain_eval(model, names, labels, 8, src, gpu, (64, 64))
    ring, nb = make_ring(names, labels, 8, src, NC, depth=3, threads=3, pitch=(120, 120))
    try:
        pipe = StreamPipeline(model, gpu, (64, 64), lanes=2, assign="random")
        counts = pipe.run_ring(ring, nb)
    finally:
        ring.stop()
    assert sum(counts) == ref and sum(pipe.seen) == 37


def test_real_jpeg_ring_many_threads_small_ring(gpu, model, tmp_path):
    """More decode threads than free slots (depth 2, 6 threads, 40 batches): a thread owns a
    slot before it takes a batch index, so the thread holding the next index can always
    commit (the old index-first order could park it behind later batches and hang)."""
    from PIL import Image
    rng = np.random.default_rng(5)
    names, labels = [], []
    for i in range(80):
        arr = rng.integers(0, 256, (int(rng.integers(30, 70)), int(rng.integers(30, 70)), 3),
                           dtype=np.uint8)
        names.append("s%03d.png" % i)
        Image.fromarray(arr).save(os.path.join(tmp_path, names[-1]))
        labels.append(int(rng.integers(0, NC)))
    src = FolderImages(str(tmp_path), 2)
    ref = plain_eval(model, names, labels, 2, src, gpu, (64, 64))
    ring, nb = make_ring(names, labels, 2, src, NC, depth=2, threads=6, pitch=(70, 70))
    try:
        pipe = StreamPipeline(model, gpu, (64, 64), lanes=2, assign="roundrobin")
        counts = pipe.run_ring(ring, nb)
    finally:
        ring.stop()
    assert sum(counts) == ref and sum(pipe.seen) == 80


def test_real_jpeg_ring_decode_error_raises(gpu, model, tmp_path):
    """A file PIL cannot decode stops the ring: the consumer raises instead of waiting for
    a batch that never comes, and feed_error names the decode failure."""
    from PIL import Image
    from mpi_pytorch_amd.engine.eval_pipeline import feed_error
    names = []
    for i in range(12):
        names.append("e%02d.png" % i)
        if i == 7:
            (tmp_path / names[-1]).write_bytes(b"not an image")
        else:
            Image.fromarray(np.zeros((20, 20, 3), np.uint8)).save(os.path.join(tmp_path, names[-1]))
    src = FolderImages(str(tmp_path), 1)
    ring, nb = make_ring(names, [0] * 12, 4, src, NC, depth=2, threads=2, pitch=(20, 20))
    try:
        pipe = StreamPipeline(model, gpu, (64, 64), lanes=1)
        with pytest.raises(RuntimeError):
            pipe.run_ring(ring, nb)
        assert feed_error(ring) is not None
    finally:
        ring.stop()


@pytest.mark.parametrize("name,hw,src", [("inception", 299, 340), ("densenet", 224, 256)])
def test_zoo_ring_pipeline_equals_plain_eval(gpu, name, hw, src):
    """The reference predicts with whichever MODEL_NAME was trained
    (``/root/reference/evaluation_pipeline.py:138-144``): Inception-v3 at 299 (BASELINE
    config 5 names it with the HIP-stream pipeline) and DenseNet-121 at 224, 2 predictor
    lanes, PIL-exact bicubic from larger sources - equal to the plain evaluation."""
    torch.manual_seed(0)
    m, _opt, _step, _ = build_training(name, NC, gpu, World(device=gpu), 1e-3)
    m.eval()
    names, labels = _manifest(37, seed=7)
    source = SyntheticImages((src, src))
    ref = plain_eval(m, names, labels, 8, source, gpu, (hw, hw))
    ring, nb = make_ring(names, labels, 8, source, NC, depth=3, threads=2)
    try:
        pipe = StreamPipeline(m, gpu, (hw, hw), lanes=2, assign="roundrobin")
        counts = pipe.run_ring(ring, nb)
    finally:
        ring.stop()
    assert sum(counts) == ref and sum(pipe.seen) == 37
