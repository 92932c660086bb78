"""Deterministic mode (MPA_DETERMINISTIC / ``_ext.set_deterministic``): fixed-order
cross-block reductions and no timing-based tile autotuning make a training step a pure
function of its inputs, so

* two identical steps from identical state are bitwise equal (loss, gradient arena,
  updated weights), and
* back-to-back HIP-graph replays of the whole step are bitwise equal to the same number of
  eager steps (docs/NOTES.md "HIP graph replay").

The reference has no GPU path; its per-step semantics (fwd -> CE -> backward -> Adam,
``/root/reference/main.py:142-156``) are what both runs execute."""
import pytest
import torch

from mpi_pytorch_amd.engine import build_training
from mpi_pytorch_amd.parallel import World

pytestmark = pytest.mark.gpu


@pytest.fixture
def det(gpu):
    from mpi_pytorch_amd.ops import _ext
    C = _ext.ext()
    old = C.deterministic()
    C.set_deterministic(1)
    yield gpu
    C.set_deterministic(int(old))


def _train(gpu, seed=0, name="resnet18", nc=100):
    torch.manual_seed(seed)
    w = World(device=gpu)
    model, opt, step, _ = build_training(name, nc, gpu, w, 1e-3)
    return model, opt, step


def _batch(gpu, B=32, hw=64, nc=100, seed=1):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = (torch.randn(B, hw, hw, 8, generator=g) * (torch.arange(8) < 3)).to(gpu, torch.bfloat16)
    y = torch.randint(0, nc, (B,), generator=g).to(gpu)
    return x, y


def test_two_identical_steps_bitwise(det):
    gpu = det
    x, y = _batch(gpu)
    outs = []
    for _ in range(2):
        model, opt, step = _train(gpu)
        losses = [step(x, y).clone() for _ in range(3)]
        torch.cuda.synchronize()
        a = model._mpa_arena
        outs.append((torch.stack(losses).cpu(), a.grad.cpu().clone(), a.master.cpu().clone(),
                     opt.exp_avg_sq.cpu().clone()))
    for u, v in zip(outs[0], outs[1]):
        assert torch.equal(u, v)


def test_graph_replays_bitwise_equal_eager(det):
    """100 back-to-back replays (no host sync between them) == 100 eager steps."""
    gpu = det
    x, y = _batch(gpu)
    n = 100
    # eager (capture's own warm-up steps are rolled back: TrainStep.capture)
    model, opt, step = _train(gpu)
    ref = torch.stack([step(x, y).clone() for _ in range(n)])
    torch.cuda.synchronize()
    ref_master = model._mpa_arena.master.clone()
    del model, opt, step
    model, opt, step = _train(gpu)
    assert step.capture(x, y, warmup=2)
    got = torch.stack([step(x, y).clone() for _ in range(n)])
    torch.cuda.synchronize()
    bad = (got != ref).nonzero()
    assert bad.numel() == 0, "first diverging replay %d: %s vs %s" % (
        int(bad[0]), float(got[bad[0]]), float(ref[bad[0]]))
    assert torch.equal(model._mpa_arena.master, ref_master)


@pytest.mark.parametrize("name,hw", [("resnet18", 64), ("vgg16", 64), ("densenet", 64),
                                     ("inception", 299)])
def test_wgrad_side_stream_bitwise(det, name, hw):
    """Conv weight gradients on the side stream (MPA_WGRAD_STREAM, joined before the
    optimizer) == all on one stream, bitwise, over 3 steps (losses, weights, Adam state)."""
    gpu = det
    import mpi_pytorch_amd.ops.functional as Fn
    x, y = _batch(gpu, B=8 if hw > 200 else 32, hw=hw)
    outs = []
    old = Fn._WGRAD_STREAM
    try:
        for on in (True, False):
            Fn._WGRAD_STREAM = on
            model, opt, step = _train(gpu, name=name)
            for mod in model.modules():  # (the dropout stream advances across the runs)
                if type(mod).__name__ == "Dropout":
                    mod.p = 0.0
            losses = [step(x, y).clone() for _ in range(3)]
            torch.cuda.synchronize()
            if on:
                assert Fn._SIDE["stream"] is not None
            a = model._mpa_arena
            outs.append((torch.stack(losses).cpu(), a.master.cpu().clone(),
                         opt.exp_avg_sq.cpu().clone()))
            del model, opt, step
    finally:
        Fn._WGRAD_STREAM = old
    for u, v in zip(outs[0], outs[1]):
        assert torch.equal(u, v)


def test_branch_stream_bitwise(det):
    """Inception side-branch chains on the branch stream (MPA_BRANCH_STREAM: forward and,
    through autograd, backward) == every branch on one stream, bitwise, over 3 steps."""
    gpu = det
    import mpi_pytorch_amd.ops.functional as Fn
    x, y = _batch(gpu, B=8, hw=299)
    outs = []
    old = Fn._BRANCH_STREAM
    try:
        for on in (True, False):
            Fn._BRANCH_STREAM = on
            Fn._BR["stream"] = None
            model, opt, step = _train(gpu, name="inception")
            for mod in model.modules():
                if type(mod).__name__ == "Dropout":
                    mod.p = 0.0
            losses = [step(x, y).clone() for _ in range(3)]
            torch.cuda.synchronize()
            assert (Fn._BR["stream"] is not None) == on
            a = model._mpa_arena
            outs.append((torch.stack(losses).cpu(), a.master.cpu().clone(),
                         opt.exp_avg_sq.cpu().clone(),
                         torch.cat([b.float().flatten().cpu() for b in model.buffers()])))
            del model, opt, step
    finally:
        Fn._BRANCH_STREAM = old
    for u, v in zip(outs[0], outs[1]):
        assert torch.equal(u, v)


def test_graph_replay_bitwise_with_headline_head(det):
    """With the headline's 64,500-class head (75 % of ResNet-18's parameters), 10 replays
    of a captured step == 10 eager steps, bitwise (losses and master weights)."""
    gpu = det
    nc = 64500
    x, y = _batch(gpu, B=16, hw=32, nc=nc)
    model, opt, step = _train(gpu, nc=nc)
    ref = torch.stack([step(x, y).clone() for _ in range(10)])
    torch.cuda.synchronize()
    ref_master = model._mpa_arena.master.clone()
    del model, opt, step
    model, opt, step = _train(gpu, nc=nc)
    assert step.capture(x, y, warmup=2)
    got = torch.stack([step(x, y).clone() for _ in range(10)])
    torch.cuda.synchronize()
    assert torch.equal(got, ref) and torch.equal(model._mpa_arena.master, ref_master)


def test_dropout_graph_replays_draw_fresh_masks(gpu):
    """Dropout's stream position lives in a device counter that the captured graph reads
    and advances: two replays of the same captured dropout draw different masks (a
    host-side offset would be frozen into the graph - one mask for every replay)."""
    from mpi_pytorch_amd.ops import functional as Fn
    x = torch.ones(64, 1024, device=gpu, dtype=torch.bfloat16)
    Fn.dropout(x, 0.5, True)  # (warm the kernel outside capture)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = Fn.dropout(x, 0.5, True)
    masks = []
    for _ in range(3):
        g.replay()
        masks.append((y != 0).clone())
    torch.cuda.synchronize()
    assert not torch.equal(masks[0], masks[1]) and not torch.equal(masks[1], masks[2])
    for m in masks:  # still Bernoulli(0.5)
        assert 0.45 < m.float().mean().item() < 0.55
    # eager calls advance the same counter: two eager draws differ as well
    a, b = Fn.dropout(x, 0.5, True), Fn.dropout(x, 0.5, True)
    assert not torch.equal(a, b)


@pytest.mark.parametrize("name,hw,B", [("alexnet", 64, 16), ("inception", 299, 4),
                                       ("densenet", 64, 8)])
def test_dropout_models_graph_replays_bitwise_equal_eager(det, name, hw, B):
    """Models with dropout (torchvision classifiers of AlexNet / Inception,
    ``/root/reference/models.py:50,87``): replays of a captured step equal eager steps
    bitwise in deterministic mode - every replay draws the mask the eager step would."""
    from mpi_pytorch_amd.ops import functional as Fn
    gpu = det
    x, y = _batch(gpu, B=B, hw=hw, nc=100, seed=3)
    n = 6
    rng0 = Fn.DropoutRNG.state()
    model, opt, step = _train(gpu, name=name, nc=100)
    ref = torch.stack([step(x, y).clone() for _ in range(n)])
    torch.cuda.synchronize()
    ref_master = model._mpa_arena.master.clone()
    del model, opt, step
    Fn.DropoutRNG.set_state(rng0)
    model, opt, step = _train(gpu, name=name, nc=100)
    assert step.capture(x, y, warmup=2)
    got = torch.stack([step(x, y).clone() for _ in range(n)])
    torch.cuda.synchronize()
    assert torch.equal(got, ref), (got, ref)
    assert torch.equal(model._mpa_arena.master, ref_master)
