"""End-to-end model parity on the GPU: the native bf16 path vs the fp32 CPU path with
identical weights and inputs (loss, gradient arena, one optimizer step), per model."""
import copy

import pytest
import torch

from mpi_pytorch_amd.engine import build_model, loss_fn
from mpi_pytorch_amd.parallel import World
from mpi_pytorch_amd.optim import build_optimizer

pytestmark = pytest.mark.gpu


def _pair(name, nc, gpu):
    torch.manual_seed(0)
    w = World()
    mc, _ = build_model(name, nc, False, torch.device("cpu"), w)
    mg, _ = build_model(name, nc, False, gpu, w)
    mg.load_state_dict(mc.state_dict())
    mg._mpa_arena.sync_shadow()
    return mc, mg


@pytest.mark.parametrize("name,hw", [("resnet18", 64), ("resnet34", 64), ("vgg", 64),
                                     ("alexnet", 127), ("squeezenet", 96), ("densenet", 64),
                                     ("inception", 299), ("vgg16", 64)])
def test_model_parity(gpu, name, hw):
    nc = 40
    mc, mg = _pair(name, nc, gpu)
    torch.manual_seed(1)
    B = 4
    x = torch.randn(B, hw, hw, 3) * 0.5
    y = torch.randint(0, nc, (B,))
    # dropout layers draw different masks on CPU/GPU: compare in a dropout-free setting
    for m in (mc, mg):
        for mod in m.modules():
            if type(mod).__name__ == "Dropout":
                mod.p = 0.0
    lc = loss_fn(mc(x), y)
    lc.backward()
    lg = loss_fn(mg(x.to(gpu).to(torch.bfloat16)), y.to(gpu))
    lg.backward()
    torch.cuda.synchronize()
    assert abs(float(lc) - float(lg)) < 0.05 * max(1.0, abs(float(lc))), (float(lc), float(lg))
    gc = mc._mpa_arena.grad
    gg = mg._mpa_arena.grad.cpu()
    ratio = float(gg.norm() / gc.norm())
    assert 0.8 < ratio < 1.25, ratio
    # The whole-model gradient DIRECTION of a deep BN net at init is chaotic w.r.t.
    # rounding - the fp32 CPU path alone moves to cos 0.39 (Inception) / 0.90 (DenseNet)
    # when only the input image is rounded to bf16
    # (test_models_cpu.py::test_whole_model_gradients_are_shattered_in_fp32) - so no tight
    # whole-model bound exists; per-unit parity (test_layer_parity_gpu.py, cos >= 0.99 for
    # every block / layer) is the real check.  What IS well conditioned end to end: the
    # classifier head's gradient (features x softmax error, no deep backward behind it).
    # (The final classifier weight; Inception's auxiliary head has BN'd convs of its own
    # and gets the looser bound with the rest of the head.)
    from mpi_pytorch_amd.models import head_parameters
    pc = [p.grad for p in head_parameters(mc) if p.grad is not None]
    pg = [p.grad.cpu() for p in head_parameters(mg) if p.grad is not None]
    cos = torch.nn.functional.cosine_similarity

    def final(m):
        main = getattr(m, "fc", None) or getattr(m, "classifier")
        return [q for q in main.parameters() if q.dim() >= 2][-1].grad

    fcos = float(cos(final(mc).reshape(-1), final(mg).cpu().reshape(-1), dim=0))
    hcos = float(cos(torch.cat([t.reshape(-1) for t in pc]),
                     torch.cat([t.reshape(-1) for t in pg]), dim=0))
    assert fcos > 0.99 and hcos > 0.95, (fcos, hcos)


def test_resnet18_training_decreases_loss(gpu):
    torch.manual_seed(0)
    w = World()
    m, _ = build_model("resnet18", 100, False, gpu, w)
    opt = build_optimizer("adam", m, 1e-3)
    x = (torch.randn(16, 64, 64, 3, device=gpu) * 0.5).to(torch.bfloat16)
    y = torch.randint(0, 100, (16,), device=gpu)
    losses = []
    for _ in range(12):
        m._mpa_arena.zero_grad()
        loss = loss_fn(m(x), y)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert losses[-1] < losses[0] * 0.5, losses


def test_step_phase_timers(gpu):
    """StepTimer (engine/step.py): HIP-event phase times of eager steps resolve without a
    per-step sync, every phase is non-negative, the compute phases are positive, and the
    phase sum tracks the host wall clock of the same steps."""
    import time
    from mpi_pytorch_amd.optim import build_optimizer as bo
    from mpi_pytorch_amd.engine.step import TrainStep
    torch.manual_seed(0)
    w = World(device=gpu)
    m, _ = build_model("resnet18", 100, False, gpu, w)
    step = TrainStep(m, bo("adam", m, 1e-3), w)
    x = (torch.randn(16, 64, 64, 3, device=gpu) * 0.5).to(torch.bfloat16)
    y = torch.randint(0, 100, (16,), device=gpu)
    step(x, y)
    t = step.enable_timers()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        step(x, y)
    torch.cuda.synchronize()
    wall_ms = (time.perf_counter() - t0) * 1e3 / 5
    s = t.summary()
    assert s["steps"] == 5
    assert all(s[k] >= 0.0 for k in t.PHASES)
    assert s["forward"] > 0 and s["backward"] > 0 and s["optimizer"] > 0
    assert 0.3 * wall_ms < s["step"] < 1.5 * wall_ms, (s, wall_ms)
    assert t.summary()["steps"] == 0  # reset
