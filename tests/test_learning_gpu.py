"""The engine learns, checked the way the reference checks itself: training-set accuracy
rising over epochs (``/root/reference/training.log:1040-1112``, produced by
``main.py:142-185``: train epochs, rank-0 eval-mode accuracy on the training sample).

ResNet-18 through the training driver (``run_training``: native ring-free device
synthetic images, bf16 MFMA kernels, fused Adam lr 4e-4, BN running statistics, eval-mode
BN for the accuracy, per-epoch checkpoint), 256 synthetic 64x64 images over 1,000
classes, batch 64: it must memorise the sample (eval accuracy >= 0.95), and a resume from
the checkpoint must continue the curve (accuracy stays, loss keeps falling).  Eager and
HIP-graph-replayed steps alike (graph mode replays one captured step ~80 times).
Parity with the reference's own numbers stays unpinned: those used pretrained weights
and real Herbarium images, neither of which exists offline."""
import pytest

from mpi_pytorch_amd.config import Config

pytestmark = pytest.mark.gpu


def _reset_world():
    import mpi_pytorch_amd.parallel.dist as D
    D._WORLD = None


@pytest.mark.parametrize("graph", ["off", "on"])
def test_resnet18_memorises_then_resumes(gpu, tmp_path, graph):
    from mpi_pytorch_amd.engine.trainer import run_training
    kw = dict(synthetic_images=256, image_size=64, NUM_CLASSES=1000, BATCH_SIZE=64, LR=4e-4,
              device="cuda", graph=graph, CHECKPOINT_DIR=str(tmp_path) + "/ck/",
              log_file=str(tmp_path / "training.log"), watchdog_s=0)
    _reset_world()
    out = run_training(Config(NUM_EPOCHS=20, **kw))
    h = out["history"]
    losses = [r["train_loss"] for r in h]
    accs = [r["acc"] for r in h]
    print("losses", [round(v, 3) for v in losses])
    print("accs", accs)
    assert losses[0] > 6.0  # ~ln(1000) at init
    assert losses[-1] < 0.1 * losses[0]
    assert accs[-1] >= 0.95 and accs[0] < 0.5
    _reset_world()
    out2 = run_training(Config(NUM_EPOCHS=23, FROM_CHECKPOINT=True, **kw))
    h2 = out2["history"]
    assert [r["epoch"] for r in h2] == [20, 21, 22]
    assert all(r["acc"] >= 0.95 for r in h2)
    assert h2[-1]["train_loss"] < 1.5 * losses[-1] + 0.05
