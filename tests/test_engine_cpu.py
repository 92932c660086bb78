"""Engine plumbing on CPU: config, checkpoint format contract, training driver (BASELINE
config 1 style), resume, evaluation pipeline vs plain eval, dataset builder, launcher."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from mpi_pytorch_amd.config import Config
from mpi_pytorch_amd.checkpoint import save_checkpoint, load_checkpoint, build_state, read_checkpoint
from mpi_pytorch_amd.engine import build_training
from mpi_pytorch_amd.parallel import World

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _reset_world():
    import mpi_pytorch_amd.parallel.dist as D
    D._WORLD = None


def test_config_fields_and_overrides(monkeypatch):
    c = Config()
    assert (c.MODEL_NAME, c.BATCH_SIZE, c.LR, c.NUM_CLASSES, c.NUM_EPOCHS) == \
        ("resnet18", 128, 4e-4, 64500, 10)
    assert c.CHECKPOINT_NAME == "checkpoint_resnet18.pt"
    monkeypatch.setenv("MPA_BATCH_SIZE", "64")
    c = Config.from_args(["--MODEL_NAME", "resnet34", "--lr", "0.01", "--DEBUG", "false"])
    assert c.MODEL_NAME == "resnet34" and c.BATCH_SIZE == 64 and c.LR == 0.01 and not c.DEBUG
    assert c.CHECKPOINT_NAME == "checkpoint_resnet34.pt"
    with pytest.raises(ValueError):
        Config(MODEL_NAME="lenet")
    # entry-point defaults (evaluation_pipeline.py: log_file) yield to explicit flags
    assert Config.from_args([], log_file="evaluation.log").log_file == "evaluation.log"
    assert Config.from_args(["--log_file", "x.log"], log_file="evaluation.log").log_file == "x.log"


def test_utils_shim():
    sys.path.insert(0, ROOT)
    import utils
    assert utils.MODEL_NAME == "resnet18" and utils.WIDTH == 128 and utils.NUM_CLASSES == 64500


def test_checkpoint_contract(tmp_path):
    model, opt, step, _ = build_training("resnet18", 100, torch.device("cpu"), World(), 4e-4)
    x = torch.randn(4, 32, 32, 3)
    y = torch.randint(0, 100, (4,))
    step(x, y)
    path = save_checkpoint(build_state(3, model, opt, 1.5), 3, "resnet18", str(tmp_path) + "/")
    assert os.path.basename(path) == "checkpoint_resnet18.pt"
    ck = read_checkpoint(path)
    assert set(ck) == {"epoch", "state_dict", "optimizer", "loss"}
    assert ck["epoch"] == 3 and ck["loss"] == 1.5
    assert ck["state_dict"]["conv1.weight"].shape == (64, 3, 7, 7)
    assert ck["state_dict"]["conv1.weight"].dtype == torch.float32
    st = ck["optimizer"]["state"]
    assert set(st[0]) == {"step", "exp_avg", "exp_avg_sq"}
    assert st[0]["exp_avg"].shape == (64, 3, 7, 7)
    pg = ck["optimizer"]["param_groups"][0]
    assert pg["lr"] == 4e-4 and pg["betas"] == (0.9, 0.999)
    # loadable into torch.optim.Adam over torchvision-shaped params
    names = [n for n, _ in model.named_parameters()]
    params = [torch.nn.Parameter(ck["state_dict"][n].clone()) for n in names]
    topt = torch.optim.Adam(params, lr=4e-4)
    topt.load_state_dict(ck["optimizer"])
    # round trip into a fresh engine model/optimizer
    m2, o2, s2, _ = build_training("resnet18", 100, torch.device("cpu"), World(), 4e-4)
    _m, _o, ep = load_checkpoint(path, m2, o2)
    assert ep == 3
    for k, v in m2.state_dict().items():
        assert torch.equal(v, ck["state_dict"][k]), k
    assert float(o2.step_t) == float(opt.step_t)
    assert torch.allclose(o2.exp_avg, opt.exp_avg)
    # an identical next step from both
    l1 = float(step(x, y))
    l2 = float(s2(x, y))
    assert abs(l1 - l2) < 1e-5


def test_sgd_state_dict_roundtrip():
    model, opt, step, _ = build_training("squeezenet", 10, torch.device("cpu"), World(), 0.1,
                                         optimizer="sgd")
    step(torch.randn(2, 64, 64, 3), torch.randint(0, 10, (2,)))
    sd = opt.state_dict()
    assert "momentum_buffer" in sd["state"][0]
    params = [torch.nn.Parameter(p.detach().clone()) for p in model.parameters()]
    torch.optim.SGD(params, lr=0.1, momentum=0.9).load_state_dict(sd)


def test_training_driver_cpu(tmp_path):
    _reset_world()
    from mpi_pytorch_amd.engine.trainer import run_training
    log = tmp_path / "training.log"
    cfg = Config(synthetic_images=32, image_size=64, NUM_EPOCHS=2, BATCH_SIZE=16,
                 CHECKPOINT_DIR=str(tmp_path) + "/ck/", device="cpu", log_file=str(log),
                 metrics_jsonl=str(tmp_path / "m.jsonl"))
    out = run_training(cfg)
    text = log.read_text()
    for s in ("INFO:Herbarium_R0:Logger Initialized", "_Files Received: 32",
              "_Training Dataset Object Created", "_Model Created: resnet18",
              "_Optimizer Created", "_Entering training Loop", "_Epoch: 0 | Train Loss: ",
              "_Creating a checkpoint at epoch 1", "_Checkpoint saved", "_Evaluating model",
              "_Epoch: 1 | Acc: ", "INFO:Herbarium_R0:_Model loaded to CPU\n"):
        assert s in text, s
    recs = [json.loads(l) for l in (tmp_path / "m.jsonl").read_text().splitlines()]
    assert len(recs) == 2 and recs[1]["train_loss"] < recs[0]["train_loss"]
    assert os.path.exists(out["checkpoint"])
    # resume continues at saved epoch + 1
    _reset_world()
    cfg2 = Config(synthetic_images=32, image_size=64, NUM_EPOCHS=3, BATCH_SIZE=16,
                  CHECKPOINT_DIR=str(tmp_path) + "/ck/", device="cpu", log_file=str(log),
                  FROM_CHECKPOINT=True)
    out2 = run_training(cfg2)
    assert [h["epoch"] for h in out2["history"]] == [2]


def test_training_driver_debug_manifest(tmp_path):
    _reset_world()
    from mpi_pytorch_amd.engine.trainer import run_training
    cfg = Config(DEBUG=True, DEBUG_SAMPLE=40, TEST_CSV=os.path.join(ROOT, "data", "test_sample.csv"),
                 image_size=32, NUM_EPOCHS=1, BATCH_SIZE=16, VALIDATE=False,
                 CHECKPOINT_DIR=str(tmp_path) + "/", device="cpu", log_file=str(tmp_path / "l"))
    out = run_training(cfg)
    assert "_Files Received: 32" in (tmp_path / "l").read_text()  # 80 % of 40


@pytest.mark.parametrize("lanes,assign", [(1, "random"), (3, "random"), (2, "roundrobin")])
def test_eval_pipeline_matches_plain_eval(tmp_path, lanes, assign):
    from mpi_pytorch_amd.engine.eval_pipeline import StreamPipeline, plain_eval, _batches
    from mpi_pytorch_amd.data.manifest import SyntheticImages
    model, opt, step, _ = build_training("resnet18", 5, torch.device("cpu"), World(), 1e-3)
    src = SyntheticImages((40, 40))
    names = ["img/%d.jpg" % i for i in range(30)]
    labels = list(np.random.default_rng(0).integers(0, 5, size=30))
    model.eval()
    ref = plain_eval(model, names, labels, 8, src, torch.device("cpu"), (32, 32))
    pipe = StreamPipeline(model, torch.device("cpu"), (32, 32), lanes=lanes, assign=assign)
    counts = pipe.run(_batches(names, labels, 8, src))
    assert sum(counts) == ref
    assert sum(pipe.seen) == 30


def test_create_dataset_flow(tmp_path):
    from mpi_pytorch_amd.data.create_dataset import make_synthetic_metadata, build
    root = tmp_path / "train"
    make_synthetic_metadata(str(root), 20, num_classes=50)
    tr, te = build(str(root), "metadata.json", 15, str(tmp_path / "data"), copy=True)
    assert len(tr) == 12 and len(te) == 3
    import pandas as pd
    df = pd.read_csv(tmp_path / "data" / "train_sample.csv")
    assert {"file_name", "id", "category_id", "height", "width"} <= set(df.columns)
    assert os.path.exists(tmp_path / "data" / "img" / "train" / df.file_name[0])


def test_real_image_path_cpu(tmp_path):
    """FolderImages + per-image GPU/CPU preprocess on variable-size JPEGs."""
    from mpi_pytorch_amd.data.create_dataset import make_synthetic_metadata
    from mpi_pytorch_amd.data.manifest import FolderImages
    from mpi_pytorch_amd.engine.trainer import ManifestBatches
    make_synthetic_metadata(str(tmp_path), 6, write_images=True, size=(50, 37))
    names = ["images/{:03d}/{:02d}/{}.jpg".format(i % 300, i % 97, 100000 + i) for i in range(6)]
    mb = ManifestBatches(names, [1] * 6, 4, (32, 32), torch.device("cpu"),
                         FolderImages(str(tmp_path)), shuffle=False)
    xs = list(mb.epoch(0))
    assert xs[0][0].shape == (4, 32, 32, 8) and xs[1][0].shape == (2, 32, 32, 8)


def test_launcher_fail_fast(tmp_path):
    script = tmp_path / "s.py"
    script.write_text("import os, sys, time\n"
                      "r = int(os.environ['RANK'])\n"
                      "sys.exit(3) if r == 1 else time.sleep(60)\n")
    from mpi_pytorch_amd.launch import launch
    import time
    t = time.time()
    rc = launch(2, [sys.executable, str(script)])
    assert rc == 3 and time.time() - t < 30


def test_synthetic_images_device_gather_matches_host():
    """SyntheticImages.load_device (the training driver's GPU-side synthetic batches) gives
    bitwise the host load's images (checked on the CPU device here)."""
    from mpi_pytorch_amd.data.manifest import SyntheticImages
    src = SyntheticImages((37, 23), seed=3)
    names = ["img_%d.jpg" % i for i in range(11)]
    host = src.load(names)
    dev = src.load_device(names, "cpu")
    assert dev.dtype == torch.uint8 and tuple(dev.shape) == host.shape
    assert np.array_equal(dev.numpy(), host)


def test_step_timer_bookkeeping():
    """StepTimer phase accounting with stand-in events on a fake clock: per-phase means,
    'data' only between consecutive steps, lazy resolution past _MAX_PENDING steps, and
    reset (which also forgets the previous step's end)."""
    from mpi_pytorch_amd.engine.step import StepTimer
    clock = [0.0]

    class Ev:
        def record(self):
            self.t = clock[0]

        def synchronize(self):
            pass

        def elapsed_time(self, other):
            return other.t - self.t

    t = StepTimer(event_factory=Ev)
    durs = [1.0, 2.0, 3.0, 0.5, 0.25]  # gap before the step, forward, backward, comm, opt
    n = StepTimer._MAX_PENDING + 5
    for _ in range(n):
        clock[0] += durs[0]
        for i, d in enumerate(durs[1:]):
            t.mark(i)
            clock[0] += d
        t.mark(4)
    s = t.summary()
    assert s["steps"] == n
    assert s["forward"] == 2.0 and s["backward"] == 3.0
    assert s["comm_wait"] == 0.5 and s["optimizer"] == 0.25 and s["data"] == 1.0
    assert s["step"] == 6.75
    clock[0] += 100.0  # e.g. checkpoint + validation between epochs: not data time
    t.mark(0); t.mark(1); t.mark(2); t.mark(3); t.mark(4)
    s = t.summary()
    assert s["steps"] == 1 and s["data"] == 0.0
