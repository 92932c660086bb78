"""Training-curve record: run the training driver (``main.py``'s ``run_training``) on
synthetic images and print one JSON line per epoch (train loss, rank-0 eval-mode accuracy
on the training sample, img/s) - the reference's own correctness oracle, training-set
accuracy rising over epochs (``/root/reference/training.log:1040-1112``, ``main.py:173-185``).

    python tools/learn_curve.py --synthetic_images 800 --image_size 224 --BATCH_SIZE 128 \\
        --NUM_CLASSES 64500 --NUM_EPOCHS 15 [--device cpu] [--resume_epochs 3]

``--resume_epochs k`` then resumes from the written checkpoint for k more epochs
(``FROM_CHECKPOINT``), printing those epochs too.
"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    import argparse
    from mpi_pytorch_amd.config import Config
    from mpi_pytorch_amd.engine.trainer import run_training
    import mpi_pytorch_amd.parallel.dist as D
    p = argparse.ArgumentParser()
    p.add_argument("--resume_epochs", type=int, default=0)
    ns, rest = p.parse_known_args(argv)
    tmp = tempfile.mkdtemp(prefix="mpa_curve_")
    defaults = dict(CHECKPOINT_DIR=tmp + "/ck/", log_file=os.path.join(tmp, "training.log"),
                    synthetic_images=256, image_size=64, NUM_CLASSES=1000, BATCH_SIZE=64,
                    NUM_EPOCHS=20)
    cfg = Config.from_args(rest, **defaults)
    t0 = time.time()
    out = run_training(cfg)
    for h in out["history"]:
        print(json.dumps({k: (round(v, 5) if isinstance(v, float) else v)
                          for k, v in h.items() if k in ("epoch", "train_loss", "acc",
                                                        "img_per_s_global", "time_s")}),
              flush=True)
    if ns.resume_epochs:
        D._WORLD = None
        cfg2 = Config.from_args(rest, **defaults)
        cfg2.FROM_CHECKPOINT = True
        cfg2.NUM_EPOCHS = cfg.NUM_EPOCHS + ns.resume_epochs
        out2 = run_training(cfg2)
        for h in out2["history"]:
            print(json.dumps({"resumed": True, **{k: (round(v, 5) if isinstance(v, float) else v)
                                                  for k, v in h.items()
                                                  if k in ("epoch", "train_loss", "acc")}}),
                  flush=True)
    print("total_s %.1f" % (time.time() - t0), flush=True)


if __name__ == "__main__":
    main()
