"""Multi-process launch paths on the CPU (gloo): bench.py's own rank spawning, the
training driver at world size 2 (per-rank epoch lines in one log), and the watchdog's
device-completion beats.  Reference: ``mpiexec -n N python -m mpi4py main.py``
(``/root/reference/README.md:38``), per-rank epoch lines (``main.py:159-160``)."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env["MASTER_ADDR"] = "127.0.0.1"
    env["OMP_NUM_THREADS"] = "2"
    return env


def test_bench_spawns_ranks_itself(tmp_path):
    """``python bench.py --gpus 2`` with no launcher environment starts 2 ranks itself and
    rank 0 prints exactly one JSON line with n_gpus 2 and the per-bucket comm stats."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
           "--image-size", "32", "--batch", "2", "--classes", "10", "--steps", "2",
           "--warmup", "1"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=_env(), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip().startswith("{")]
    # the headline line as soon as it is measured, then the complete record with the extras
    assert len(lines) == 2, r.stdout
    head, rec = json.loads(lines[0]), json.loads(lines[1])
    assert "multi_gpu" not in head
    assert {k: v for k, v in rec.items() if k in head} == head
    assert rec["n_gpus"] == 2
    assert rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["global_batch"] == 4
    assert rec["steps"] == 2 and rec["warmup"] == 1
    comm = rec["comm"]
    assert comm["world"] == 2 and comm["timed"]
    assert len(comm["buckets"]) >= 2 and all(b["calls"] == 2 for b in comm["buckets"])
    assert rec["grad_allreduce_mb"] == pytest.approx(comm["mb_per_step"], rel=1e-3)
    assert "phases_ms" not in rec  # host runs have no HIP-event timers
    # multi-GPU decision data: the comm alternatives timed like the headline + a raw probe
    mg = rec["multi_gpu"]
    for k in ("comm_ctas8", "comm_bf16"):
        v = mg[k]
        assert v["img_per_s"] > 0 and v["ms_per_step"] > 0
        assert v["comm"]["world"] == 2 and v["comm"]["steps"] == 2
    assert mg["comm_ctas8"]["capped_communicator"] is False  # (gloo: no RCCL CTA cap)
    assert mg["comm_bf16"]["comm_dtype"] == "bf16"
    pr = mg["allreduce_probe"]["default"]
    assert pr["mb"] == pytest.approx(126.0) and pr["ms"] > 0 and pr["busbw_gbs"] > 0


def test_bench_rejects_rank_count_mismatch(tmp_path):
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
           "--image-size", "32", "--batch", "2", "--classes", "10", "--steps", "1",
           "--warmup", "0"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0 and "ranks" in (r.stderr + r.stdout)


def _bench_cpu(tmp_path, inject, extra=(), timeout=300):
    env = _env()
    env["MPA_BENCH_INJECT"] = inject
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
           "--image-size", "32", "--batch", "2", "--classes", "10", "--steps", "3",
           "--warmup", "1"] + list(extra)
    t0 = time.time()
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True,
                       timeout=timeout)
    lines = [l for l in r.stdout.splitlines() if l.strip().startswith("{")]
    return r, lines, time.time() - t0


def test_bench_keeps_headline_when_a_variant_throws(tmp_path):
    """Every multi-GPU decision variant raises: the headline line is printed, the final
    record carries each variant's error, and the job exits 0."""
    r, lines, _ = _bench_cpu(tmp_path, "variant_raise")
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 2, r.stdout
    rec = json.loads(lines[1])
    assert rec["value"] > 0 and rec["n_gpus"] == 2
    mg = rec["multi_gpu"]
    for k in ("comm_ctas8", "comm_bf16", "wgrad_stream_on"):
        assert "injected variant failure" in mg[k]["error"]
    assert mg["allreduce_probe"]["default"]["ms"] > 0


def test_bench_prints_headline_when_extras_hang(tmp_path):
    """The extras after the headline never finish: the headline line is already out, the
    extras budget ends every rank with 0 and no final record is printed."""
    r, lines, dt = _bench_cpu(tmp_path, "extras_hang", ["--extras-budget", "5"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["value"] > 0 and "multi_gpu" not in rec
    assert "timeout: extras exceeded" in r.stderr


def test_bench_backstop_ends_a_rank_stuck_holding_the_gil(tmp_path):
    """Both ranks block in a native call that holds the GIL inside the extras (libc sleep
    through ctypes.PyDLL - what a blocking HIP call without a GIL release does), so neither
    the budget timer thread nor the watchdog thread can run: the faulthandler backstop
    (budget + 30 s, no Python thread) dumps the stacks and ends the job non-zero, the
    headline line already on stdout (bench.py)."""
    r, lines, dt = _bench_cpu(tmp_path, "extras_gil_hang", ["--extras-budget", "2"],
                              timeout=300)
    assert r.returncode != 0, r.stderr[-3000:]
    assert len(lines) >= 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["value"] > 0 and "multi_gpu" not in rec
    assert "Timeout" in r.stderr and "launch: rank" in r.stderr
    assert dt < 200


def test_bench_keeps_headline_when_a_rank_aborts_in_extras(tmp_path):
    """Rank 1 dies inside the extras (os._exit(134), what a native abort or a GPU fault in
    a multi-GPU variant does): the headline line is on stdout, and the job exits non-zero
    with the launcher naming the rank."""
    r, lines, dt = _bench_cpu(tmp_path, "extras_abort=1", timeout=300)
    assert r.returncode == 134, (r.returncode, r.stderr[-3000:])
    assert len(lines) >= 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["value"] > 0 and rec["n_gpus"] == 2
    assert "launch: rank 1 exited with code 134" in r.stderr


def test_bench_hanging_rank_exits_rank_tagged_nonzero(tmp_path):
    """Rank 1 stops before its second timed step (its peer blocks in the all-reduce): the
    device-progress watchdog ends the job with exit 75 and a rank-tagged message well
    inside the driver's command limit, and no headline line is printed."""
    r, lines, dt = _bench_cpu(tmp_path, "hang_rank=1", ["--watchdog", "6"], timeout=200)
    assert r.returncode == 75, (r.returncode, r.stderr[-3000:])
    assert lines == []
    err = r.stderr
    assert "no bench progress" in err and ("rank 1:" in err or "rank 0:" in err)
    assert "launch: rank" in err
    assert dt < 150


def test_training_driver_two_ranks_logs_every_rank(tmp_path):
    """main.py under the launcher at world size 2: the shared training.log holds both
    ranks' epoch lines, each with its own rank tag, written whole by rank 0."""
    log = tmp_path / "training.log"
    cmd = [sys.executable, "-m", "mpi_pytorch_amd.launch", "-n", "2", "--timeout", "500",
           os.path.join(ROOT, "main.py"), "--device", "cpu", "--synthetic_images", "16",
           "--image_size", "32", "--NUM_EPOCHS", "2", "--BATCH_SIZE", "4",
           "--NUM_CLASSES", "10", "--VALIDATE", "false", "--log_file", str(log),
           "--CHECKPOINT_DIR", str(tmp_path) + "/ck/", "--step_timers", "true",
           "--metrics_jsonl", str(tmp_path / "m.jsonl")]
    env = _env()
    env["PYTHONPATH"] = ROOT
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    text = log.read_text()
    for e in (0, 1):
        for rk in (0, 1):
            assert "INFO:Herbarium_R{}:_Epoch: {} | Train Loss: ".format(rk, e) in text, text
    assert "_Files Received: 8" in text
    recs = [json.loads(l) for l in (tmp_path / "m.jsonl").read_text().splitlines()]
    assert {r_["rank"] for r_ in recs} == {0, 1}
    assert all(r_["comm"]["world"] == 2 for r_ in recs)


class _StalledEvent:
    """A device event that never completes (a GPU stuck in a collective)."""

    def query(self):
        return False


class _DoneEvent:
    def query(self):
        return True


def test_watchdog_fires_on_stalled_device_while_host_enqueues():
    from mpi_pytorch_amd.parallel.watchdog import Watchdog
    hits = []
    dog = Watchdog(0.3, rank=1, on_timeout=hits.append, poll_s=0.02).start()
    # the host keeps enqueuing steps (what an async GPU loop does) - none completes
    t0 = time.monotonic()
    step = 0
    while time.monotonic() - t0 < 1.0 and not hits:
        step += 1
        dog.beat_on(step, _StalledEvent())
        time.sleep(0.005)
    dog.stop()
    assert hits and "rank 1" in hits[0]
    assert dog.pending_events() <= Watchdog._MAX_EVENTS + 1


def test_watchdog_counts_completed_device_steps():
    from mpi_pytorch_amd.parallel.watchdog import Watchdog
    hits = []
    dog = Watchdog(0.3, rank=0, on_timeout=hits.append, poll_s=0.02).start()
    t0 = time.monotonic()
    step = 0
    while time.monotonic() - t0 < 0.8:
        step += 1
        dog.beat_on(step, _DoneEvent())
        time.sleep(0.01)
    time.sleep(0.05)
    assert not hits and dog._step == step
    # paused: no deadline during the epoch-end checkpoint / validation
    dog.pause()
    time.sleep(0.5)
    assert not hits
    dog.resume()
    time.sleep(0.1)
    assert not hits
    dog.stop()


def test_log_rank_lines_tags_each_rank(tmp_path):
    from mpi_pytorch_amd.utils.logging import init_logger, log_rank_lines
    path = tmp_path / "t.log"
    log = init_logger(0, str(path), stream=False)
    log_rank_lines(log, "_Epoch: 0 | Train Loss: 1.0 | Time: 2.0", 0, 3,
                   gather=lambda m: [m, m.replace("2.0", "5.0"), m.replace("2.0", "6.0")])
    log.info("after")
    lines = path.read_text().splitlines()
    assert lines == ["INFO:Herbarium_R0:_Epoch: 0 | Train Loss: 1.0 | Time: 2.0",
                     "INFO:Herbarium_R1:_Epoch: 0 | Train Loss: 1.0 | Time: 5.0",
                     "INFO:Herbarium_R2:_Epoch: 0 | Train Loss: 1.0 | Time: 6.0",
                     "INFO:Herbarium_R0:after"]
    for h in list(log.handlers):
        log.removeHandler(h)
        h.close()


def test_eval_pipeline_two_ranks_sum_reduces_accuracy(tmp_path):
    """evaluation_pipeline.py under the launcher at world size 2: each rank evaluates its
    ``array_split`` shard with two predictor lanes and rank 0 logs the SUM-reduced accuracy,
    which must equal one process's plain batched evaluation of the whole manifest with the
    same checkpoint (reference: ``/root/reference/evaluation_pipeline.py:190-199``)."""
    import re
    import torch
    from mpi_pytorch_amd.checkpoint import save_checkpoint
    from mpi_pytorch_amd.config import Config
    from mpi_pytorch_amd.data.manifest import SyntheticImages, synthetic_manifest
    from mpi_pytorch_amd.engine.eval_pipeline import load_predictor, plain_eval
    from mpi_pytorch_amd.models import initialize_model
    torch.manual_seed(3)
    model, _ = initialize_model("resnet18", 10, False, False)
    ckdir = str(tmp_path / "ck") + "/"
    ck = save_checkpoint({"epoch": 0, "state_dict": model.state_dict()}, 0, "resnet18", ckdir)
    log = tmp_path / "evaluation.log"
    cmd = [sys.executable, "-m", "mpi_pytorch_amd.launch", "-n", "2", "--timeout", "500",
           os.path.join(ROOT, "evaluation_pipeline.py"), "--device", "cpu",
           "--synthetic_images", "44", "--image_size", "32", "--NUM_CLASSES", "10",
           "--MODEL_NAME", "resnet18", "--eval_batch", "8", "--eval_lanes", "2",
           "--CHECKPOINT_DIR", ckdir, "--log_file", str(log)]
    env = _env()
    env["PYTHONPATH"] = ROOT
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    text = log.read_text()
    acc = float(re.search(r"Accuracy is ([-+0-9.eE]+)", text).group(1))
    assert "Finished node 3, acc" in text and "Finished node 4, acc" in text
    assert "2 lanes x 2 ranks" in text
    cfg = Config(device="cpu", synthetic_images=44, image_size=32, NUM_CLASSES=10,
                 MODEL_NAME="resnet18", CHECKPOINT_DIR=ckdir)
    df = synthetic_manifest(44, 10, cfg.seed)
    oracle = load_predictor(cfg, torch.device("cpu"), ck)
    correct = plain_eval(oracle, list(df["file_name"].values), list(df["category_id"].values), 8,
                         SyntheticImages((64, 64)), torch.device("cpu"), (32, 32))
    assert acc == pytest.approx(correct / 44, abs=1e-9)
