"""Checkpoint I/O with the reference's exact format.

Reference: ``helpers.save_checkpoint`` / ``helpers.load_checkpoint``
(``/root/reference/helpers.py:4-15``) and the payload built at ``main.py:163-168``::

    {'epoch': int, 'state_dict': model.state_dict(), 'optimizer': optimizer.state_dict(),
     'loss': float}

written to ``CHECKPOINT_DIR + 'checkpoint_{MODEL_NAME}.pt'`` (overwritten every epoch).

Here ``state_dict`` carries torchvision key names with OIHW fp32 conv weights (our
internal KRSC/bf16 layouts are converted by the layer modules), and ``optimizer`` is in
``torch.optim.Adam`` / ``torch.optim.SGD`` format, so a file written here loads into a
torchvision model + ``torch.optim.Adam`` and vice versa.

Robustness additions: the write is atomic (temp file + ``os.replace``), so a crash during
the write never leaves a truncated checkpoint behind; loads use ``weights_only=True``
(nothing in the file is executed).
"""
from __future__ import annotations

import os
import tempfile
from typing import Any, Dict, Optional, Tuple

import torch


def checkpoint_path(checkpoint_dir: str, model_name: str) -> str:
    return os.path.join(checkpoint_dir, "checkpoint_{}.pt".format(model_name))


def _to_cpu(obj: Any) -> Any:
    if torch.is_tensor(obj):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return type(obj)((k, _to_cpu(v)) for k, v in obj.items())
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


def save_checkpoint(state: Dict[str, Any], epoch: int, model_name: str, checkpoint_dir: str,
                    best_model_dir: Optional[str] = None, is_best: bool = True) -> str:
    """Same signature as ``helpers.save_checkpoint`` (``is_best``/``best_model_dir`` are
    accepted and, as in the reference, unused)."""
    os.makedirs(checkpoint_dir or ".", exist_ok=True)
    path = checkpoint_path(checkpoint_dir, model_name)
    fd, tmp = tempfile.mkstemp(prefix="tmp_ckpt_", suffix=".pt", dir=checkpoint_dir or ".")
    os.close(fd)
    try:
        torch.save(_to_cpu(state), tmp)
        os.replace(tmp, path)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)
    return path


def load_checkpoint(checkpoint_fpath: str, model, optimizer=None,
                    map_location="cpu") -> Tuple[Any, Any, int]:
    """Restore model (+ optimizer) and return ``(model, optimizer, epoch)`` like
    ``helpers.load_checkpoint``.  The flat-arena bf16 weight shadow is refreshed."""
    ck = torch.load(checkpoint_fpath, map_location=map_location, weights_only=True)
    model.load_state_dict(ck["state_dict"])
    arena = getattr(model, "_mpa_arena", None)
    if arena is not None:
        arena.sync_shadow()
    if optimizer is not None and "optimizer" in ck:
        optimizer.load_state_dict(ck["optimizer"])
    return model, optimizer, int(ck.get("epoch", 0))


def read_checkpoint(path: str) -> Dict[str, Any]:
    return torch.load(path, map_location="cpu", weights_only=True)


def build_state(epoch: int, model, optimizer, loss: float) -> Dict[str, Any]:
    """The payload of ``main.py:163-168``."""
    return {"epoch": epoch, "state_dict": model.state_dict(),
            "optimizer": optimizer.state_dict(), "loss": loss}
