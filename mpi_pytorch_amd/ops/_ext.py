"""Loader for the in-tree native extension ``mpi_pytorch_amd._C``.

The extension holds every hand-written gfx950 HIP kernel (``csrc/kernels/*.hip``) and
the C++ runtime pieces (``csrc/runtime``).  It is built in-tree by ``setup.py
build_ext --inplace`` (see ``__graft_entry__.build``).

Policy: GPU tensors ALWAYS go through the native kernels.  If the extension is missing
or fails to import and a CUDA/HIP tensor reaches an op, we raise - there is no silent
fallback to PyTorch/MIOpen kernels.  CPU tensors use the reference implementations in
``cpu_ref.py`` (the reference framework itself is CPU-only).
"""
from __future__ import annotations

import importlib
import os

_ext = None
_err = None


def load():
    global _ext, _err
    if _ext is not None:
        return _ext
    if _err is not None:
        raise _err
    try:
        _ext = importlib.import_module("mpi_pytorch_amd._C")
    except Exception as e:  # pragma: no cover - depends on build state
        _err = RuntimeError(
            "mpi_pytorch_amd native extension (_C) is not importable: {}. Build it with "
            "`python setup.py build_ext --inplace` (PYTORCH_ROCM_ARCH=gfx950).".format(e))
        raise _err
    return _ext


def available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False


def ext():
    """Return the native module; raises loudly when it is missing."""
    return load()


def so_path() -> str:
    m = load()
    return os.path.abspath(m.__file__)
