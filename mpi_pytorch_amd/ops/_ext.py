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
_synced = None

# Serialized-kernel debug mode: MPA_DEBUG_SYNC=1 makes every native op
# synchronize the device when it returns, so an asynchronous HIP fault is raised at the op
# that launched it, with its name.  For kernel-level serialization export
# AMD_SERIALIZE_KERNEL=3 and HIP_LAUNCH_BLOCKING=1 as well (read at HIP init; the launcher
# does it for every rank when MPA_DEBUG_SYNC=1 is set).
_DEBUG_SYNC = os.environ.get("MPA_DEBUG_SYNC", "0") == "1"


class SyncedExt:
    """The native module with a device sync + error attribution after every op call."""

    def __init__(self, mod, sync=None):
        self._mod = mod
        self._sync = sync

    def __getattr__(self, name):
        f = getattr(self._mod, name)
        if not callable(f) or isinstance(f, type):
            return f  # (classes such as BatchRing pass through)

        def call(*args, **kwargs):
            out = f(*args, **kwargs)
            try:
                if self._sync is not None:
                    self._sync()
                else:
                    import torch
                    torch.cuda.synchronize()
            except RuntimeError as e:
                raise RuntimeError("native op '%s' failed on the device: %s" % (name, e)) from e
            return out

        call.__name__ = name
        return call


_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def source_hash(root: str = _ROOT):
    """setup.py's hash of the csrc/ tree next to this package (None without one)."""
    if not os.path.isdir(os.path.join(root, "csrc")) or \
            not os.path.exists(os.path.join(root, "setup.py")):
        return None
    import importlib.util
    spec = importlib.util.spec_from_file_location("_mpa_setup_hash", os.path.join(root, "setup.py"))
    src = open(os.path.join(root, "setup.py")).read()
    # only the hashing function: executing setup.py would run setup()
    start = src.index("def source_hash(")
    end = src.index("\n\n\n", start)
    ns = {"os": os, "ROOT": root}
    exec(compile(src[start:end], spec.origin, "exec"), ns)
    return ns["source_hash"](root)


def check_fresh(mod, root: str = _ROOT) -> None:
    """Refuse a native binary built from other sources than the csrc/ tree beside it
    (MPA_ALLOW_STALE=1 to override, e.g. while bisecting)."""
    if os.environ.get("MPA_ALLOW_STALE", "0") == "1":
        return
    want = source_hash(root)
    if want is None:
        return
    have = mod.src_hash() if hasattr(mod, "src_hash") else "<none>"
    if have != want:
        raise RuntimeError(
            "mpi_pytorch_amd native extension {} was built from other sources (hash {}) than "
            "{}/csrc (hash {}): rebuild with `python setup.py build_ext --inplace`".format(
                getattr(mod, "__file__", "_C"), have, root, want))


def load():
    global _ext, _err
    if _ext is not None:
        return _ext
    if _err is not None:
        raise _err
    try:
        mod = importlib.import_module("mpi_pytorch_amd._C")
    except Exception as e:  # pragma: no cover - depends on build state
        _err = RuntimeError(
            "mpi_pytorch_amd native extension (_C) is not importable: {}. Build it with "
            "`python setup.py build_ext --inplace` (PYTORCH_ROCM_ARCH=gfx950).".format(e))
        raise _err
    try:
        check_fresh(mod)
    except RuntimeError as e:
        _err = e
        raise
    _ext = mod
    return _ext


def available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False


def ext():
    """Return the native module; raises loudly when it is missing.  Under MPA_DEBUG_SYNC=1
    the module is wrapped so every op synchronizes and names itself on a device error."""
    global _synced
    m = load()
    if not _DEBUG_SYNC:
        return m
    if _synced is None:
        _synced = SyncedExt(m)
    return _synced


def so_path() -> str:
    m = load()
    return os.path.abspath(m.__file__)
