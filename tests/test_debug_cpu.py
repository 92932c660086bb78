"""Serialized-kernel debug mode (``MPA_DEBUG_SYNC=1``): every native op is
followed by a device sync, and an asynchronous device error is re-raised naming the op
that launched it; the launcher adds AMD_SERIALIZE_KERNEL / HIP_LAUNCH_BLOCKING for every
rank.  Checked here with a stand-in module and sync (no GPU on the CPU box)."""
import os
import subprocess
import sys

import pytest

from mpi_pytorch_amd.ops._ext import SyncedExt


class _FakeMod:
    class BatchRing:  # classes pass through unwrapped
        pass

    version = 3

    @staticmethod
    def conv_fwd(x):
        return x + 1

    @staticmethod
    def bad_kernel(x):
        return x


def test_synced_ext_syncs_after_every_op_and_names_failures():
    calls = []
    state = {"fail": False}

    def sync():
        calls.append(1)
        if state["fail"]:
            raise RuntimeError("hipErrorIllegalAddress")

    m = SyncedExt(_FakeMod, sync)
    assert m.conv_fwd(1) == 2 and len(calls) == 1
    assert m.BatchRing is _FakeMod.BatchRing and m.version == 3 and len(calls) == 1
    state["fail"] = True
    with pytest.raises(RuntimeError, match="native op 'bad_kernel' failed on the device"):
        m.bad_kernel(0)


def test_launcher_exports_serialization_env(tmp_path):
    script = tmp_path / "s.py"
    out = tmp_path / "env.txt"
    script.write_text("import os\nopen(os.environ['OUT'] + os.environ['RANK'], 'w').write("
                      "os.environ.get('AMD_SERIALIZE_KERNEL', '') + ' ' + "
                      "os.environ.get('HIP_LAUNCH_BLOCKING', ''))\n")
    env = dict(os.environ, MPA_DEBUG_SYNC="1", OUT=str(out))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "mpi_pytorch_amd.launch", "-n", "2", str(script)],
                       env=dict(env, PYTHONPATH=root), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    for rank in (0, 1):
        assert (tmp_path / ("env.txt%d" % rank)).read_text() == "3 1"


def test_stale_binary_guard(tmp_path):
    """_ext.check_fresh compares the hash compiled into _C with setup.py's hash of the
    csrc/ tree beside it: any source edit makes the old binary refuse to load."""
    import shutil
    import types
    from mpi_pytorch_amd.ops import _ext as E
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    shutil.copytree(os.path.join(root, "csrc"), tmp_path / "csrc")
    shutil.copy(os.path.join(root, "setup.py"), tmp_path / "setup.py")
    h = E.source_hash(str(tmp_path))
    assert h == E.source_hash(root) and len(h) == 32
    mod = types.SimpleNamespace(src_hash=lambda: h, __file__="_C.so")
    E.check_fresh(mod, str(tmp_path))  # matching: loads
    with open(tmp_path / "csrc" / "kernels" / "common.h", "a") as f:
        f.write("\n// edited\n")
    with pytest.raises(RuntimeError, match="other sources"):
        E.check_fresh(mod, str(tmp_path))
    old = os.environ.get("MPA_ALLOW_STALE")
    os.environ["MPA_ALLOW_STALE"] = "1"
    try:
        E.check_fresh(mod, str(tmp_path))
    finally:
        if old is None:
            del os.environ["MPA_ALLOW_STALE"]
        else:
            os.environ["MPA_ALLOW_STALE"] = old
