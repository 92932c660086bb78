"""Single-node launcher: ``python -m mpi_pytorch_amd.launch -n N script.py [args...]``.

The reference launches with ``mpiexec -n N python -m mpi4py main.py`` (README.md:38); MPI
is not available on the MI355X image, so this spawns N ranks itself (one per GPU), with
RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, and mirrors
``python -m mpi4py``'s failure semantics: if any rank exits non-zero the others are
terminated and the launcher exits with that code (fail fast instead of hanging in a
collective).  ``torchrun`` and MPI launchers work too (see parallel/dist.py).
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(nprocs: int, cmd, env_extra=None, timeout: float = 0.0) -> int:
    port = free_port()
    procs = []
    for r in range(nprocs):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": str(nprocs), "LOCAL_RANK": str(r),
                    "LOCAL_WORLD_SIZE": str(nprocs), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port)})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if env.get("MPA_DEBUG_SYNC") == "1":  # serialized-kernel debug mode (ops/_ext.py)
            env.setdefault("AMD_SERIALIZE_KERNEL", "3")
            env.setdefault("HIP_LAUNCH_BLOCKING", "1")
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        if env_extra:
            env.update(env_extra)
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
    t0 = time.time()
    rc = 0
    try:
        while True:
            alive = False
            for r, p in enumerate(procs):
                code = p.poll()
                if code is None:
                    alive = True
                elif code != 0 and rc == 0:
                    rc = code
                    sys.stderr.write("launch: rank %d exited with code %d; stopping the job\n"
                                     % (r, code))
            if rc != 0 or not alive:
                break
            if timeout and time.time() - t0 > timeout:
                rc = 124
                sys.stderr.write("launch: job exceeded its %.0f s limit; stopping ranks %s\n"
                                 % (timeout, [r for r, p in enumerate(procs) if p.poll() is None]))
                break
            time.sleep(0.1)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
    return rc


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("-n", "--nprocs", type=int, default=1)
    ap.add_argument("--timeout", type=float, default=0.0)
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = [sys.executable, a.script] + list(a.args)
    if a.script.startswith("-m"):
        cmd = [sys.executable] + a.script.split(None, 1) + list(a.args)
    return launch(a.nprocs, cmd, timeout=a.timeout)


if __name__ == "__main__":
    sys.exit(main())
