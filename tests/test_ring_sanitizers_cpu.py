"""Race detection for the native runtime's threaded code: the batch
ring's scheduling core (``csrc/runtime/ring_core.h``, the part of ``BatchRing`` that
producer threads, Python decode threads and the consumer share) is built on the host with
ThreadSanitizer and with AddressSanitizer + UndefinedBehaviorSanitizer and stress-tested by
``csrc/runtime/ring_stress.cpp`` (native and external producers, in-order hand-off,
payload integrity, stop() waking blocked threads).  GPU sanitizers are not available on
this pool; the kernels are covered by the bitwise engine / determinism tests instead.

Reference: the reference's own concurrency hazards (shared ``training.log``, collective
count mismatch, MPI sentinel ordering) have no checker at all."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "csrc", "runtime", "ring_stress.cpp")


@pytest.mark.parametrize("sanitizer", ["thread", "address,undefined"])
def test_ring_core_under_host_sanitizers(tmp_path, sanitizer):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "ring_stress")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=" + sanitizer, "-I", os.path.join(ROOT, "csrc", "runtime"), SRC,
           "-o", exe, "-pthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="halt_on_error=1 detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1")
    r = subprocess.run([exe, "1500"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "ring_stress ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "runtime error" not in r.stderr
