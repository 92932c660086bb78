"""Per-rank progress watchdog: fail fast instead of hanging.

The reference's only failure handling is ``python -m mpi4py`` turning an uncaught exception
into an MPI abort (``/root/reference/README.md:38``).  That cannot catch
the failure mode that matters on a GPU node - a rank stuck forever inside a collective
because a peer died or diverged (different bucket order, a skipped step).  Here:

* ``Watchdog(timeout_s)`` runs a daemon thread; the GPU training loop calls
  ``beat_on(step, event)`` after every step with a HIP event recorded behind the step's
  last kernel, and the thread counts the step only when that event has completed on the
  device (``beat(step)`` is the host-only form).  ``pause()`` / ``resume()`` bracket the
  epoch-end checkpoint and rank-0 validation.  If no beat arrives for ``timeout_s`` the watchdog logs a rank-tagged
  message with the last step, dumps every thread's Python stack (``faulthandler``) and
  terminates the process with exit code 75, so the launcher (``launch.py``, torchrun)
  tears the job down - the analogue of MPI_Abort.
* RCCL's own error propagation is switched on (``TORCH_NCCL_ASYNC_ERROR_HANDLING``) by
  :func:`parallel.dist.init_world`, so a communicator error surfaces as an exception in the
  rank that sees it, not a hang.
* ``on_timeout`` replaces the exit for tests.
"""
from __future__ import annotations

import faulthandler
import logging
import os
import sys
import threading
import time
from typing import Callable, Optional

EXIT_STALLED = 75


class Watchdog:
    def __init__(self, timeout_s: float, rank: int = 0, name: str = "train",
                 on_timeout: Optional[Callable[[str], None]] = None, poll_s: float = 0.0):
        self.timeout_s = float(timeout_s)
        self.rank = rank
        self.name = name
        self.on_timeout = on_timeout
        self.poll_s = poll_s if poll_s > 0 else max(min(self.timeout_s / 10.0, 5.0), 0.01)
        self._last = time.monotonic()
        self._step = -1
        self._stop = threading.Event()
        self.fired = False
        self._paused = False
        self._lock = threading.Lock()
        self._events: list = []  # (step, device event) not yet seen complete
        self._thread: Optional[threading.Thread] = None

    _MAX_EVENTS = 64

    def start(self) -> "Watchdog":
        if self.timeout_s <= 0 or self._thread is not None:
            return self
        self._last = time.monotonic()
        self._thread = threading.Thread(target=self._run, name="mpa-watchdog", daemon=True)
        self._thread.start()
        return self

    def beat(self, step: int = -1) -> None:
        self._last = time.monotonic()
        if step >= 0:
            self._step = step

    def beat_on(self, step: int, event) -> None:
        """Count ``step`` as progress only once ``event`` (recorded on the device stream
        after the step's last kernel) has COMPLETED.  The host enqueues steps far ahead of
        the GPU; a rank stuck inside an RCCL collective keeps enqueuing until the launch
        queue or the allocator backs up, so enqueue-time beats would keep a hung job
        alive.  The watchdog thread polls ``event.query()`` (never blocks)."""
        with self._lock:
            self._events.append((step, event))
            if len(self._events) > self._MAX_EVENTS:
                # the device completes in order: thinning the middle of the queue only
                # coarsens the step numbers reported, never hides a stall
                keep = self._events[:1] + self._events[2::2]
                self._events = keep

    def _poll_events(self) -> None:
        with self._lock:
            evs = self._events
            if not evs:
                return
            done = -1
            if evs[-1][1].query():
                done = len(evs) - 1
            else:
                for i, (_s, ev) in enumerate(evs):
                    if not ev.query():
                        break
                    done = i
            if done >= 0:
                self._step = evs[done][0]
                self._last = time.monotonic()
                del evs[:done + 1]

    def pending_events(self) -> int:
        return len(self._events)

    def pause(self) -> None:
        """Suspend the deadline (e.g. around checkpoint writes or evaluation on rank 0)."""
        self._paused = True

    def resume(self) -> None:
        self._paused = False
        self._last = time.monotonic()

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=1.0)
            self._thread = None

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            self._poll_events()
            if self._paused:
                continue
            idle = time.monotonic() - self._last
            if idle > self.timeout_s:
                self._fire(idle)
                return

    def _fire(self, idle: float) -> None:
        self.fired = True
        msg = ("rank %d: no %s progress for %.1f s (last completed step %d) - aborting job"
               % (self.rank, self.name, idle, self._step))
        logging.getLogger("Herbarium").error(msg)
        if self.on_timeout is not None:
            self.on_timeout(msg)
            return
        sys.stderr.write(msg + "\n")
        faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        sys.stderr.flush()
        os._exit(EXIT_STALLED)

    def __enter__(self) -> "Watchdog":
        return self.start()

    def __exit__(self, *exc) -> None:
        self.stop()
