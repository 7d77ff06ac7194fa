"""Failure detection: fail fast instead of hanging.

``Watchdog(timeout_s)`` runs a daemon thread; the training loop calls ``beat()`` every step.  If
no heartbeat arrives for ``timeout_s`` (a hung collective, a dead peer, a stuck loader), it dumps
every thread's Python stack to stderr and terminates the process with exit code 3 so the launcher
(``rocfm.launch``, or torchrun's ``--max-restarts``) restarts the job, which resumes from the
latest complete checkpoint (the ``checkpoint`` index is replaced atomically).  torch.distributed's
own timeout (``dist_timeout_s``) bounds every collective as a second line of defence.
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time


class Watchdog:
    def __init__(self, timeout_s: float, name: str = "rocfm", exit_code: int = 3):
        self.timeout = float(timeout_s)
        self.name = name
        self.exit_code = exit_code
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._thread = None
        self.fired = False

    def start(self) -> "Watchdog":
        if self.timeout > 0 and self._thread is None:
            self._thread = threading.Thread(target=self._run, name=f"{self.name}-watchdog", daemon=True)
            self._thread.start()
        return self

    def beat(self) -> None:
        self._last = time.monotonic()

    def stop(self) -> None:
        self._stop.set()

    def _run(self) -> None:
        while not self._stop.wait(min(1.0, self.timeout / 4)):
            idle = time.monotonic() - self._last
            if idle > self.timeout:
                self.fired = True
                sys.stderr.write(f"[{self.name}] watchdog: no progress for {idle:.0f}s (> {self.timeout:.0f}s); "
                                 f"dumping stacks and exiting with {self.exit_code}\n")
                sys.stderr.flush()
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                sys.stderr.flush()
                os._exit(self.exit_code)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
        return False
