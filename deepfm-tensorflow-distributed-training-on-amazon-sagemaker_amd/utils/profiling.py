"""Tracing / profiling hooks.

The reference has none in-script (profiler explicitly disabled, NB-PS:117-118); rocfm provides:

* ``trace_range(name)`` — a roctx range (``torch.cuda.nvtx`` is roctx on ROCm builds) around
  loader / step / eval / checkpoint phases, visible in ``rocprofv3 --marker-trace`` timelines;
  a no-op on CPU.
* ``StepProfiler("a:b", out_dir)`` — the ``--profile_steps a:b`` flag: wraps global steps [a, b)
  with ``torch.profiler`` (CPU + HIP activities) and writes a Chrome trace plus a per-kernel table
  (``kernel_table.txt``) under ``out_dir``.
* ``StepTimer`` — host wall time per logged interval and the fraction of it the training loop
  spent waiting for the input pipeline (the "loader stall %" of §5.5).
"""
from __future__ import annotations

import contextlib
import os
import time
from typing import Optional, Tuple

import torch


@contextlib.contextmanager
def trace_range(name: str):
    on = torch.cuda.is_available()
    if on:
        try:
            torch.cuda.nvtx.range_push(name)
        except Exception:  # roctx unavailable in this build
            on = False
    try:
        yield
    finally:
        if on:
            torch.cuda.nvtx.range_pop()


def parse_steps(spec: str) -> Optional[Tuple[int, int]]:
    if not spec:
        return None
    a, _, b = str(spec).partition(":")
    a, b = int(a), int(b or int(a) + 1)
    if b <= a:
        raise ValueError(f"profile_steps must be a:b with b > a, got {spec!r}")
    return a, b


class StepProfiler:
    """torch.profiler over global steps [a, b); call ``step(global_step)`` after every step."""

    def __init__(self, spec: str, out_dir: str):
        self.window = parse_steps(spec)
        self.out_dir = out_dir
        self.prof = None
        self.done = False

    def step(self, global_step: int) -> None:
        if self.window is None or self.done:
            return
        a, b = self.window
        if self.prof is None and a <= global_step < b:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self.prof = torch.profiler.profile(activities=acts, record_shapes=False)
            self.prof.__enter__()
        elif self.prof is not None and global_step >= b:
            self.close()

    def close(self) -> None:
        if self.prof is None:
            return
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self.prof.__exit__(None, None, None)
        os.makedirs(self.out_dir, exist_ok=True)
        self.prof.export_chrome_trace(os.path.join(self.out_dir, "trace.json"))
        with open(os.path.join(self.out_dir, "kernel_table.txt"), "w") as f:
            sort = "self_cuda_time_total" if torch.cuda.is_available() else "self_cpu_time_total"
            f.write(self.prof.key_averages().table(sort_by=sort, row_limit=40))
        self.prof = None
        self.done = True


class StepTimer:
    """Wall time and input-wait time between log points."""

    def __init__(self):
        self.t0 = time.perf_counter()
        self.wait = 0.0

    @contextlib.contextmanager
    def waiting(self):
        t = time.perf_counter()
        try:
            yield
        finally:
            self.wait += time.perf_counter() - t

    def lap(self) -> Tuple[float, float]:
        """(seconds since the last lap, fraction of them spent waiting for input)."""
        now = time.perf_counter()
        dt = now - self.t0
        frac = self.wait / dt if dt > 0 else 0.0
        self.t0, self.wait = now, 0.0
        return dt, frac
