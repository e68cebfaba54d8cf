"""Tracing / profiling hooks: roctx ranges (visible in rocprofv3 --marker-trace and
torch.profiler), HIP-event step timers on the compute stream, and a torch.profiler context factory.
The reference has none (grep profil|trace|nvtx is empty)."""
from __future__ import annotations

import contextlib
import ctypes
import os
import time

import torch

_roctx = None


def _lib():
    global _roctx
    if _roctx is None:
        cands = [os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so"), "/opt/rocm/lib/libroctx64.so"]
        for c in cands:
            if os.path.exists(c):
                try:
                    _roctx = ctypes.CDLL(c)
                    _roctx.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    break
                except OSError:
                    continue
        if _roctx is None:
            _roctx = False
    return _roctx


@contextlib.contextmanager
def range(name: str):
    """roctx range (no-op when roctx is unavailable or PDT_ROCTX=0)."""
    lib = _lib() if os.environ.get("PDT_ROCTX", "1") == "1" else False
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


class StepTimer:
    """Per-phase GPU time via HIP events; read with ``summary()`` (one sync at read time only)."""

    def __init__(self, enabled=True):
        self.enabled = enabled and torch.cuda.is_available()
        self.events = {}
        self.cpu = {}

    @contextlib.contextmanager
    def phase(self, name):
        if not self.enabled:
            t = time.perf_counter()
            yield
            self.cpu.setdefault(name, []).append(time.perf_counter() - t)
            return
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        with range(name):
            yield
        e.record()
        self.events.setdefault(name, []).append((s, e))

    def summary(self):
        out = {}
        if self.enabled:
            torch.cuda.synchronize()
            for k, v in self.events.items():
                ms = [s.elapsed_time(e) for s, e in v]
                out[k] = {"mean_ms": sum(ms) / len(ms), "n": len(ms)}
        for k, v in self.cpu.items():
            out[k] = {"mean_ms": 1000 * sum(v) / len(v), "n": len(v)}
        return out


def torch_profiler(out_dir: str, wait=1, warmup=1, active=3):
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    return torch.profiler.profile(activities=acts,
                                  schedule=torch.profiler.schedule(wait=wait, warmup=warmup, active=active),
                                  on_trace_ready=torch.profiler.tensorboard_trace_handler(out_dir))
