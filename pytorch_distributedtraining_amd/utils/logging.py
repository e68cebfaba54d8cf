"""Rank-aware logging, EMA loss meter, throughput meter and metric sinks.

* ``RankLogger.print(msg, ranks=None)``   -- Stoke's print_on_devices (default: info rank only).
* ``EMAMeter``                             -- ema = w*new + (1-w)*ema, w = 0.1 (Stoke default).
* ``MetricsSink``                          -- rank-0 JSONL always, optional Weights & Biases (imported
                                              lazily, NEVER a retry-forever init loop like the reference's
                                              Stoke-DDP.py:316-322; W&B failures are logged and ignored).
* ``ThroughputMeter``                      -- samples/s, tokens/s (whole job), MFU estimate.
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch.distributed as dist


def _rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


class RankLogger:
    def __init__(self, info_rank=0, verbose=True, stream=None):
        self.info_rank = info_rank
        self.verbose = verbose
        self.stream = stream or sys.stdout

    def print(self, msg, ranks=None):
        r = _rank()
        if ranks is None:
            ranks = [self.info_rank] if not isinstance(self.info_rank, (list, tuple)) else self.info_rank
        if ranks == "all" or r in ranks:
            print(f"[rank {r}] {msg}" if ranks == "all" or len(ranks) > 1 else msg, file=self.stream, flush=True)

    def will_print(self, ranks=None) -> bool:
        """Whether ``print(msg, ranks)`` on this rank would print (callers skip building the message -- and
        any host read it needs -- otherwise)."""
        r = _rank()
        if ranks is None:
            ranks = [self.info_rank] if not isinstance(self.info_rank, (list, tuple)) else self.info_rank
        return ranks == "all" or r in ranks

    def info(self, msg):
        if self.verbose:
            self.print(msg)


class EMAMeter:
    def __init__(self, weight=0.1):
        self.weight = weight
        self.value = None

    def update(self, x: float) -> float:
        self.value = x if self.value is None else self.weight * x + (1 - self.weight) * self.value
        return self.value

    def reset(self):
        self.value = None


class MetricsSink:
    def __init__(self, path=None, wandb_project=None, config=None):
        self.rank0 = _rank() == 0
        self.f = None
        if self.rank0 and path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            self.f = open(path, "a")
        self.wandb = None
        if self.rank0 and wandb_project:
            try:
                import wandb  # noqa: F401

                self.wandb = wandb.init(project=wandb_project, config=config or {}, reinit=True)
            except Exception as e:  # no network / not installed: keep training
                print(f"[metrics] W&B disabled: {e!r}", file=sys.stderr)

    def log(self, data: dict, step=None):
        if not self.rank0:
            return
        rec = dict(data)
        rec["time"] = time.time()
        if step is not None:
            rec["step"] = step
        if self.f:
            self.f.write(json.dumps(rec, default=float) + "\n")
            self.f.flush()
        if self.wandb is not None:
            try:
                self.wandb.log(data, step=step)
            except Exception:
                pass

    def close(self):
        if self.f:
            self.f.close()
        if self.wandb is not None:
            try:
                self.wandb.finish()
            except Exception:
                pass


class ThroughputMeter:
    def __init__(self, world_size=1, flops_per_sample=None):
        self.world = world_size
        self.flops = flops_per_sample
        self.t0 = None
        self.n = 0

    def start(self):
        self.t0 = time.perf_counter()
        self.n = 0

    def add(self, samples_per_rank: int):
        self.n += samples_per_rank

    def rate(self) -> dict:
        dt = max(time.perf_counter() - (self.t0 or time.perf_counter()), 1e-9)
        sps = self.n * self.world / dt
        out = {"samples_per_s": sps, "elapsed_s": dt}
        if self.flops:
            out["tflops_per_s"] = sps * self.flops / 1e12
        return out
