"""Failure detection and fault injection.

* ``configure_watchdog()`` -- RCCL async error handling + a bounded collective timeout, so a dead rank
  makes the survivors exit with an error instead of hanging (TORCH_NCCL_ASYNC_ERROR_HANDLING etc.).
* ``maybe_inject_fault(step)`` -- env-triggered faults for tests: PDT_FAULT_RANK=<r>,
  PDT_FAULT_STEP=<s>, PDT_FAULT_MODE=exit|raise|hang|delay (delay seconds via PDT_FAULT_DELAY).
"""
from __future__ import annotations

import os
import sys
import time

import torch.distributed as dist


def configure_watchdog(timeout_s: float = 600.0):
    """Called by ``init_distributed`` before the process group exists (the NCCL/RCCL env is read then)."""
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    os.environ.setdefault("TORCH_NCCL_ENABLE_MONITORING", "1")
    os.environ.setdefault("TORCH_NCCL_HEARTBEAT_TIMEOUT_SEC", str(int(timeout_s)))
    os.environ.setdefault("TORCH_NCCL_DUMP_ON_TIMEOUT", "0")


class InjectedFault(RuntimeError):
    pass


def maybe_inject_fault(step: int):
    """Called by ``Trainer.step`` before optimizer step ``step`` (0-based).  Fires only in the launch attempt
    ``PDT_FAULT_RESTART`` (default 0, from TORCHELASTIC_RESTART_COUNT), so a restarted group runs clean."""
    fr = os.environ.get("PDT_FAULT_RANK")
    fs = os.environ.get("PDT_FAULT_STEP")
    if fr is None or fs is None:
        return
    if os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") != os.environ.get("PDT_FAULT_RESTART", "0"):
        return
    rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
    if rank != int(fr) or step != int(fs):
        return
    mode = os.environ.get("PDT_FAULT_MODE", "exit")
    if mode == "exit":
        print(f"[fault] rank {rank} exiting at step {step}", file=sys.stderr, flush=True)
        os._exit(17)
    if mode == "raise":
        raise InjectedFault(f"injected fault on rank {rank} at step {step}")
    if mode == "hang":
        while True:
            time.sleep(1)
    if mode == "delay":
        time.sleep(float(os.environ.get("PDT_FAULT_DELAY", "5")))
