"""Process-group bootstrap: env:// rendezvous (MASTER_ADDR / MASTER_PORT,
RANK / WORLD_SIZE / LOCAL_RANK as set by torchrun or our launcher), one process per GPU, RCCL
('nccl') on MI355X and gloo on CPU, explicit timeout, device bound from LOCAL_RANK.
Fixes the reference's LOCAL_RANK handling (Stoke-DDP.py:153,191: ``int(os.getenv('LOCAL_RANK'))``
raises when unset) and its hard-coded gloo backend (Fairscale-DDP.py:27)."""
from __future__ import annotations

import datetime
import os
import socket

import torch
import torch.distributed as dist


def env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    try:
        return int(v) if v not in (None, "", "None") else default
    except ValueError:
        return default


def local_rank() -> int:
    return env_int("LOCAL_RANK", 0)


def find_free_port(host: str = "127.0.0.1") -> str:
    """Bind port 0 and return the chosen port as a string (the reference's test_dist_gpu helper,
    Fairscale-DDP.py:123)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        return str(s.getsockname()[1])


def init_distributed(backend: str | None = None, timeout_s: float = 1800.0, rank: int | None = None,
                     world_size: int | None = None, init_method: str = "env://", device_bind: bool = True):
    """Initialise the default process group if needed; returns (rank, world_size, device)."""
    world_size = env_int("WORLD_SIZE", 1) if world_size is None else world_size
    rank = env_int("RANK", 0) if rank is None else rank
    lr = local_rank()
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    if torch.cuda.is_available() and lr >= torch.cuda.device_count():
        # more local ranks than devices: ranks share GPUs round-robin (the 1-GPU rehearsal of a multi-rank
        # run over gloo + the xGMI kernels); RCCL itself refuses two ranks on one device, loudly
        lr = lr % torch.cuda.device_count()
    device = torch.device("cuda", lr) if use_gpu else torch.device("cpu")
    if use_gpu and device_bind:
        torch.cuda.set_device(device)
    if world_size > 1 and not dist.is_initialized():
        from .fault import configure_watchdog
        configure_watchdog(timeout_s)    # RCCL async error handling: a dead peer ends the job, never a hang
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if use_gpu else "gloo"
        kw = dict(backend=backend, init_method=init_method, rank=rank, world_size=world_size,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl" and use_gpu:
            kw["device_id"] = device
        dist.init_process_group(**kw)
    if dist.is_initialized():
        rank, world_size = dist.get_rank(), dist.get_world_size()
    return rank, world_size, device


def destroy():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def is_main_process() -> bool:
    return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0
