"""World-W rehearsal on ONE device through torch's ``fake`` process-group backend.

This process plays rank R of a world of W.  Every engine (DDP, SyncBN, OSS, ShardedDDP, FSDP) then takes its
multi-rank path -- for ``Comm`` that is the nccl branch (``reduce_scatter_tensor`` with AVG,
``all_gather_into_tensor``, ``all_reduce``), the same code RCCL runs on an 8-GPU node -- with the shard shapes,
bucket plans and per-step collective counts of world W, while the collectives move no data.  ``Recorder`` logs
every torch.distributed call the engines make (name, op, shapes, dtypes) so a test can assert the contract.
The reference trains on 4 ranks (Stoke-DDP.py:1-2, Fairscale-DDP.py:112-133); SURVEY §2.E lists the collectives.
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist

_NAMES = ("all_reduce", "reduce_scatter_tensor", "all_gather_into_tensor", "all_gather", "broadcast", "reduce",
          "barrier", "all_gather_object", "broadcast_object_list")


@contextlib.contextmanager
def fake_world(rank: int, world: int):
    from torch.testing._internal.distributed.fake_pg import FakeStore
    if dist.is_initialized():
        raise RuntimeError("a default process group already exists in this process")
    dist.init_process_group("fake", rank=rank, world_size=world, store=FakeStore())
    try:
        yield
    finally:
        dist.destroy_process_group()


def _desc(x):
    if torch.is_tensor(x):
        return ("T", tuple(x.shape), x.dtype, x.device.type)
    if isinstance(x, (list, tuple)) and x and all(torch.is_tensor(t) for t in x):
        return ("L", len(x), tuple(x[0].shape), x[0].dtype)
    return None


class Recorder:
    """Context manager: every torch.distributed collective called inside is recorded as a dict
    {name, args (tensor descriptors), op (ReduceOp name or None)} and then run (on the fake group)."""

    def __init__(self):
        self.calls: list[dict] = []
        self._saved = {}

    def __enter__(self):
        for n in _NAMES:
            real = getattr(dist, n)
            self._saved[n] = real

            def wrap(*a, _n=n, _real=real, **k):
                op = k.get("op")
                self.calls.append({"name": _n, "args": [_desc(x) for x in a],
                                   "op": None if op is None else str(op).split(".")[-1].upper(),
                                   "group": k.get("group")})
                return _real(*a, **k)
            setattr(dist, n, wrap)
        return self

    def __exit__(self, *exc):
        for n, f in self._saved.items():
            setattr(dist, n, f)
        return False

    def of(self, name):
        return [c for c in self.calls if c["name"] == name]

    def reset(self):
        self.calls.clear()


def check_nccl_branch(rec: Recorder, world: int, max_all_reduce_numel: int | None = None):
    """No gloo emulation anywhere: a reduce-scatter never arrives as an all_reduce of the full buffer plus a
    local slice, an all-gather never as a list of per-rank views."""
    assert not rec.of("all_gather"), "gloo-style list all_gather used where all_gather_into_tensor belongs"
    for c in rec.of("reduce_scatter_tensor"):
        out, inp = c["args"][0], c["args"][1]
        n_out = int(torch.Size(out[1]).numel())
        n_in = int(torch.Size(inp[1]).numel())
        assert n_in == world * n_out, (n_in, n_out)
        assert out[2] == inp[2]
    for c in rec.of("all_gather_into_tensor"):
        out, inp = c["args"][0], c["args"][1]
        assert int(torch.Size(out[1]).numel()) == world * int(torch.Size(inp[1]).numel())
        assert out[2] == inp[2]
    if max_all_reduce_numel is not None:
        for c in rec.of("all_reduce"):
            assert int(torch.Size(c["args"][0][1]).numel()) <= max_all_reduce_numel, c
