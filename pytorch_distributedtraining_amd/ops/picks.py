"""Per-shape kernel picks (hand GEMM vs hipBLASLt, 1x1 conv as GEMM vs MIOpen, BGRADB) and how ranks agree on them.

A pick is made where a shape is first met -- inside a forward or a backward -- by timing both arms on this rank
(``timed_choice``).  Nothing is communicated there: a collective issued from inside autograd would hang or
mismatch as soon as ranks meet different shapes (an uneven last batch, per-rank padding, rank-0-only eval), and an
engine built on a sub-group must never touch the default group.

Agreement is a separate, explicit step at a point every rank of an engine reaches together: ``agree(comm)`` gathers
every rank's (time_a, time_b) per pick over THAT engine's ``Comm`` (its group, not the default one) and, for the
picks every rank has made, sets the choice from the times summed over ranks -- so all ranks run the same kernels.
Picks only some ranks have met keep their local choice.  ``Trainer.step`` calls it after its first optimizer steps,
``bench.py`` after the warm-up steps.  Correctness never depends on it: gradients are averaged by the engines, so
per-rank kernel differences cannot desynchronise parameters; agreement only keeps ranks' step times alike.
"""
from __future__ import annotations

import torch

# (table id, normalised key) -> [table, key, time_a, time_b, margin, agreed]
_PENDING: dict = {}


def _norm(k):
    """A key that means the same on every rank: devices by type only (rank r's cuda:r), shapes as tuples."""
    if isinstance(k, torch.device):
        return k.type
    if isinstance(k, (tuple, list, torch.Size)):
        return tuple(_norm(v) for v in k)
    if isinstance(k, torch.dtype):
        return str(k)
    return k


def _timed_ms(fn, iters: int = 3) -> float:
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1)


def record(table: dict | None, key, name: str, ta: float, tb: float, margin: float) -> bool:
    """Register one rank-local timing and return the local choice (``fa`` faster than ``margin`` x ``fb``)."""
    c = ta < margin * tb
    if table is not None:
        _PENDING[(name, repr(_norm(key)))] = [table, key, ta, tb, margin, False]
    return c


def timed_choice(fa, fb, margin: float = 1.0, table: dict | None = None, key=None, name: str = "") -> bool:
    """Whether ``fa`` runs faster than ``margin`` x ``fb`` on this rank -- no collective (module docstring).
    With ``table`` / ``key`` the timing is kept so that ``agree`` can later overwrite ``table[key]`` with the
    choice all ranks share.  The env switches of each pick (PDT_NT_HIP, PDT_WGRAD_HIP, PDT_CONV1X1) pin the
    choice outright and never get here."""
    return record(table, key, name, _timed_ms(fa), _timed_ms(fb), margin)


def agree(comm) -> int:
    """Collective over ``comm`` (every rank of its group calls it at the same point): make the picks every rank
    has timed identical on all ranks.  Returns how many picks were agreed in this call."""
    if comm is None or comm.world_size <= 1:
        return 0
    mine = {k: (v[2], v[3]) for k, v in _PENDING.items() if not v[5]}
    allp = comm.all_gather_object(mine)
    common = set(mine)
    for d in allp:
        common &= set(d)
    n = 0
    for k in sorted(common):
        ta = sum(d[k][0] for d in allp)
        tb = sum(d[k][1] for d in allp)
        ent = _PENDING[k]
        ent[0][ent[1]] = ta < ent[4] * tb
        ent[5] = True
        n += 1
    return n


def pending() -> int:
    """Picks timed on this rank and not yet agreed."""
    return sum(1 for v in _PENDING.values() if not v[5])


def clear():
    _PENDING.clear()
