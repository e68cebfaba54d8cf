"""Gradient slots: where a sharded engine wants a parameter's gradient written.

FSDP (parallel/fsdp.py) reduce-scatters each unit's gradient as ONE flat buffer.  Instead of autograd assembling
that flat from per-parameter gradients (a ``cat`` of every weight gradient per unit per backward), the unit
allocates the flat when its backward starts and registers one slot per parameter here, keyed by the parameter
view's (storage, offset) -- the saved weight a Linear's backward unpacks is a view of the same storage.  The
framework ops that produce large weight gradients (``ops.linear``) ``claim`` the slot and write dW straight into
it (the GEMM's output), returning no gradient for that input; gradients from any other consumer still arrive
through autograd and are added by the unit.

A slot claimed twice in one backward (a weight used by two framework ops) is accumulated into: ``claim`` returns
``accumulate=True`` for every claim after the first.
"""
from __future__ import annotations

import torch

_SLOTS: dict = {}


def _key(t: torch.Tensor):
    return (t.untyped_storage().data_ptr(), t.storage_offset())


def register(view: torch.Tensor, dst: torch.Tensor, owner, index: int) -> tuple:
    """Gradients for parameter ``view`` go to ``dst`` (same shape) until ``release``; returns the slot key."""
    k = _key(view)
    _SLOTS[k] = [dst, False, owner, index]
    return k


def release(keys) -> None:
    for k in keys:
        _SLOTS.pop(k, None)


def claim(w: torch.Tensor):
    """(dst, accumulate) for parameter view ``w`` if it has a slot with its shape and dtype, else None.  The first
    claim of a backward overwrites ``dst``; later ones must add to it."""
    if not _SLOTS:
        return None
    ent = _SLOTS.get(_key(w))
    if ent is None or ent[0].shape != w.shape or ent[0].dtype != w.dtype:
        return None
    acc = ent[1]
    ent[1] = True
    ent[2].slot_written(ent[3])
    return ent[0], acc


def is_sharded_param(w: torch.Tensor) -> bool:
    """A parameter view installed by a sharded engine (its framework ops must run their own backward so they can
    claim the slot, on CPU too)."""
    return getattr(w, "_pdt_fsdp_unit", None) is not None
