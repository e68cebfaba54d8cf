"""Selective activation recomputation: keep the GEMM outputs, recompute the cheap ops in backward.

Whole-layer checkpointing (torch.utils.checkpoint) re-runs a transformer block's forward in backward -- its GEMMs
included, ~1/3 of the step again.  Here a tensor that a cheap op produced (a norm output, the attention output,
the SwiGLU output) is tagged with a *recipe* (``tag``): inside ``selective_recompute()`` autograd's saved-tensor
pack hook stores the recipe instead of the tensor, so the tensor is freed after forward, and the unpack hook
re-runs the recipe under no_grad when a backward node needs it.  The GEMM outputs those recipes read (the qkv
projection, the gate/up projection) and the residual stream stay saved, so no GEMM runs twice.

A recipe may produce several tensors (flash attention's output and log-sum-exp) and be unpacked by several
nodes (the output projection's dW and the attention backward): it runs once and its results are held until the
last node that packed one of them has unpacked it.  The recomputed values are bitwise equal to the forward's
(deterministic kernels: each recipe calls the exact kernel its tensor came from, on the exact saved inputs).

Used by models/llama.py (``LlamaConfig.checkpoint_policy = "selective"``), BASELINE.json config 5.
"""
from __future__ import annotations

import contextlib

import torch

_ACTIVE = [0]


class Recipe:
    """fn() -> tuple of tensors, recomputed on first unpack and dropped after the last one."""

    __slots__ = ("fn", "pending", "cache", "runs")

    def __init__(self, fn):
        self.fn, self.pending, self.cache, self.runs = fn, 0, None, 0

    def get(self, index):
        if self.cache is None:
            with torch.no_grad():
                out = self.fn()
            self.cache = out if isinstance(out, tuple) else (out,)
            self.runs += 1
        return self.cache[index]

    def hold(self):
        """One more consumer that will call ``get`` (and then ``release``) outside the saved-tensor hooks."""
        self.pending += 1

    def release(self):
        self.pending -= 1
        if self.pending <= 0:
            self.cache = None


class _Packed:
    __slots__ = ("recipe", "index", "view")

    def __init__(self, recipe, index, view):
        self.recipe, self.index, self.view = recipe, index, view


def tag(t: torch.Tensor, recipe: Recipe, index: int = 0, view=None) -> torch.Tensor:
    """Mark ``t`` as recomputable: ``view(recipe.get(index))`` (or the result itself) reproduces it."""
    if _ACTIVE[0]:
        t._pdt_recipe = (recipe, index, view)
    return t


def active() -> bool:
    return _ACTIVE[0] > 0


def _pack(t):
    r = getattr(t, "_pdt_recipe", None)
    if r is None:
        return t
    recipe, index, view = r
    recipe.pending += 1
    return _Packed(recipe, index, view)


def _unpack(p):
    if not isinstance(p, _Packed):
        return p
    rc = p.recipe
    out = rc.get(p.index)
    if p.view is not None:
        out = p.view(out)
    rc.release()
    return out


@contextlib.contextmanager
def selective_recompute(enabled: bool = True):
    """Within this context, saved activations tagged with a recipe are stored as that recipe."""
    if not enabled:
        yield
        return
    _ACTIVE[0] += 1
    try:
        with torch.autograd.graph.saved_tensors_hooks(_pack, _unpack):
            yield
    finally:
        _ACTIVE[0] -= 1
