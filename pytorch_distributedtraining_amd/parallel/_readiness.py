"""Bucket readiness for the reducers (DDP, ShardedDataParallel): which gradient buckets are complete, released
strictly in plan order so every rank issues the same collective sequence.

Two implementations behind one interface:
  * native (default when ``_pdt_hooks`` is built): C++ post hooks on the parameters' AccumulateGrad nodes
    (csrc/hooks/reducer_hooks.cpp, the mechanism of torch's C++ Reducer); Python runs once per ready bucket
    and once per backward, not once per parameter;
  * python: a ``register_post_accumulate_grad_hook`` closure per parameter over the native ``ReadyTracker``
    -- used while a reducer still records the gradient order (DDP's first-iteration bucket rebuild) or when
    ``PDT_NATIVE_HOOKS=0``.
"""
from __future__ import annotations

import os

from ..utils.native import require_runtime

_hooks_mod = None


def native_hooks():
    """The ``_pdt_hooks`` module, or None (not built / disabled)."""
    global _hooks_mod
    if os.environ.get("PDT_NATIVE_HOOKS", "1") != "1":
        return None
    if _hooks_mod is None:
        try:
            from .. import _pdt_hooks as m   # noqa: F401
            _hooks_mod = m
        except ImportError:
            try:
                from .. import _build
                _build.build_hooks()
                from .. import _pdt_hooks as m   # noqa: F811
                _hooks_mod = m
            except Exception:   # pragma: no cover - no toolchain
                _hooks_mod = False
    return _hooks_mod or None


class Readiness:
    def __init__(self, params, buckets, on_first, on_ready, observe=None, native: bool = True):
        """params: the reducer's parameters (index = position); buckets: parameter indices per bucket in
        release order; on_first(): first ready gradient of a backward; on_ready(bucket); observe(idx): if
        given, called for every ready parameter (forces the Python path)."""
        self.n = len(params)
        mod = native_hooks() if native and observe is None else None
        self._br = None
        self._handles = []
        self.enabled = True
        self.observing = observe is not None
        if mod is not None:
            self._br = mod.BucketReadiness([list(b) for b in buckets], self.n, on_first, on_ready)
            self._br.attach(list(params))
            self.kind = "native"
        else:
            self._tracker = require_runtime().ReadyTracker([list(b) for b in buckets], self.n)
            self._on_first, self._on_ready, self._observe = on_first, on_ready, observe
            self._handles = [p.register_post_accumulate_grad_hook(self._make_hook(i))
                             for i, p in enumerate(params) if p.requires_grad]
            self._count = 0
            self.kind = "python"

    def _make_hook(self, idx):
        def hook(_p):
            if not self.enabled:
                return
            if self._observe is not None:
                self._observe(idx)
            if self._count == 0:
                self._on_first()
            self._count += 1
            for b in self._tracker.mark_ready(idx):
                self._on_ready(b)
        return hook

    def set_enabled(self, on: bool):
        self.enabled = bool(on)
        if self._br is not None:
            self._br.set_enabled(self.enabled)

    def flush(self):
        return list(self._br.flush()) if self._br is not None else list(self._tracker.flush())

    def all_released(self) -> bool:
        return self._br.all_released() if self._br is not None else self._tracker.all_launched()

    def reset(self):
        if self._br is not None:
            self._br.reset()
        else:
            self._tracker.reset()
            self._count = 0

    def remove(self):
        if self._br is not None:
            self._br.detach()
            self._br = None
        for h in self._handles:
            h.remove()
        self._handles = []


class NullReadiness:
    """One rank: no collective to launch, so no hook at all.  (Native hooks hold the parameters' AccumulateGrad
    nodes, which remember the stream they were created on; a HIP-graph capture on another stream then has
    autograd synchronise with that uncaptured stream -- torch 2.10 warns "AccumulateGrad node's stream does
    not match" -- and ROCm faults ending such a capture.  Trainer.graph runs on exactly this one-rank path.)"""
    kind = "none"
    observing = False
    enabled = False

    def set_enabled(self, on: bool):
        pass

    def flush(self):
        return []

    def all_released(self) -> bool:
        return True

    def reset(self):
        pass

    def remove(self):
        pass

