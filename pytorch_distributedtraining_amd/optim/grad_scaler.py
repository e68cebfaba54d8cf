"""Dynamic loss scaling for fp16 (bf16 needs none) -- a sharded-aware GradScaler.

Semantics of torch.amp.GradScaler (grad_scaler.py:123-129 defaults: init 2**16, growth 2.0,
backoff 0.5, interval 2000; reference AMPConfig(init_scale=2**14) Stoke-DDP.py:182-184) and of the
sharded variant that all-reduces ``found_inf`` (fsdp/sharded_grad_scaler.py:262-283).

MI355X design: unscale + inf-check + clip are ONE fused norm pass producing device scalars
(``grad_multiplier``, ``found_inf``) that the fused AdamW consumes -- gradients are never rewritten
and the only host sync is the scale update (``found_inf.item()``), as in torch.
"""
from __future__ import annotations

import torch

from .clip import clip_grad_norm_


class GradScaler:
    def __init__(self, init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000,
                 enabled=True, comm=None, sharded=False):
        self.enabled = enabled
        self._scale = float(init_scale)
        self.growth_factor, self.backoff_factor, self.growth_interval = growth_factor, backoff_factor, growth_interval
        self._growth_tracker = 0
        self.comm, self.sharded = comm, sharded
        self._pending = None

    def get_scale(self) -> float:
        return self._scale if self.enabled else 1.0

    def scale(self, loss):
        return loss * self._scale if self.enabled else loss

    def unscale_and_clip(self, parameters, max_norm: float = 0.0):
        """Compute (norm, multiplier, found_inf) without touching the gradients."""
        inv = 1.0 / self.get_scale()
        norm, coef, found = clip_grad_norm_(parameters, max_norm if max_norm else 0.0, comm=self.comm,
                                            sharded=self.sharded, inv_scale=inv, apply=False)
        if self.comm is not None and self.comm.world_size > 1 and not self.sharded:
            # replicated grads (DDP): every rank saw the same grads, found_inf already consistent
            pass
        self._pending = (coef, found)
        return norm, coef, found

    def step(self, optimizer, parameters=None, max_norm: float = 0.0):
        if self._pending is None:
            params = parameters if parameters is not None else [p for g in optimizer.param_groups for p in g["params"]]
            self.unscale_and_clip(params, max_norm)
        coef, found = self._pending
        optimizer.step(grad_scale=coef, found_inf=found)
        return found

    def update(self):
        if not self.enabled or self._pending is None:
            self._pending = None
            return
        _, found = self._pending
        self._pending = None
        if int(found.reshape(-1)[0].item()) != 0:
            self._scale *= self.backoff_factor
            self._growth_tracker = 0
        else:
            self._growth_tracker += 1
            if self._growth_tracker == self.growth_interval:
                self._scale *= self.growth_factor
                self._growth_tracker = 0

    def state_dict(self):
        return {"scale": self._scale, "growth_factor": self.growth_factor, "backoff_factor": self.backoff_factor,
                "growth_interval": self.growth_interval, "_growth_tracker": self._growth_tracker}

    def load_state_dict(self, sd):
        self._scale = float(sd["scale"])
        self.growth_factor = sd.get("growth_factor", self.growth_factor)
        self.backoff_factor = sd.get("backoff_factor", self.backoff_factor)
        self.growth_interval = sd.get("growth_interval", self.growth_interval)
        self._growth_tracker = sd.get("_growth_tracker", 0)
