"""FusedAdamW: torch.optim-compatible AdamW whose step is ONE gfx950 multi-tensor launch per
(param group, grad dtype).

* ``param_groups`` / ``state_dict`` layout identical to torch.optim.AdamW
  ({state: {idx: {step, exp_avg, exp_avg_sq}}, param_groups: [...]}, torch/optim/optimizer.py:677-760),
  so LR schedulers (OneCycleLR cycling betas, Stoke-DDP.py:300) and checkpoints interoperate.
* Sync-free mixed precision: ``step(grad_scale=t, found_inf=f)`` takes device scalars produced by the
  fused clip / unscale kernels; no host round trip between backward and the update.
* fp16 overflow: a step whose ``found_inf`` flag is set changes nothing -- parameters, moments and the
  step count (torch.amp.GradScaler skips ``optimizer.step()``, grad_scaler.py:360); the device count
  advances only when the flag is clear.
* Graph capture (``capturable=True``): the step count of each param group lives in a device tensor that a
  captured kernel increments, and the AdamW kernel derives its bias corrections from it, so a training step
  captured into a HIP graph (``utils.graphs.GraphedStep``) replays with the right step every time.  The
  learning rate is read when the step is captured (a schedule needs a re-capture).
* Sharded engines: a parameter carrying ``_pdt_lp_shard`` (FSDP / ZeRO flat shards) gets its bf16
  compute copy written by the same kernel (fused cast epilogue = the all-gather input).

Reference: AdamW(lr=1e-3, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-4) in Stoke-DDP.py:226-235
and Fairscale-DDP.py:78-86; math order torch/optim/adam.py:419-547.
"""
from __future__ import annotations

import torch
from torch.optim import Optimizer

from ..ops import multi_tensor as mt
from ..ops.multi_tensor import _dense
from ._grads import grad_of


def _same_layout(g, p) -> bool:
    """Same element order in memory: strides equal wherever the size is not 1 (a size-1 dimension's stride is
    arbitrary -- a contiguous [Cout, Cin, 1, 1] gradient of a channels_last 1x1-conv weight is already in its order,
    and autograd's layout contract accepts it as is)."""
    return g.shape == p.shape and all(gs == ps for gs, ps, n in zip(g.stride(), p.stride(), p.shape) if n != 1)


def _like(g, p):
    """The gradient in the parameter's memory layout (the kernel walks storage linearly)."""
    if p.dim() <= 1:
        return g if g.is_contiguous() else g.contiguous()
    if _same_layout(g, p) and _dense(g):
        return g
    return torch.empty_like(p, dtype=g.dtype).copy_(g)


class FusedAdamW(Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False,
                 decoupled=True, capturable=False, **_ignored):
        if amsgrad:
            raise ValueError("FusedAdamW: amsgrad is not supported")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, foreach=None, capturable=capturable, differentiable=False, fused=None,
                        decoupled=decoupled)
        super().__init__(params, defaults)
        self._tables = mt.TableCache()
        self._dsteps: dict = {}

    def _counters(self, present):
        """Device step counters for this step's parameters (those with a gradient), as [(counter, params)].

        torch counts steps per parameter.  Parameters whose step histories are identical share ONE device counter
        (one ``step_inc`` launch, one AdamW launch); a counter whose parameters did not all get a gradient this
        step is split (the ones stepping get a clone), so a parameter that skips steps -- an unused branch, a late
        unfreeze -- keeps its own count and bias correction.  Parameters without a counter (new state, or a host
        step loaded from a checkpoint) are grouped by their step value.  ``_dsteps``: id(counter) -> (counter,
        set of ids of the parameters sharing it)."""
        members = self._dsteps
        shared, fresh = {}, {}
        for p in present:
            c = self._init_state(p)["step"]
            ent = members.get(id(c))
            if ent is not None and ent[0] is c:
                shared.setdefault(id(c), []).append(p)
            else:
                fresh.setdefault((float(c), p.device), []).append(p)
        out = []
        for (v, dev), ps in fresh.items():
            c = torch.full((), v, dtype=torch.float32, device=dev)
            for p in ps:
                old = self.state[p]["step"]
                ent = members.get(id(old))
                if ent is not None and ent[0] is old:
                    ent[1].discard(id(p))
                    if not ent[1]:
                        del members[id(old)]
                self.state[p]["step"] = c
            members[id(c)] = (c, {id(p) for p in ps})
            out.append((c, ps))
        for cid, ps in shared.items():
            c, mem = members[cid]
            if len(ps) != len(mem):
                ids = {id(p) for p in ps}
                mem -= ids
                c = c.clone()
                members[id(c)] = (c, ids)
                for p in ps:
                    self.state[p]["step"] = c
            out.append((c, ps))
        return out

    def zero_grad(self, set_to_none: bool = True):
        """torch semantics for ``.grad``, except for engine-owned flat gradients: DDP's compute-dtype masters
        (``_pdt_zero_grad``) and parameters whose ``.grad`` is still a view of a DDP bucket flat
        (``_pdt_grad_flat``) get their flat zeroed in place -- ONE fill per flat instead of a None per
        parameter that the next forward would re-attach view by view (ResNet-50: 161 views, a host gap at
        every step start).  Those gradients therefore read as zeros, not None, after ``set_to_none=True`` (as
        with torch DDP's ``gradient_as_bucket_view``, whose views stay attached to the bucket).  A flat is filled
        whole only when every parameter viewing it (``_pdt_grad_members``) belongs to THIS optimizer; otherwise
        only this optimizer's own views are zeroed, so another optimizer stepping the same bucket later still
        sees its gradients."""
        mine = {id(p) for group in self.param_groups for p in group["params"]}
        flats, views, rest, owned = {}, [], [], {}
        for group in self.param_groups:
            for p in group["params"]:
                zero = getattr(p, "_pdt_zero_grad", None)
                if zero is not None:
                    flats[id(zero)] = zero
                    continue
                g = p.grad
                if g is None:
                    continue
                f = getattr(p, "_pdt_grad_flat", None)
                if f is not None and g._base is f:
                    ok = owned.get(id(f))
                    if ok is None:
                        members = getattr(p, "_pdt_grad_members", None)
                        ok = owned[id(f)] = members is not None and all(id(q) in mine for q in members)
                    if ok:
                        flats[id(f)] = f.zero_
                    else:
                        views.append(g)      # keep the view attached: the bucket reduction reads it in place
                    continue
                rest.append(p)
        for zero in flats.values():
            if getattr(zero, "_pdt_set_to_none", False):
                zero(set_to_none)      # an engine that keeps per-parameter gradients (DDP._steal_grads)
            else:
                zero()
        if views:
            torch._foreach_zero_(views)
        if set_to_none:
            for p in rest:
                p.grad = None
        elif rest:
            grads = []
            for p in rest:
                if p.grad.grad_fn is not None:
                    p.grad.detach_()
                else:
                    p.grad.requires_grad_(False)
                grads.append(p.grad)
            torch._foreach_zero_(grads)

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._dsteps.clear()     # device step counters are rebuilt from the loaded per-parameter steps
        for p in self.state:
            p._pdt_opt_state = True   # engines must not re-lay-out this parameter any more (DDP rebuild)

    def _init_state(self, p):
        st = self.state[p]
        if len(st) == 0:
            st["step"] = torch.tensor(0.0, dtype=torch.float32)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format, dtype=torch.float32)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format, dtype=torch.float32)
            p._pdt_opt_state = True
        return st

    @torch.no_grad()
    def step(self, closure=None, grad_scale: torch.Tensor | None = None, found_inf: torch.Tensor | None = None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            beta1, beta2 = group["betas"]
            lr = float(group["lr"]) if not torch.is_tensor(group["lr"]) else float(group["lr"].item())
            buckets = {}
            cap = bool(group.get("capturable", False))
            # An overflowed fp16 step (found_inf != 0) must leave params, moments AND the step count alone:
            # torch.amp.GradScaler skips optimizer.step() entirely.  With a device flag the count lives on the
            # device and advances conditionally (pdt_step_inc), so no host sync is needed; once a parameter has a
            # device count it keeps it (mixing the two counters would double-count).
            # GPU parameters always count on the device: one step_inc launch per counter instead of a host tensor
            # add + .item() per parameter (161 of them for ResNet-50: ~1 ms of host time per step, a GPU-idle gap
            # in front of the AdamW launch -- profiles/r3_s4h_resnet50-ddp_kernel_table.txt)
            on_gpu = bool(group["params"]) and group["params"][0].device.type == "cuda"
            dev_step = cap or on_gpu or (found_inf is not None and found_inf.device.type == "cuda") or any(
                id(self.state[p].get("step")) in self._dsteps for p in group["params"] if p in self.state)
            if found_inf is not None and found_inf.device.type != "cuda" and int(found_inf.reshape(-1)[0]) != 0:
                continue
            present = []
            for p in group["params"]:
                g = grad_of(p)
                if g is None:
                    continue
                if g.is_sparse:
                    raise RuntimeError("FusedAdamW does not support sparse gradients")
                if p.dtype != torch.float32:
                    raise TypeError("FusedAdamW keeps fp32 master params; wrap low-precision models with an "
                                    "engine (FSDP/ZeRO) or keep params fp32 and use autocast")
                present.append(p)
            counters = {}
            if dev_step:
                for c, ps in self._counters(present):
                    mt.step_inc_(c, found_inf)    # one device increment per counter (graph-capturable)
                    counters[id(c)] = c
                    for p in ps:
                        buckets.setdefault((grad_of(p).dtype, id(c), p.device), []).append(p)
            else:
                for p in present:
                    st = self._init_state(p)
                    st["step"] += 1
                    buckets.setdefault((grad_of(p).dtype, -int(st["step"].item()), p.device), []).append(p)
            used = set()
            for (gdt, ckey, dev), ps in buckets.items():
                dstep = counters.get(ckey)
                step = -ckey if dstep is None else 1
                grads = [_like(grad_of(p), p) for p in ps]
                ms = [self.state[p]["exp_avg"] for p in ps]
                vs = [self.state[p]["exp_avg_sq"] for p in ps]
                lps = [getattr(p, "_pdt_lp_shard", None) for p in ps]
                # the kernel's epilogue writes bf16 compute copies; an fp32 "copy" (a DDP compute-copy model's
                # batch-norm group) is refreshed by a plain copy after the step
                lp_other = [(p, x) for p, x in zip(ps, lps) if x is not None and x.dtype != torch.bfloat16]
                lps = [x if (x is not None and x.dtype == torch.bfloat16) else None for x in lps]
                has_lp = any(x is not None for x in lps)
                table = None
                if dev.type == "cuda":
                    cols = [ps, grads, ms, vs, lps if has_lp else [None] * len(ps)]
                    name = (gi, gdt, ckey if dstep is not None else 0)
                    used.add(name)
                    table = self._tables.get(name, cols)
                mt.adamw_step(ps, grads, ms, vs, lr=lr, beta1=beta1, beta2=beta2, eps=group["eps"],
                              weight_decay=group["weight_decay"], step=max(step, 1),
                              decoupled=group.get("decoupled", True), grad_scale=grad_scale, found_inf=found_inf,
                              out_bf16=lps if has_lp else None, table=table, dstep=dstep)
                with torch.no_grad():
                    for p, x in lp_other:
                        x.copy_(p)
                for p in ps:
                    if getattr(p, "_pdt_lp_shard", None) is not None:
                        p._pdt_lp_version = p._version   # compute copy already refreshed by the kernel
            if buckets:
                # tables of this group's counters that no longer exist (a split counter, a reloaded checkpoint)
                # are dropped, so their device tables do not pile up over a long run
                self._tables.retain(lambda n, gi=gi: n[0] != gi or n in used)
        return loss
