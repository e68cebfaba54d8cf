"""Gradient clipping by global L2 norm with one fused norm launch and (for sharded engines) ONE
1-float all-reduce.  Semantics of torch.nn.utils.clip_grad_norm_ (clip_grad.py:50-186:
coef = max_norm / (total_norm + 1e-6), clamped to 1); reference config ClipGradNormConfig(max_norm=0.1,
norm_type=2.0) in Stoke-DDP.py:253.  With ``apply=False`` the coefficient is returned as a device
scalar so the caller can fold it into the fused AdamW step (no extra pass over the gradients).
"""
from __future__ import annotations

import torch

from ..ops import multi_tensor as mt
from ._grads import grad_of


def _device(parameters, comm):
    if parameters:
        return parameters[0].device
    if comm is not None and comm.backend == "nccl" and torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def grad_norm_sq(parameters, comm=None, sharded=False) -> torch.Tensor:
    parameters = list(parameters)
    grads = [grad_of(p) for p in parameters if grad_of(p) is not None]
    if grads:
        total = mt.l2norm_sq(grads)
    else:
        # a rank that owns no gradient (more ranks than sharded tensors) still joins the all-reduce below,
        # or every other rank would wait for it forever
        total = torch.zeros(1, dtype=torch.float32, device=_device(parameters, comm))
    if sharded and comm is not None and comm.world_size > 1:
        comm.all_reduce(total, "sum")
    return total


def clip_grad_norm_(parameters, max_norm: float, norm_type: float = 2.0, comm=None, sharded: bool = False,
                    inv_scale=1.0, apply: bool = True):
    """Returns (total_norm, grad_multiplier, found_inf) device tensors.

    sharded=True: each rank holds a disjoint shard of the gradients (ZeRO/FSDP) -> the squared norms
    are summed across ranks.  inv_scale: 1/loss_scale for fp16 (the norm is of the unscaled grads).
    apply=True multiplies the grads in place (torch semantics); False leaves that to the optimizer."""
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    parameters = list(parameters)
    if norm_type != 2.0:
        grads = [grad_of(p) for p in parameters if grad_of(p) is not None]
        dev = _device(parameters, comm)
        if norm_type == float("inf"):
            local = torch.stack([g.detach().abs().max().float() for g in grads]).max().reshape(1) if grads \
                else torch.zeros(1, device=dev)
            if sharded and comm is not None:
                comm.all_reduce(local, "max")
            total = local
        else:
            local = sum((g.detach().float().abs().pow(norm_type).sum() for g in grads),
                        torch.zeros((), device=dev)).reshape(1)
            if sharded and comm is not None:
                comm.all_reduce(local, "sum")
            total = local.pow(1.0 / norm_type)
        inv = inv_scale if not torch.is_tensor(inv_scale) else inv_scale.float()
        total = total * inv
        coef = torch.clamp(max_norm / (total + 1e-6), max=1.0) * inv
        found = (~torch.isfinite(total)).to(torch.int32)
        if apply:
            mt.scale_(grads, coef)
        return total, coef, found
    sq = grad_norm_sq(parameters, comm, sharded)
    norm, coef, found = mt.clip_coef(sq, max_norm, inv_scale)
    if apply:
        mt.scale_([grad_of(p) for p in parameters if grad_of(p) is not None], coef)
    return norm, coef, found
