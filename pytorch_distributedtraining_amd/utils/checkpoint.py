"""Checkpoint IO in the Stoke envelope layout.

One file per save: ``{path}/stoke-{name}-backward-step-{N}.{ext}`` holding
    {backward_step, grad_accum_step, optimizer_step, stoke_status, model_state_dict,
     optimizer_state_dict, scaler_state_dict, extras}
* model_state_dict: the UNWRAPPED model's full state dict (no 'module.' prefix; FSDP/ZeRO engines
  hand over full unflattened fp32 tensors), so ``model.load_state_dict`` works on a plain model;
* optimizer_state_dict: torch layout {state: {idx: {step, exp_avg, exp_avg_sq}}, param_groups}
  (ZeRO shards consolidated to rank 0 first);
* only plain types -> loadable with ``torch.load(weights_only=True)`` (torch/serialization.py:77-78).
Only rank 0 writes, with barriers around the write (reference: stoke_model.save at Stoke-DDP.py:142-145).
Also: pretrained import accepting ``{'params': sd}`` or a raw state dict (Stoke-DDP.py:209-213).
"""
from __future__ import annotations

import enum
import os

import torch


def _plain(x):
    if torch.is_tensor(x):
        return x.detach().cpu()
    if isinstance(x, dict):
        return {(k if isinstance(k, (str, int, float, bool)) or k is None else str(k)): _plain(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_plain(v) for v in x) if isinstance(x, list) else tuple(_plain(v) for v in x)
    if isinstance(x, enum.Enum):
        return x.value
    if isinstance(x, torch.dtype):
        return str(x)
    if isinstance(x, (str, int, float, bool)) or x is None:
        return x
    return str(x)


def checkpoint_tag(name: str, backward_step: int) -> str:
    return f"stoke-{name}-backward-step-{backward_step}"


def save_checkpoint(path: str, name: str, *, model_state, optimizer_state=None, scaler_state=None,
                    backward_step: int = 0, grad_accum_step: int = 0, optimizer_step: int = 0, status=None,
                    extras=None, extension: str = "pt", rank: int = 0, barrier=None, create_directory=True):
    """Write the envelope on rank 0; returns (path, tag) on every rank."""
    tag = checkpoint_tag(name, backward_step)
    if barrier:
        barrier()
    if rank == 0:
        if create_directory:
            os.makedirs(path, exist_ok=True)
        payload = {
            "backward_step": int(backward_step),
            "grad_accum_step": int(grad_accum_step),
            "optimizer_step": int(optimizer_step),
            "stoke_status": _plain(status or {}),
            "model_state_dict": _plain(model_state),
            "optimizer_state_dict": _plain(optimizer_state) if optimizer_state is not None else None,
            "scaler_state_dict": _plain(scaler_state) if scaler_state is not None else None,
            "extras": _plain(extras) if extras is not None else None,
        }
        f = os.path.join(path, f"{tag}.{extension}")
        tmp = f + ".tmp"
        torch.save(payload, tmp)
        os.replace(tmp, f)  # atomic: a crash never leaves a half-written checkpoint
    if barrier:
        barrier()
    return path, tag


def load_checkpoint(path: str, tag: str, extension: str = "pt", map_location="cpu"):
    f = os.path.join(path, f"{tag}.{extension}") if not tag.endswith("." + extension) else os.path.join(path, tag)
    return torch.load(f, map_location=map_location, weights_only=True)


def latest_checkpoint(path: str, name: str | None = None, extension: str = "pt"):
    """Tag of the newest envelope in ``path`` (highest backward step), or None -- for auto-resume."""
    if not os.path.isdir(path):
        return None
    best, best_step = None, -1
    for f in os.listdir(path):
        if not (f.startswith("stoke-") and f.endswith("." + extension)) or ".tmp" in f:
            continue
        stem = f[: -len(extension) - 1]
        if name is not None and not stem.startswith(f"stoke-{name}-"):
            continue
        try:
            step = int(stem.rsplit("-backward-step-", 1)[1])
        except (IndexError, ValueError):
            continue
        if step > best_step:
            best, best_step = stem, step
    return best


def load_pretrained(model: torch.nn.Module, src, key: str = "params", strict: bool = True):
    """Load ``{key: sd}`` or a raw state dict (path or dict) into ``model`` (weights_only load)."""
    sd = torch.load(src, map_location="cpu", weights_only=True) if isinstance(src, (str, os.PathLike)) else src
    if isinstance(sd, dict) and key in sd and isinstance(sd[key], dict):
        sd = sd[key]
    return model.load_state_dict(sd, strict=strict)
