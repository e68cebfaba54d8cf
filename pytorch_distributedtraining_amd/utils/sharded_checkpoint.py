"""Sharded (per-rank) checkpoints for the flat-parameter engine -- the fast path of SURVEY.md §5.4.

A full state dict of Llama-3 8B is ~32 GB of fp32 gathered on one rank; with 288 GB HBM per GPU the
natural layout is "every rank writes what it owns":
    {path}/{tag}.rank{r}-of-{W}.pt   flat fp32 master shard + optimizer-state shards of every unit
    {path}/{tag}.manifest.json       world size, per-unit flat layout (param fqns, offsets, shapes)
Save is embarrassingly parallel (no collective beyond a barrier).  Loading works at the SAME or a
DIFFERENT world size (each rank rebuilds the units' full flat buffers from all shard files and cuts
its own slice), and ``consolidate_to_full`` converts a sharded checkpoint to the full, unflattened
torch layout used by the Stoke envelope -- all with weights_only loads.
"""
from __future__ import annotations

import json
import os

import torch


def _unit_meta(u):
    return {"name": u.name, "total": u.total, "shard_numel": u.shard_numel,
            "params": [{"fqn": fqn, "shape": list(shape), "offset": off, "numel": n}
                       for (_m, _pn, fqn, shape), off, n in zip(u.params, u.offsets, u.numels)]}


def save_sharded(path: str, tag: str, fsdp, optimizer=None, extras=None):
    os.makedirs(path, exist_ok=True)
    comm = fsdp.comm
    r, W = comm.rank, comm.world_size
    units = fsdp.all_units()
    payload = {"flat_params": [u.flat_param.detach().cpu() for u in units], "optim": None, "extras": extras}
    if optimizer is not None:
        states = []
        for u in units:
            st = optimizer.state.get(u.flat_param, {})
            states.append({k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in st.items()})
        groups = [{k: v for k, v in g.items() if k != "params"} for g in optimizer.param_groups]
        payload["optim"] = {"states": states, "param_groups": groups}
    f = os.path.join(path, f"{tag}.rank{r}-of-{W}.pt")
    torch.save(payload, f + ".tmp")
    os.replace(f + ".tmp", f)
    if r == 0:
        man = {"world_size": W, "units": [_unit_meta(u) for u in units], "format": "pdt-sharded-v1"}
        with open(os.path.join(path, f"{tag}.manifest.json"), "w") as fh:
            json.dump(man, fh, indent=1)
    comm.barrier()
    return path, tag


def _read_all(path, tag):
    with open(os.path.join(path, f"{tag}.manifest.json")) as fh:
        man = json.load(fh)
    W = man["world_size"]
    shards = [torch.load(os.path.join(path, f"{tag}.rank{r}-of-{W}.pt"), map_location="cpu", weights_only=True)
              for r in range(W)]
    return man, shards


def _full_flat(man, shards, ui, key=None):
    parts = []
    for sh in shards:
        if key is None:
            parts.append(sh["flat_params"][ui])
        else:
            parts.append(sh["optim"]["states"][ui][key])
    return torch.cat([p.reshape(-1).float() for p in parts])


def consolidate_to_full(path: str, tag: str):
    """-> (model_state_dict, optimizer_state_dict) in the full torch layout (keyed by fqn / param index)."""
    man, shards = _read_all(path, tag)
    sd, ostate = {}, {}
    idx = 0
    has_optim = shards[0].get("optim") is not None
    for ui, u in enumerate(man["units"]):
        full = _full_flat(man, shards, ui)
        st0 = shards[0]["optim"]["states"][ui] if has_optim else {}
        fulls = {k: _full_flat(man, shards, ui, k) for k, v in st0.items() if torch.is_tensor(v) and v.dim() == 1}
        for p in u["params"]:
            o, n = p["offset"], p["numel"]
            sd[p["fqn"]] = full[o:o + n].view(p["shape"]).clone()
            if has_optim and fulls:
                ent = {k: v[o:o + n].view(p["shape"]).clone() for k, v in fulls.items()}
                for k, v in st0.items():
                    if k not in ent:
                        ent[k] = v
                ostate[idx] = ent
            idx += 1
    osd = None
    if has_optim:
        osd = {"state": ostate, "param_groups": [dict(g, params=list(range(idx)))
                                                 for g in shards[0]["optim"]["param_groups"][:1]]}
    return sd, osd


def load_sharded(path: str, tag: str, fsdp, optimizer=None):
    """Load into an FSDP model of ANY world size (re-slicing the flat buffers)."""
    man, shards = _read_all(path, tag)
    comm = fsdp.comm
    units = fsdp.all_units()
    if len(units) != len(man["units"]):
        raise ValueError("sharded checkpoint unit structure differs from the model")
    has_optim = optimizer is not None and shards[0].get("optim") is not None
    for ui, u in enumerate(units):
        mu = man["units"][ui]
        if [p["fqn"] for p in mu["params"]] != [fqn for (_m, _pn, fqn, _s) in u.params]:
            raise ValueError(f"unit {ui}: parameter list differs from the checkpoint")
        full = _full_flat(man, shards, ui)
        s0 = comm.rank * u.shard_numel

        def cut(t):
            out = torch.zeros(u.shard_numel, dtype=torch.float32)
            # padding layouts may differ across world sizes: copy parameter by parameter
            for p, off_new, n in zip(mu["params"], u.offsets, u.numels):
                a, b = max(off_new, s0), min(off_new + n, s0 + u.shard_numel)
                if a < b:
                    out[a - s0:b - s0] = t[p["offset"] + (a - off_new): p["offset"] + (b - off_new)]
            return out.to(u.flat_param.device)

        with torch.no_grad():
            u.flat_param.copy_(cut(full))
        u.refresh_lp(force=True)
        if has_optim:
            st0 = shards[0]["optim"]["states"][ui]
            new = {}
            for k, v in st0.items():
                if torch.is_tensor(v) and v.dim() == 1:
                    new[k] = cut(_full_flat(man, shards, ui, k))
                else:
                    new[k] = v.clone() if torch.is_tensor(v) else v
            optimizer.state[u.flat_param] = new
    return shards[comm.rank if comm.rank < len(shards) else 0].get("extras")
