"""ZeRO-1 optimizer-state sharding (``OSS``) and ZeRO-2 gradient sharding (``ShardedDataParallel``).

API-compatible with what the reference drives from Fairscale:
  * ``OSS(params=model.parameters(), optim=AdamW, lr=..., betas=..., eps=..., weight_decay=...)`` and
    ``.step()`` (Fairscale-DDP.py:86,101), ``broadcast_fp16`` (FairscaleOSSConfig, Stoke-DDP.py:197-199),
    ``consolidate_state_dict(recipient_rank)`` + ``state_dict()`` (Stoke save path),
    ``clip_grad_norm`` over the sharded state, ``param_groups`` usable by LR schedulers
    (Stoke-DDP.py:300-301).
  * ``ShardedDataParallel(model, optimizer)``, ``.zero_grad()``, ``no_sync()`` (Fairscale-DDP.py:89,97).
Semantics reference: greedy partition of torch/distributed/optim/zero_redundancy_optimizer.py:680-700
(native ``greedy_partition``); owners update their parameters and the rest receive them (:758-810).

MI355X-first design (not Fairscale's per-rank broadcasts and per-parameter reduces):
  * ONE owner-contiguous flat buffer per (dtype, device) -- the native ``ZeroLayout``: every rank's owned
    parameters packed into one segment, segments padded to a common length.  The module parameters are
    views into it, so the post-step exchange is ONE all-gather of the owners' segments (world_size
    broadcasts before), and a rank's optimizer state / fp32 master / gradient shard is one contiguous
    slice.
  * ``broadcast_fp16``: the all-gather payload is a bf16 (fp16 on CPU) flat; the fused AdamW writes the
    owner's slice of it in its epilogue (no cast pass), receivers cast only the peers' slices back.
  * ``compute_dtype=torch.bfloat16``: the module itself runs on bf16 parameters (views of the bf16 flat)
    while each rank keeps fp32 masters for its OWN segment only; the fused AdamW updates the masters and
    writes the bf16 parameters in its epilogue, the all-gather then moves bf16.  No per-forward fp32->bf16
    weight casts and no bf16->fp32 gradient casts (the autocast "cast storm").
  * ``ShardedDataParallel`` (ZeRO-2, ``reduce_mode="reduce"``): a rank keeps a persistent gradient buffer
    for its own segment only; gradients of other owners' parameters are produced by autograd, packed per
    bucket (a window of one owner's segment; the wire-dtype cast fused into the same kernel) into a slot of
    a small ring of persistent staging buffers (no allocation per bucket), reduced (AVG) to the owner
    asynchronously from the grad hooks, and freed -- per-rank gradient memory is ~1/world of the model.
    ``reduce_mode="all_reduce"`` is the ZeRO-1 gradient path (DDP + OSS): full gradients, bucketed
    all-reduces over the same flat.
  * Optimizer-state consolidation gathers flat per-key state slices (tensors, no pickled state), plus one
    tiny all-reduce of the per-parameter step counts.
"""
from __future__ import annotations

import weakref
from contextlib import contextmanager

import torch
import torch.nn as nn
from torch.optim import Optimizer

from ..optim.clip import clip_grad_norm_
from ..utils import profiling as prof
from ..utils.native import require_runtime
from ._readiness import NullReadiness, Readiness
from .comm import Comm, default_comm
from .ddp import sync_buffers

ALIGN = 16


class _Bank:
    """Parameters of one (storage dtype, device): owner-contiguous flat + views + (optional) payload/masters."""

    def __init__(self, params, idxs, owners, world, rank, flat_dtype, device):
        self.params, self.idxs, self.owners = params, idxs, owners
        self.world, self.rank, self.device, self.dtype = world, rank, device, flat_dtype
        lay = self.layout(1 << 62)
        self.seg, self.total = int(lay.seg), int(lay.total)
        self.offsets = list(lay.offsets)
        self.flat = torch.zeros(self.total, dtype=flat_dtype, device=device)
        self.lp = None          # broadcast_fp16 payload
        self.master_flat = None  # compute-dtype mode: fp32 masters of this rank's segment
        self.masters = {}       # local param index -> fp32 master Parameter

    def layout(self, bucket_elems):
        """Native owner-contiguous layout; offsets do not depend on the bucket cap."""
        return require_runtime().ZeroLayout([p.numel() for p in self.params], self.owners, self.world, ALIGN,
                                            max(1, int(bucket_elems)))

    def own(self, t):
        return t[self.rank * self.seg:(self.rank + 1) * self.seg]

    def view(self, t, li):
        p = self.params[li]
        o = self.offsets[li]
        return t[o:o + p.numel()].view(p.shape)


class OSS(Optimizer):
    """Optimizer state sharding wrapper (ZeRO-1)."""

    def __init__(self, params, optim=None, comm: Comm | None = None, broadcast_fp16: bool = False, group=None,
                 compute_dtype: torch.dtype | None = None, **defaults):
        from ..optim import FusedAdamW

        self.comm = comm or (Comm(group) if group is not None else default_comm())
        self.optim_cls = optim or FusedAdamW
        self.broadcast_fp16 = broadcast_fp16
        self.compute_dtype = compute_dtype
        if compute_dtype is not None and not issubclass(self.optim_cls, FusedAdamW):
            # the fp32 masters read their gradient through _pdt_grad_src, which only FusedAdamW follows: a
            # torch optimizer would see master.grad None and silently never update anything
            raise ValueError("OSS(compute_dtype=...) needs optim=FusedAdamW (the fp32 masters' gradients are "
                             f"the compute-dtype module gradients), got {self.optim_cls.__name__}")
        super().__init__(params, defaults)
        world, rank = self.comm.world_size, self.comm.rank
        self._all_params = [p for g in self.param_groups for p in g["params"]]
        self._index = {id(p): i for i, p in enumerate(self._all_params)}
        self.owner = list(require_runtime().greedy_partition([p.numel() for p in self._all_params], world))
        self._owner_of = {id(p): r for p, r in zip(self._all_params, self.owner)}
        if self.comm.world_size > 1:      # identical start everywhere (rank 0 wins), before the re-layout
            self.comm.broadcast_coalesced([p.data for p in self._all_params])
        self._build_banks()
        # local optimizer over what this rank owns: the module parameters themselves, or (compute-dtype
        # mode) the fp32 masters shadowing them -- one local group per wrapper group
        local_groups = []
        for g in self.param_groups:
            lg = {k: v for k, v in g.items() if k != "params"}
            lg["params"] = [self._opt_param(p) for p in g["params"] if self._owner_of[id(p)] == rank]
            local_groups.append(lg)
        self._local_group_idx = [i for i, g in enumerate(local_groups) if g["params"]]
        nonempty = [g for g in local_groups if g["params"]]
        self.optim = self.optim_cls(nonempty, **defaults) if nonempty else None
        self._fused = isinstance(self.optim, FusedAdamW)
        self._state_cache = None

    # ---------------------------------------------------------------- layout
    def _build_banks(self):
        world, rank = self.comm.world_size, self.comm.rank
        by = {}
        for i, p in enumerate(self._all_params):
            dt = self.compute_dtype if (self.compute_dtype is not None and p.dtype == torch.float32) else p.dtype
            by.setdefault((dt, p.device), []).append(i)
        self._banks = []
        self._bank_of = {}
        for (dt, dev), idxs in by.items():
            ps = [self._all_params[i] for i in idxs]
            bank = _Bank(ps, idxs, [self.owner[i] for i in idxs], world, rank, dt, dev)
            mixed = dt != ps[0].dtype
            if mixed:
                bank.master_flat = torch.zeros(bank.seg, dtype=torch.float32, device=dev)
            with torch.no_grad():
                for li, p in enumerate(ps):
                    v = bank.view(bank.flat, li)
                    v.copy_(p.detach())
                    if mixed and bank.owners[li] == rank:
                        o = bank.offsets[li] - rank * bank.seg
                        mv = bank.master_flat[o:o + p.numel()].view(p.shape)
                        mv.copy_(p.detach())                 # exact fp32 values, not the rounded bf16 copy
                        m = nn.Parameter(mv)
                        m._pdt_grad_src = p                  # the optimizer reads the module parameter's grad
                        m._pdt_lp_shard = v                  # ... and writes its bf16 value in the epilogue
                        bank.masters[li] = m
                    p.data = v
            if self.broadcast_fp16 and not mixed and dt == torch.float32:
                bank.lp = torch.zeros(bank.total, dtype=torch.bfloat16 if dev.type == "cuda" else torch.float16,
                                      device=dev)
                for li, p in enumerate(ps):
                    if bank.owners[li] == rank:
                        p._pdt_lp_shard = bank.view(bank.lp, li)   # AdamW epilogue writes the payload
                # The epilogue only rewrites what it steps: a frozen / gradient-less parameter or a skipped
                # (found_inf) step leaves the owner's slice as is, so it must hold the current values from
                # the start -- never zeros that the all-gather would spread to every peer.
                with torch.no_grad():
                    bank.own(bank.lp).copy_(bank.own(bank.flat))
            for li, i in enumerate(idxs):
                self._bank_of[i] = (bank, li)
            self._banks.append(bank)

    def _opt_param(self, p):
        bank, li = self._bank_of[self._index[id(p)]]
        return bank.masters.get(li, p)

    def owned_params(self):
        """The tensors this rank's optimizer steps (fp32 masters in compute-dtype mode)."""
        r = self.comm.rank
        return [self._opt_param(p) for p in self._all_params if self._owner_of[id(p)] == r]

    def banks(self):
        return self._banks

    # ---------------------------------------------------------------- step
    def _sync_hparams(self):
        if self.optim is None:
            return
        for li, gi in enumerate(self._local_group_idx):
            for k, v in self.param_groups[gi].items():
                if k != "params":
                    self.optim.param_groups[li][k] = v

    @torch.no_grad()
    def step(self, closure=None, **kw):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._sync_hparams()
        if self.optim is not None:
            if self._fused:
                self.optim.step(**kw)
            else:
                found = kw.get("found_inf")
                if found is None or int(found.reshape(-1)[0]) == 0:
                    self.optim.step()
        self._exchange()
        return loss

    def _exchange(self):
        """Owners -> everyone: ONE all-gather per bank of the owners' (payload) segments."""
        with prof.range("oss.all_gather"):
            self._exchange_banks()

    def _exchange_banks(self):
        for bank in self._banks:
            if bank.master_flat is not None and not self._fused:
                for li, m in bank.masters.items():          # non-fused optimizer: write the compute copy here
                    bank.view(bank.flat, li).copy_(m.detach())
            src = bank.lp if bank.lp is not None else bank.flat
            if bank.lp is not None and not self._fused:
                bank.own(bank.lp).copy_(bank.own(bank.flat))
            if self.comm.world_size == 1:
                continue
            self.comm.all_gather(src, bank.own(src))
            if bank.lp is not None:        # receivers: fp32 params from the compressed payload (peers only)
                r, s = self.comm.rank, bank.seg
                if r > 0:
                    bank.flat[:r * s].copy_(bank.lp[:r * s])
                if r + 1 < self.comm.world_size:
                    bank.flat[(r + 1) * s:].copy_(bank.lp[(r + 1) * s:])

    def zero_grad(self, set_to_none: bool = True):
        for p in self._all_params:
            if p.grad is not None:
                if getattr(p, "_pdt_keep_grad_view", False):
                    p.grad.zero_()
                elif set_to_none:
                    p.grad = None
                else:
                    p.grad.zero_()

    def clip_grad_norm(self, max_norm: float, norm_type: float = 2.0):
        """Global norm over the owned gradients (each parameter counted once): one 1-float all-reduce."""
        norm, _, _ = clip_grad_norm_(self.owned_params(), max_norm, norm_type=norm_type, comm=self.comm,
                                     sharded=True)
        return norm

    # ---------------------------------------------------------------- full parameters
    @torch.no_grad()
    def full_parameters(self):
        """{module parameter: full fp32 value} on every rank (compute-dtype mode gathers the fp32 masters;
        otherwise the module parameters already hold full values)."""
        out = {}
        for bank in self._banks:
            if bank.master_flat is None:
                for p in bank.params:
                    out[p] = p.detach()
                continue
            full = torch.empty(bank.total, dtype=torch.float32, device=bank.device)
            self.comm.all_gather(full, bank.master_flat)
            for li, p in enumerate(bank.params):
                out[p] = bank.view(full, li).clone()
        return out

    @torch.no_grad()
    def load_full_parameters(self, values):
        """Set module parameters (and this rank's masters) from full fp32 values {param: tensor}."""
        for bank in self._banks:
            for li, p in enumerate(bank.params):
                if p not in values:
                    continue
                v = values[p].to(device=bank.device)
                bank.view(bank.flat, li).copy_(v)
                if bank.lp is not None:               # keep the all-gather payload in step with the values
                    bank.view(bank.lp, li).copy_(v)
                if li in bank.masters:
                    bank.masters[li].copy_(v)
                    bank.masters[li]._pdt_lp_version = bank.masters[li]._version

    # ---------------------------------------------------------------- checkpointing
    def _state_keys(self):
        keys = set()
        if self.optim is not None:
            for st in self.optim.state.values():
                keys.update(k for k, v in st.items() if torch.is_tensor(v) and v.dim() > 0)
        allk = self.comm.all_gather_object(sorted(keys))     # key NAMES only -- the state moves as tensors
        return sorted(set(k for ks in allk for k in ks))

    @torch.no_grad()
    def consolidate_state_dict(self, recipient_rank: int = 0):
        """Gather the optimizer state on ``recipient_rank`` (Stoke/Fairscale save path):
        per bank and state key, every owner's flat segment moves in one all-gather; step counts in one
        tiny all-reduce."""
        rank, world = self.comm.rank, self.comm.world_size
        keys = self._state_keys() if world > 1 else sorted(
            {k for st in (self.optim.state.values() if self.optim else []) for k, v in st.items()
             if torch.is_tensor(v) and v.dim() > 0})
        dev = self._banks[0].device if self._banks else torch.device("cpu")
        n = len(self._all_params)
        steps = torch.zeros(n, dtype=torch.float64, device=dev)
        has = torch.zeros(n, dtype=torch.float64, device=dev)
        full = {}
        for bank in self._banks:
            for k in keys:
                seg = torch.zeros(bank.seg, dtype=torch.float32, device=bank.device)
                for li, p in enumerate(bank.params):
                    if bank.owners[li] != rank:
                        continue
                    st = self.optim.state.get(self._opt_param(p), {}) if self.optim is not None else {}
                    if k in st:
                        o = bank.offsets[li] - rank * bank.seg
                        seg[o:o + p.numel()].copy_(st[k].reshape(-1))
                g = torch.empty(bank.total, dtype=torch.float32, device=bank.device)
                self.comm.all_gather(g, seg)
                full[(id(bank), k)] = g
            for li, p in enumerate(bank.params):
                if bank.owners[li] == rank and self.optim is not None:
                    st = self.optim.state.get(self._opt_param(p))
                    if st and "step" in st:
                        steps[bank.idxs[li]] = float(st["step"])
                        has[bank.idxs[li]] = 1.0
        self.comm.all_reduce(steps, "sum")
        self.comm.all_reduce(has, "sum")
        if rank != recipient_rank:
            self._state_cache = None
            return
        steps, has = steps.cpu(), has.cpu()
        state = {}
        for bank in self._banks:
            for li, p in enumerate(bank.params):
                gi = bank.idxs[li]
                if not has[gi]:
                    continue
                ent = {"step": torch.tensor(float(steps[gi]))}
                for k in keys:
                    ent[k] = bank.view(full[(id(bank), k)], li).detach().to("cpu", copy=True).view(p.shape)
                state[gi] = ent
        self._state_cache = state

    def state_dict(self):
        """torch layout: {state: {global_idx: {...}}, param_groups: [...]} (call consolidate first)."""
        if self._state_cache is None:
            if self.comm.world_size == 1:
                self.consolidate_state_dict()
            else:
                raise RuntimeError("OSS.state_dict(): call consolidate_state_dict(recipient_rank) first "
                                   "(only the recipient holds the full state)")
        groups = []
        for g in self.param_groups:
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = [self._index[id(p)] for p in g["params"]]
            groups.append(d)
        return {"state": dict(self._state_cache), "param_groups": groups}

    def load_state_dict(self, sd):
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            for k, v in sg.items():
                if k != "params":
                    g[k] = v
        if self.optim is None:
            return
        local = {"state": {}, "param_groups": []}
        lidx = 0
        for li, gi in enumerate(self._local_group_idx):
            lg = {k: v for k, v in self.optim.param_groups[li].items() if k != "params"}
            lg.update({k: v for k, v in self.param_groups[gi].items() if k != "params"})
            ps = self.optim.param_groups[li]["params"]
            lg["params"] = list(range(lidx, lidx + len(ps)))
            owned = [p for p in self.param_groups[gi]["params"] if self._owner_of[id(p)] == self.comm.rank]
            for j, p in enumerate(owned):
                gidx = self._index[id(p)]
                st = sd["state"].get(gidx, sd["state"].get(str(gidx)))
                if st is not None:
                    local["state"][lidx + j] = st
            lidx += len(ps)
            local["param_groups"].append(lg)
        self.optim.load_state_dict(local)


class _Window:
    """ZeRO-2 reduce-scatter bucket: the window [lo, lo + n) of EVERY owner's segment of one bank.  Packed
    owner-major ([owner 0's window | owner 1's | ...]) into one staging slot, a single reduce-scatter (AVG)
    leaves owner r's reduced window in rank r's persistent gradient segment."""

    __slots__ = ("bank", "lo", "n", "members", "drop")

    def __init__(self, bank, lo, n):
        self.bank, self.lo, self.n = bank, lo, n
        self.members = []   # (slot offset, local param idx, param-local start a, end b), sorted by slot offset
        self.drop = []      # non-owned local param idx whose LAST window this is (gradient freed after packing)


def _merge_in_order(seqs):
    """Merge sequences of (key, ...) tuples by key, keeping each sequence's own order (ties: earlier sequence)."""
    heads = [0] * len(seqs)
    out = []
    while True:
        best = None
        for i, sq in enumerate(seqs):
            if heads[i] < len(sq) and (best is None or sq[heads[i]][0] < seqs[best][heads[best]][0]):
                best = i
        if best is None:
            return out
        out.append(seqs[best][heads[best]])
        heads[best] += 1


class ShardedDataParallel(nn.Module):
    """ZeRO-2: gradients are reduce-scattered (averaged) onto the ranks that own their optimizer shard, and
    non-owners drop them.  ``reduce_mode="all_reduce"``: ZeRO-1 (full gradients all-reduced, DDP + OSS).

    Fairscale's ShardedDDP reduces every parameter to its owner (``dist.reduce`` per parameter or small-param
    bucket).  On a full xGMI mesh a reduce into ONE destination loads that destination's inbound
    links only, and W owners mean W collectives per gradient region.  Here a bucket is the same window of every
    owner's segment (``_Window``): one reduce-scatter per window moves every rank's share at once over all
    links, and each rank's reduced gradient lands directly in its persistent segment.  Readiness: a parameter
    belongs to the FIRST window it touches and windows are released strictly in order, so a window is launched
    only when every parameter intersecting it has its gradient (a parameter spanning windows keeps its
    gradient until the last of them is packed)."""

    def __init__(self, module: nn.Module, sharded_optimizer: OSS, comm: Comm | None = None,
                 broadcast_buffers: bool = True, sync_models_at_startup: bool = True,
                 reduce_buffer_size: int = 2 ** 23, reduce_fp16: bool = False, reduce_mode: str = "reduce",
                 buffer_sync: str = "changed", staging_slots: int = 4, **_ignored):
        super().__init__()
        if staging_slots < 1:
            raise ValueError(f"staging_slots must be >= 1, got {staging_slots}")
        self.STAGING_SLOTS = staging_slots   # windows in flight at once (ring of pack buffers)
        if reduce_mode not in ("reduce", "all_reduce"):
            raise ValueError(f"reduce_mode must be 'reduce' or 'all_reduce', got {reduce_mode}")
        self.module = module
        self.optimizer = sharded_optimizer
        self.comm = comm or sharded_optimizer.comm
        self.broadcast_buffers = broadcast_buffers
        self.buffer_sync = buffer_sync
        self.reduce_fp16 = reduce_fp16
        self.reduce_mode = reduce_mode
        self._no_sync = False
        self._callback_queued = False
        self._handles = []
        if sync_models_at_startup and self.comm.world_size > 1:
            # parameters were already synced by OSS (before its re-layout); buffers here
            bufs = list(module.buffers())
            if bufs:
                self.comm.broadcast_coalesced(bufs)
        self.params = sharded_optimizer._all_params
        self._pad = {}
        self._rings = {}            # (wire dtype, device) -> staging ring (_slot)
        # gradient storage: own segment only (ZeRO-2) or the full flat (ZeRO-1)
        self._grad = {}             # bank id -> gradient flat
        self._buckets = []          # all_reduce: (bank, owner, start, numel, [local idx]); reduce: _Window
        readiness = []              # global parameter indices per bucket, in release order
        for bank in sharded_optimizer.banks():
            n = bank.seg if reduce_mode == "reduce" else bank.total
            self._grad[id(bank)] = torch.zeros(n, dtype=bank.dtype, device=bank.device)
        if reduce_mode == "reduce":
            # every bank's windows in release order, merged across banks by when backward completes them -- the
            # smallest parameter index a window touches arrives last (backward runs in reverse registration
            # order) -- so with several banks (dtypes / devices) bank 1's first window is not queued behind bank
            # 0's last one; each bank keeps its own order (a k-way merge, never a sort)
            seqs = []
            for bank in sharded_optimizer.banks():
                wins, first = self._plan_windows(bank, reduce_buffer_size)
                seqs.append([(-min((bank.idxs[m[1]] for m in w.members), default=0), w,
                              [bank.idxs[li] for li in first.get(k, [])]) for k, w in enumerate(wins)])
            for _key, w, ready in _merge_in_order(seqs):
                self._buckets.append(w)
                readiness.append(ready)
        else:
            tmp = []
            for bank in sharded_optimizer.banks():
                esz = torch.tensor([], dtype=bank.dtype).element_size()
                for b in bank.layout(reduce_buffer_size // esz).buckets:
                    tmp.append((bank, int(b.owner), int(b.start), int(b.numel), list(b.params)))
            tmp.sort(key=lambda b: -min(b[0].idxs[li] for li in b[4]))
            self._buckets = tmp
            readiness = [[bank.idxs[li] for li in lidx] for bank, _o, _s, _n, lidx in tmp]
        self._attach()
        self._bank_li = {}
        for bank in sharded_optimizer.banks():
            for li, gi in enumerate(bank.idxs):
                self._bank_li[gi] = (bank, li)
        # bucket readiness on C++ AccumulateGrad post hooks (parallel/_readiness.py): Python runs once per ready
        # bucket; frozen parameters get no hook and their buckets are released at the end of backward
        self._readiness_plan = readiness
        self._ready = None
        self._arm_readiness(native=True)

    def _arm_readiness(self, native: bool):
        if self._ready is not None:
            self._ready.remove()
        ref = weakref.ref(self)
        self._ready = NullReadiness() if self.comm.world_size == 1 else \
            Readiness(self.params, self._readiness_plan, on_first=lambda: ref()._queue_finalize(),
                      on_ready=lambda b: ref()._launch(b), native=native)
        self._ready.set_enabled(self.comm.world_size > 1 and not self._no_sync)

    def prepare_capture(self):
        """Per-parameter Python readiness hooks before a HIP-graph capture (Trainer.graph at world > 1; see
        DistributedDataParallel.prepare_capture)."""
        if getattr(self._ready, "kind", "none") == "native":
            self._arm_readiness(native=False)

    def _wire_dtype(self, bank):
        if self.reduce_fp16 and bank.dtype == torch.float32:
            return torch.bfloat16 if bank.device.type == "cuda" else torch.float16
        return bank.dtype

    def _plan_windows(self, bank, reduce_buffer_size):
        """Windows over the segment coordinate.  Window length: the whole bucket (every owner's window) is
        about ``reduce_buffer_size`` bytes on the wire, in 16-element granules.  Segments list their owner's
        parameters in reverse registration order (native ZeroLayout), so window 0 holds each owner's
        last-layer gradients -- the first ones backward produces."""
        W = bank.world
        esz = torch.tensor([], dtype=self._wire_dtype(bank)).element_size()
        w = max(ALIGN, (reduce_buffer_size // (esz * W)) // ALIGN * ALIGN)
        nwin = max(1, -(-bank.seg // w))
        wins = [_Window(bank, k * w, min(w, bank.seg - k * w)) for k in range(nwin)]
        first, last = {}, {}
        for li, p in enumerate(bank.params):
            r = bank.owners[li]
            s0 = bank.offsets[li] - r * bank.seg          # segment coordinate of the parameter's first element
            s1 = s0 + p.numel()
            k0, k1 = s0 // w, (s1 - 1) // w
            for k in range(k0, k1 + 1):
                win = wins[k]
                a, b = max(s0, win.lo), min(s1, win.lo + win.n)
                win.members.append((r * win.n + (a - win.lo), li, a - s0, b - s0))
            first.setdefault(k0, []).append(li)
            last[li] = k1
        for win in wins:
            win.members.sort()
        for li, k in last.items():
            if bank.owners[li] != bank.rank:
                wins[k].drop.append(li)
        return wins, first

    # ------------------------------------------------------------------ gradient storage
    def _grad_view(self, bank, li):
        p = bank.params[li]
        o = bank.offsets[li] - (bank.rank * bank.seg if self.reduce_mode == "reduce" else 0)
        return self._grad[id(bank)][o:o + p.numel()].view(p.shape)

    def _persistent(self, bank, li) -> bool:
        return self.reduce_mode == "all_reduce" or bank.owners[li] == bank.rank

    def _attach(self):
        """Persistent gradients are views of the flat (autograd accumulates in place, no copy-in)."""
        for bank in self.optimizer.banks():
            for li, p in enumerate(bank.params):
                if self._persistent(bank, li):
                    v = self._grad_view(bank, li)
                    if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                        p.grad = v
                    p._pdt_keep_grad_view = True

    def grad_bytes(self) -> int:
        """Gradient bytes this rank currently holds (persistent flat + any live non-owned .grad)."""
        n = sum(t.numel() * t.element_size() for t in self._grad.values())
        for bank in self.optimizer.banks():
            for li, p in enumerate(bank.params):
                if not self._persistent(bank, li) and p.grad is not None:
                    n += p.grad.numel() * p.grad.element_size()
        return n

    def staging_bytes(self) -> int:
        """Bytes of the persistent pack rings (STAGING_SLOTS x world x the longest window, per wire dtype)."""
        return sum(t.numel() * t.element_size() for r in self._rings.values() for t in r["bufs"])

    def collectives_per_backward(self) -> int:
        """Collectives one synchronised backward issues (one per bucket)."""
        return len(self._buckets) if self.comm.world_size > 1 else 0

    # ------------------------------------------------------------------ hooks / reduction
    def _zeros(self, n, dtype, device):
        z = self._pad.get((n, dtype, device))
        if z is None:
            z = self._pad[(n, dtype, device)] = torch.zeros(n, dtype=dtype, device=device)
        return z

    def _slot(self, bank, n, dtype):
        """A staging slot of ``n`` elements from the (dtype, device) ring of STAGING_SLOTS persistent buffers,
        each world x the longest window.  A slot is reused only after the collective that last read it was
        waited for (stream-ordered on device, so no host sync): ZeRO-2 keeps its memory bound -- the ring is a
        few buckets, not the (W-1)/W of the gradients a buffer per bucket would pin -- while the pack
        allocates nothing."""
        key = (dtype, bank.device)
        ring = self._rings.get(key)
        if ring is None:
            size = max(w.bank.world * w.n for w in self._buckets if w.bank.device == bank.device)
            ring = self._rings[key] = {"bufs": [torch.empty(size, dtype=dtype, device=bank.device)
                                                for _ in range(self.STAGING_SLOTS)],
                                       "busy": [None] * self.STAGING_SLOTS, "next": 0}
        i = ring["next"]
        ring["next"] = (i + 1) % self.STAGING_SLOTS
        if ring["busy"][i] is not None:
            ring["busy"][i].wait()
            ring["busy"][i] = None
        return ring, i, ring["bufs"][i][:n]

    def _pack_window(self, win, dtype):
        """Every owner's window of this bucket, owner-major, into one ring slot: the rank's own window is one
        contiguous slice of its persistent segment, peers' windows are (pieces of) the autograd gradients of
        their parameters (gaps = zeros); the wire-dtype cast is fused into the single ``cat``."""
        bank, n, W, r = win.bank, win.n, win.bank.world, win.bank.rank
        own = self._grad[id(bank)][win.lo:win.lo + n]
        parts = [(r * n, own)]
        for off, li, a, b in win.members:
            if bank.owners[li] != r:
                g = bank.params[li].grad
                parts.append((off, g.reshape(-1)[a:b] if g is not None else self._zeros(b - a, bank.dtype,
                                                                                        bank.device)))
        parts.sort(key=lambda x: x[0])
        pieces, cur = [], 0
        for off, t in parts:
            if off > cur:
                pieces.append(self._zeros(off - cur, bank.dtype, bank.device))
            pieces.append(t)
            cur = off + t.numel()
        if W * n > cur:
            pieces.append(self._zeros(W * n - cur, bank.dtype, bank.device))
        ring, i, slot = self._slot(bank, W * n, dtype)
        torch.cat(pieces, out=slot)
        for li in win.drop:                             # ZeRO-2: a non-owner drops the gradient once packed
            bank.params[li].grad = None
        return ring, i, slot, own

    def _launch(self, b):
        with prof.range(f"sddp.{self.reduce_mode}[bucket {b}]"):
            self._launch_bucket(b)

    def _launch_bucket(self, b):
        if self.reduce_mode == "all_reduce":
            bank, _owner, start, n, _lidx = self._buckets[b]
            wire = self._wire_dtype(bank)
            buf = self._grad[id(bank)][start:start + n]
            payload = buf if wire == buf.dtype else buf.to(wire)
            h = self.comm.all_reduce(payload, "avg", async_op=True)
            self._handles.append((h, buf if payload is not buf else None, payload))
            return
        win = self._buckets[b]
        wire = self._wire_dtype(win.bank)
        ring, i, slot, own = self._pack_window(win, wire)
        out = own if wire == own.dtype else torch.empty(win.n, dtype=wire, device=own.device)
        h = self.comm.reduce_scatter(out, slot, "avg", async_op=True)
        ring["busy"][i] = h
        self._handles.append((h, own if out is not own else None, out))

    def _queue_finalize(self):
        if self._callback_queued:
            return
        self._callback_queued = True
        torch.autograd.Variable._execution_engine.queue_callback(self._finalize)

    def _finalize(self):
        self._callback_queued = False
        self.comm.check_errors()
        for b in self._ready.flush():       # buckets with parameters that got no gradient
            self._launch(b)
        for h, dst, payload in self._handles:
            h.wait()
            if dst is not None:
                dst.copy_(payload)
        self._handles.clear()
        for ring in self._rings.values():
            ring["busy"] = [None] * self.STAGING_SLOTS
        self._ready.reset()

    # ------------------------------------------------------------------ forward
    def forward(self, *args, **kwargs):
        self._attach()        # a torch-style zero_grad(set_to_none) may have dropped the views
        if self.broadcast_buffers and self.comm.world_size > 1 and self.module.training:
            sync_buffers(self.module, self.comm, self, self.buffer_sync)
        return self.module(*args, **kwargs)

    def zero_grad(self, set_to_none: bool = False):
        for g in self._grad.values():
            g.zero_()
        for bank in self.optimizer.banks():
            for li, p in enumerate(bank.params):
                if not self._persistent(bank, li):
                    p.grad = None

    @contextmanager
    def no_sync(self):
        old = self._no_sync
        self._no_sync = True
        self._ready.set_enabled(False)
        try:
            yield
        finally:
            self._no_sync = old
            self._ready.set_enabled(not old and self.comm.world_size > 1)

    # ------------------------------------------------------------------ checkpoint helpers
    def full_state_dict(self):
        """Module state dict with full fp32 parameter values (no 'module.' prefix)."""
        sd = self.module.state_dict()
        name_of = {id(p): n for n, p in self.module.named_parameters()}
        for p, v in self.optimizer.full_parameters().items():
            if id(p) in name_of:
                sd[name_of[id(p)]] = v.to(torch.float32)
        return sd

    def load_full_state_dict(self, sd, strict=True):
        name_of = {id(p): n for n, p in self.module.named_parameters()}
        vals = {p: sd[name_of[id(p)]] for p in self.params if id(p) in name_of and name_of[id(p)] in sd}
        rest = {k: v for k, v in sd.items() if k not in set(name_of.values())}
        res = self.module.load_state_dict(rest, strict=False)
        self.optimizer.load_full_parameters(vals)
        if strict:
            missing = [n for n in name_of.values() if n not in sd] + list(res.missing_keys)
            missing = [k for k in missing if k not in sd]
            if missing or res.unexpected_keys:
                raise RuntimeError(f"load_full_state_dict: missing={missing} unexpected={res.unexpected_keys}")
        return res
