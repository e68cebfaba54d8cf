"""Fully-sharded data parallel (ZeRO-3 / ZeRO-2) flat-parameter engine over RCCL / xGMI.

Design (MI355X-first, not a port of torch FSDP):
  * Each wrapped block (by class) becomes a *unit*; its parameters are flattened by the native
    ``FlatLayout`` planner (16-element aligned, padded to a multiple of world_size) into
      - ``flat_param``: the fp32 MASTER shard (an nn.Parameter -- what the optimizer steps),
      - ``lp_shard``:   the bf16 compute copy of the shard (all-gather input, refreshed by the fused
                        AdamW epilogue, so no separate cast pass),
      - ``full``:       the bf16 gathered buffer; its storage is released after forward
                        (FULL_SHARD) and re-gathered before backward.
    The original parameters are replaced by views into ``full`` -- the outputs of ONE autograd node per unit
    (``_UnitViewsFn``) -- so module code and state_dict keys are unchanged.
  * Gradients land in ONE flat buffer per unit, allocated when the unit's backward starts: each parameter gets a
    slot in it (``ops.grad_slots``), the framework Linears write their weight gradients straight into their slots
    (the GEMM output), and whatever else produces a parameter gradient is copied / added in by the unit's node.
    No per-parameter gradient is concatenated (the ``split`` -> ``cat`` of the first design).
  * Forward: the unit's all-gather is issued asynchronously and the NEXT unit (recorded forward order)
    is prefetched, so RCCL all-gathers overlap the current block's GEMMs.  Backward: pre-backward
    hooks on the unit outputs re-gather and prefetch the previous unit.
  * The unit's gradient arrives as one flat bf16 tensor; it is reduce-scattered (AVG) asynchronously
    on c10d's RCCL stream while backward continues; the fp32 shard gradient is produced at the end of
    backward (``flat_param.grad``).  Gradient accumulation (``no_sync()`` micro-steps): ``accumulate="sharded"``
    (default) reduce-scatters every micro-step and accumulates the fp32 SHARD (gradient memory stays 1/world);
    ``accumulate="local"`` keeps an unsharded fp32 gradient per unit and communicates on the last micro-step
    only (torch FSDP's no_sync: fewer collectives, world x the gradient memory).
  * world_size == 1: ``full`` IS ``lp_shard`` and no collective is issued.
  * ``state_dict()`` returns the FULL, unflattened fp32 state dict under the original keys
    (FULL_STATE_DICT semantics), as the Stoke checkpoint envelope expects.

Semantics reference (not code): torch/distributed/fsdp/_flat_param.py:948,1091-1160,1362-1479 and
_runtime_utils.py:831-941 (pad/chunk, pre/post divide).  BASELINE.json configs 4-5.
"""
from __future__ import annotations

import enum
from contextlib import contextmanager
from dataclasses import dataclass

import torch
import torch.nn as nn

from ..ops import grad_slots
from ..utils import profiling as prof
from ..utils.native import require_runtime
from .comm import Comm, default_comm


class ShardingStrategy(enum.Enum):
    FULL_SHARD = "full_shard"        # ZeRO-3: params gathered just in time, freed after use
    SHARD_GRAD_OP = "shard_grad_op"  # ZeRO-2: params stay gathered between forward and backward


@dataclass
class MixedPrecision:
    param_dtype: torch.dtype = torch.bfloat16
    reduce_dtype: torch.dtype = torch.bfloat16


ALIGN = 16


class _Unit:
    SHARDED, GATHERING, GATHERED = 0, 1, 2

    def __init__(self, owner, name, module, params, comm: Comm, device, mp: MixedPrecision, reshard: bool):
        self.owner, self.name, self.module = owner, name, module
        self.comm, self.device, self.mp, self.reshard_after_forward = comm, device, mp, reshard
        self.params = params  # list of (submodule, attr_name, fqn, shape)
        rt = require_runtime()
        numels = [int(torch.Size(s).numel()) for (_, _, _, s) in params]
        ws, rank = comm.world_size, comm.rank
        self.layout = rt.FlatLayout(numels, ws, ALIGN)
        self.total, self.shard_numel = int(self.layout.total), int(self.layout.shard_numel)
        self.offsets = list(self.layout.offsets)
        self.numels = numels
        self.state = self.SHARDED
        self.handle = None
        self.pending = []          # (Handle, rs_out) waiting for finalize
        self.accum_full = None     # accumulate="local": fp32 full grad accumulated under no_sync
        self.accum_shard = None    # accumulate="sharded": fp32 reduced shard accumulated under no_sync
        self.pending_acc = []      # accumulate="sharded": (Handle, rs_out) of a no_sync micro-step
        self.in_backward = False
        self.bwd_hooked = False
        self.order_idx = -1
        self.grad_flat = None      # this backward's flat gradient (slots of ops.grad_slots), see begin_backward
        self.slot_keys = []
        self.written = []

    # -------------------------------------------------------------- construction
    def materialize(self, tensors):
        """Build the flat master shard from the original parameter tensors."""
        ws, rank = self.comm.world_size, self.comm.rank
        s0 = rank * self.shard_numel
        shard = torch.zeros(self.shard_numel, dtype=torch.float32, device=self.device)
        for (t, off, n) in zip(tensors, self.offsets, self.numels):
            a, b = max(off, s0), min(off + n, s0 + self.shard_numel)
            if a < b:
                shard[a - s0:b - s0].copy_(t.detach().reshape(-1)[a - off:b - off].to(torch.float32))
        self.flat_param = nn.Parameter(shard)
        self.flat_param._pdt_unit = self
        self.lp_shard = torch.empty(self.shard_numel, dtype=self.mp.param_dtype, device=self.device)
        self.flat_param._pdt_lp_shard = self.lp_shard
        self.refresh_lp(force=True)
        if ws == 1:
            self.full = self.lp_shard
            self.state = self.GATHERED
        else:
            self.full = torch.empty(self.total, dtype=self.mp.param_dtype, device=self.device)
            # The collective writes through a second tensor object that aliases the same storage but
            # has its OWN version counter: re-gathering in backward must not look like an in-place
            # modification of the views autograd saved in forward.
            self._comm_buf = torch.empty(0, dtype=self.mp.param_dtype, device=self.device)
            self._comm_buf.set_(self.full.untyped_storage(), 0, (self.total,))
            self._free_full()

    def refresh_lp(self, force=False):
        fp = self.flat_param
        if force or getattr(fp, "_pdt_lp_version", None) != fp._version:
            with torch.no_grad():
                self.lp_shard.copy_(fp.detach())
            fp._pdt_lp_version = fp._version

    # -------------------------------------------------------------- storage management
    def _free_full(self):
        if self.comm.world_size == 1:
            return
        st = self.full.untyped_storage()
        if st.size() != 0:
            st.resize_(0)
        self.state = self.SHARDED

    def _alloc_full(self):
        st = self.full.untyped_storage()
        nbytes = self.total * self.full.element_size()
        if st.size() != nbytes:
            st.resize_(nbytes)

    def gather(self):
        """Issue (async) the all-gather of this unit's compute params."""
        self.refresh_lp()
        if self.state != self.SHARDED:
            return
        self._alloc_full()
        with prof.range(f"fsdp.all_gather[{self.name or 'root'}]"):
            self.handle = self.comm.all_gather(self._comm_buf, self.lp_shard, async_op=True)
        self.state = self.GATHERING

    def wait(self):
        if self.state == self.SHARDED:
            self.gather()
        if self.state == self.GATHERING:
            self.handle.wait()
            self.handle = None
            self.state = self.GATHERED

    def reshard(self):
        if self.comm.world_size > 1 and self.state == self.GATHERED:
            self._free_full()

    def views_of(self, full_tensor):
        """The parameter views of a flat [total] tensor (one per unique parameter, in ``params`` order)."""
        return [full_tensor[off:off + n].view(shape) for (_m, _a, _f, shape), off, n in
                zip(self.params, self.offsets, self.numels)]

    def install_views(self, views):
        for (mod, attr, _fqn, _shape), v in zip(self.params, views):
            setattr(mod, attr, v)

    # -------------------------------------------------------------- gradients
    def begin_backward(self):
        """Allocate this backward's flat gradient and register one slot per parameter (ops.grad_slots), keyed by
        the gathered storage the saved parameter views point at (so call after the unit is gathered)."""
        if self.grad_flat is not None:
            return
        self.grad_flat = torch.empty(self.total, dtype=self.mp.param_dtype, device=self.device)
        self.written = [False] * len(self.params)
        full = self.full.view(-1)
        self.slot_keys = [grad_slots.register(v, d, self, i) for i, (v, d) in
                          enumerate(zip(self.views_of(full), self.views_of(self.grad_flat)))]

    def slot_written(self, i):
        self.written[i] = True

    def post_backward_views(self, grads):
        """Called once per backward by the unit's node with the gradients autograd carried for each parameter view
        (None where no consumer produced one, or where a framework op wrote its slot instead)."""
        if self.grad_flat is None:      # backward entered without the pre-backward hook (e.g. the root unit
            self.begin_backward()       # through a path that skipped the loss-side hook)
        flat = self.grad_flat
        grad_slots.release(self.slot_keys)
        cur = 0
        for i, (g, off, n) in enumerate(zip(grads, self.offsets, self.numels)):
            if off > cur:
                flat[cur:off].zero_()                   # alignment padding
            cur = off + n
            slot = flat[off:off + n]
            if g is None:
                if not self.written[i]:
                    slot.zero_()
            elif self.written[i]:
                slot.add_(g.reshape(-1))
            else:
                slot.copy_(g.reshape(-1))
        if self.total > cur:
            flat[cur:].zero_()
        self.grad_flat, self.slot_keys, self.written = None, [], []
        self.post_backward(flat)

    def post_backward(self, grad_full):
        """The unit's flat gradient (param dtype, length total) of one backward."""
        self.in_backward = False
        grad = grad_full.detach()
        owner = self.owner
        if owner._no_sync and owner.accumulate == "local":
            if self.accum_full is None:
                self.accum_full = grad.to(torch.float32)
            else:
                self.accum_full.add_(grad)
        else:
            if self.accum_full is not None:
                grad = (self.accum_full.add_(grad)).to(self.mp.reduce_dtype)
                self.accum_full = None
            elif grad.dtype != self.mp.reduce_dtype:
                grad = grad.to(self.mp.reduce_dtype)
            if self.comm.world_size == 1:
                out, h = grad, None
            else:
                out = torch.empty(self.shard_numel, dtype=self.mp.reduce_dtype, device=grad.device)
                with prof.range(f"fsdp.reduce_scatter[{self.name or 'root'}]"):
                    h = self.comm.reduce_scatter(out, grad, op="avg", async_op=True)
            if owner._no_sync:          # accumulate="sharded": fold the reduced shard into the fp32 accumulator
                self.pending_acc.append((h, out))
            else:
                self.pending.append((h, out))
        # params are not needed again until the next forward (which re-gathers the updated shard)
        self.reshard()

    def fold_accumulation(self):
        """accumulate="sharded": wait for this micro-step's reduce-scatters and add them to the fp32 shard."""
        for h, out in self.pending_acc:
            if h is not None:
                h.wait()
            if self.accum_shard is None:
                self.accum_shard = out.to(torch.float32) if out.dtype != torch.float32 else out.clone()
            else:
                self.accum_shard.add_(out)
        self.pending_acc = []

    def finalize(self):
        self.fold_accumulation()
        for h, out in self.pending:
            if h is not None:
                h.wait()
            fp = self.flat_param
            if self.accum_shard is not None:
                # the micro-steps' reduced shards (fp32) plus this one: an fp32 .grad for the optimizer
                out = self.accum_shard.add_(out)
                self.accum_shard = None
                if fp.grad is not None:
                    fp.grad.add_(out)
                else:
                    fp.grad = out
                fp._pdt_grad = None
            elif fp.grad is not None:
                fp.grad.add_(out)
            elif self.owner.keep_low_precision_grads and out.dtype != torch.float32:
                # the reduced bf16 shard gradient is handed to the fused optimizer as is (no fp32 cast
                # pass, half the optimizer's gradient read); overwritten every synced backward
                fp._pdt_grad = out
            else:
                fp.grad = out.to(torch.float32) if out.dtype != torch.float32 else out.clone()
        self.pending.clear()


class _UnitViewsFn(torch.autograd.Function):
    """One node per unit: forward hands out the parameter views of the gathered flat buffer, backward receives
    each parameter's gradient (None where a framework op wrote the unit's slot itself) and builds the unit's flat
    gradient (``_Unit.post_backward_views``)."""

    @staticmethod
    def forward(ctx, flat_param, unit):
        ctx.unit = unit
        ctx.set_materialize_grads(False)
        return tuple(unit.views_of(unit.full.view(-1)))

    @staticmethod
    def backward(ctx, *grads):
        ctx.unit.post_backward_views(grads)
        return None, None


class FullyShardedDataParallel(nn.Module):
    """FSDP wrapper.

    Args:
        module: model to shard (may live on CPU or GPU; shards are created on ``device``).
        wrap_classes: block classes that become separate units (default: ``module.block_class`` if
            defined); everything else goes into the root unit.
        sharding_strategy: FULL_SHARD (ZeRO-3, default) or SHARD_GRAD_OP (ZeRO-2).
        mixed_precision: compute/all-gather dtype and gradient reduce dtype (bf16 / bf16 default).
        comm: collective layer (default: the initialised default process group).
        forward_prefetch / backward_prefetch: overlap the next unit's all-gather with compute.
        keep_low_precision_grads: leave the reduced shard gradient in ``reduce_dtype`` as
            ``flat_param._pdt_grad`` (read by FusedAdamW / clip_grad_norm_) instead of materialising an
            fp32 ``.grad`` -- use with the framework's fused optimizer.
        accumulate: "sharded" (default) or "local" -- gradient accumulation under ``no_sync`` (module docstring).
    """

    def __init__(self, module: nn.Module, wrap_classes=None, sharding_strategy=ShardingStrategy.FULL_SHARD,
                 mixed_precision: MixedPrecision | None = None, comm: Comm | None = None, device=None,
                 forward_prefetch: bool = True, backward_prefetch: bool = True, sync_module_states: bool = True,
                 keep_low_precision_grads: bool = False, accumulate: str = "sharded"):
        super().__init__()
        if accumulate not in ("sharded", "local"):
            raise ValueError(f"accumulate must be 'sharded' or 'local', got {accumulate!r}")
        self.accumulate = accumulate
        self.keep_low_precision_grads = keep_low_precision_grads
        self.module = module
        self.comm = comm or default_comm()
        self.mp = mixed_precision or MixedPrecision()
        self.sharding_strategy = sharding_strategy
        self.forward_prefetch, self.backward_prefetch = forward_prefetch, backward_prefetch
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else \
                torch.device("cpu")
        self.device = torch.device(device)
        if wrap_classes is None:
            bc = getattr(module, "block_class", None)
            wrap_classes = (bc,) if bc is not None else ()
        self.wrap_classes = tuple(wrap_classes)
        self._no_sync = False
        self._fwd_order = []
        self._order_frozen = False
        self._callback_queued = False
        self._orig_keys = list(module.state_dict().keys())
        self._param_fqns = [n for n, _ in module.named_parameters()]

        if sync_module_states and self.comm.world_size > 1:
            # identical init on all ranks (rank 0 wins), like sync_module_states=True
            self.comm.broadcast_coalesced([p.data.to(self.device) if p.device != self.device else p.data
                                           for p in module.parameters()])

        # ---- build units (child blocks first, root gets the rest)
        claimed = set()
        self.units = []
        for name, sub in module.named_modules():
            if name and isinstance(sub, self.wrap_classes) and not any(name.startswith(c + ".") for c in claimed):
                claimed.add(name)
                self.units.append(self._make_unit(name, sub, prefix=name + "."))
        self.root_unit = self._make_unit("", module, prefix="", skip=claimed)
        if self.root_unit is not None:
            self.root_unit.reshard_after_forward = False  # used first in backward
        self._flat_params = nn.ParameterList([u.flat_param for u in self.all_units()])
        for u in self.units:
            u.module.register_forward_pre_hook(self._make_pre_forward(u))
            u.module.register_forward_hook(self._make_post_forward(u))
        module.to(self.device)  # buffers

    # -------------------------------------------------------------- construction helpers
    def _make_unit(self, name, sub, prefix, skip=()):
        params, tensors, seen = [], [], {}
        for mname, m in sub.named_modules():
            full_m = (prefix + mname) if mname else prefix.rstrip(".")
            if skip and any(full_m == s or full_m.startswith(s + ".") for s in skip):
                continue
            for pname, p in list(m._parameters.items()):
                if p is None:
                    continue
                fqn = (full_m + "." if full_m else "") + pname
                if id(p) in seen:   # tied parameter: alias to the first occurrence
                    params.append((m, pname, fqn, tuple(p.shape)))
                    tensors.append(None)
                    continue
                seen[id(p)] = len(params)
                params.append((m, pname, fqn, tuple(p.shape)))
                tensors.append(p)
        if not params:
            return None
        # tied params: keep only first occurrence in the flat buffer; others alias it
        uniq, ties, uniq_t = [], [], []
        first_index = {}
        for (m, pn, fqn, shape), t in zip(params, tensors):
            if t is None:
                ties.append((m, pn, fqn, shape))
            else:
                first_index[fqn] = len(uniq)
                uniq.append((m, pn, fqn, shape))
                uniq_t.append(t)
        unit = _Unit(self, name, sub, uniq, self.comm, self.device, self.mp,
                     self.sharding_strategy == ShardingStrategy.FULL_SHARD)
        unit.materialize(uniq_t)
        # tie resolution: (module, attr) -> index of the aliased param in uniq
        unit.ties = []
        for (m, pn, fqn, shape) in ties:
            src = next(i for i, (mm, pp, ff, ss) in enumerate(uniq) if getattr(mm, "_parameters").get(pp) is
                       getattr(m, "_parameters").get(pn))
            unit.ties.append((m, pn, fqn, src))
        for (m, pn, _f, _s) in uniq + [(a, b, c, None) for (a, b, c, _i) in unit.ties]:
            if pn in m._parameters:
                del m._parameters[pn]
        # start with views installed (no-grad) so attribute access works outside forward
        if unit.state == unit.GATHERED:
            self._install(unit, unit.views_of(unit.full.view(-1)))
        return unit

    def _install(self, unit, views):
        for v in views:
            v._pdt_fsdp_unit = unit       # framework ops route these through their own backward (ops.grad_slots)
        unit.install_views(views)
        for (m, pn, _fqn, src) in getattr(unit, "ties", []):
            sm, sattr = unit.params[src][0], unit.params[src][1]
            setattr(m, pn, getattr(sm, sattr))

    def all_units(self):
        return self.units + ([self.root_unit] if self.root_unit is not None else [])

    # -------------------------------------------------------------- hooks
    def _activate(self, unit):
        """Gather (wait) and install autograd-tracked views for one unit's forward."""
        unit.refresh_lp()
        unit.wait()
        if torch.is_grad_enabled():
            views = _UnitViewsFn.apply(unit.flat_param, unit)
        else:
            views = unit.views_of(unit.full.view(-1))
        self._install(unit, views)

    def _make_pre_forward(self, unit):
        def hook(_mod, _args):
            if not unit.in_backward and not self._order_frozen and unit not in self._fwd_order:
                unit.order_idx = len(self._fwd_order)
                self._fwd_order.append(unit)
            self._activate(unit)
            if self.forward_prefetch and self._order_frozen and not unit.in_backward:
                i = unit.order_idx + 1
                if i < len(self._fwd_order):
                    self._fwd_order[i].gather()
        return hook

    def _make_post_forward(self, unit):
        def hook(_mod, _args, output):
            if unit.in_backward:      # activation-checkpoint recompute inside backward: keep params
                return output
            if torch.is_grad_enabled():
                self._register_pre_backward(unit, output)
            if unit.reshard_after_forward:
                unit.reshard()
            return output
        return hook

    def _register_pre_backward(self, unit, output):
        tensors = [t for t in _flatten(output) if torch.is_tensor(t) and t.requires_grad]
        if not tensors:
            return
        fired = {"done": False}

        def pre_bwd(grad):
            if not fired["done"]:
                fired["done"] = True
                unit.in_backward = True
                unit.wait()
                unit.begin_backward()
                if self.backward_prefetch:
                    i = unit.order_idx - 1
                    if 0 <= i < len(self._fwd_order):
                        self._fwd_order[i].gather()
            return grad
        for t in tensors:
            t.register_hook(pre_bwd)

    def _queue_finalize(self):
        if self._callback_queued:
            return
        self._callback_queued = True

        def cb():
            self._callback_queued = False
            self._order_frozen = True
            self.comm.check_errors()
            if self._no_sync:
                for u in self.all_units():
                    u.fold_accumulation()
                return
            for u in self.all_units():
                u.finalize()
        torch.autograd.Variable._execution_engine.queue_callback(cb)

    # -------------------------------------------------------------- forward
    def forward(self, *args, **kwargs):
        root = self.root_unit
        if root is not None:
            self._activate(root)
        if self._order_frozen and self.forward_prefetch and self._fwd_order:
            self._fwd_order[0].gather()
        if torch.is_grad_enabled():
            # finalize hook is queued from the first backward node that runs (loss side)
            out = self.module(*args, **kwargs)
            for t in _flatten(out):
                if torch.is_tensor(t) and t.requires_grad:
                    t.register_hook(self._loss_side_hook)
                    break
            return out
        return self.module(*args, **kwargs)

    def _loss_side_hook(self, grad):
        self._queue_finalize()
        if self.root_unit is not None:        # the root's parameters (head, embeddings) get their slots first
            self.root_unit.begin_backward()
        return grad

    def accumulator_bytes(self) -> int:
        """Bytes of gradient-accumulation state held between no_sync micro-steps (fp32 full / shard buffers)."""
        return sum(t.numel() * t.element_size() for u in self.all_units()
                   for t in (u.accum_full, u.accum_shard) if t is not None)

    @contextmanager
    def no_sync(self):
        old = self._no_sync
        self._no_sync = True
        try:
            yield
        finally:
            self._no_sync = old

    # -------------------------------------------------------------- utilities
    def flat_parameters(self):
        return [u.flat_param for u in self.all_units()]

    def sync_lp_params(self):
        for u in self.all_units():
            u.refresh_lp()

    def clip_grad_norm_(self, max_norm: float, norm_type: float = 2.0):
        """Global grad norm over all shards (one 1-float all-reduce) and in-place clipping."""
        from ..optim.clip import clip_grad_norm_
        return clip_grad_norm_(self.flat_parameters(), max_norm, norm_type=norm_type, comm=self.comm,
                               sharded=True)

    # -------------------------------------------------------------- full state dict
    def _gather_full_fp32(self, unit, src=None):
        src = unit.flat_param.detach() if src is None else src
        full = torch.empty(unit.total, dtype=torch.float32, device=src.device)
        self.comm.all_gather(full, src.contiguous())
        return full

    def state_dict(self, *args, destination=None, prefix="", keep_vars=False, rank0_only: bool = False,
                   offload_to_cpu: bool = False):
        """FULL unflattened fp32 state dict under the original keys.

        Default: identical on every rank (nn.Module semantics).  ``rank0_only``: units are gathered one at a
        time and only rank 0 keeps the result (other ranks return {}); ``offload_to_cpu``: each unit's
        parameters go to host memory right after its gather, so the device holds at most ONE unit's full
        fp32 copy (Llama-3 8B: ~1 GB instead of ~32 GB per rank) -- what a checkpoint save uses."""
        keep = not rank0_only or self.comm.rank == 0
        sd = {}
        for u in self.all_units():
            full = self._gather_full_fp32(u)
            if keep:
                if offload_to_cpu:
                    full = full.cpu()
                for (m, pn, fqn, shape), off, n in zip(u.params, u.offsets, u.numels):
                    sd[fqn] = full[off:off + n].view(shape).clone()
                for (m, pn, fqn, src) in getattr(u, "ties", []):
                    sd[fqn] = sd[u.params[src][2]]
            del full
        if not keep:
            return {} if destination is None else destination
        for k, v in self.module.state_dict().items():   # buffers
            sd.setdefault(k, v.cpu() if offload_to_cpu else v)
        ordered = {}
        for k in self._orig_keys:
            if k in sd:
                ordered[prefix + k] = sd[k] if keep_vars else sd[k].detach()
        for k, v in sd.items():
            if prefix + k not in ordered:
                ordered[prefix + k] = v
        if destination is not None:
            destination.update(ordered)
            return destination
        return ordered

    def full_optim_state_dict(self, optimizer, rank0_only: bool = False, offload_to_cpu: bool = False):
        """Optimizer state in torch layout keyed by ORIGINAL parameter index (unflattened, fp32); same
        ``rank0_only`` / ``offload_to_cpu`` semantics as ``state_dict``."""
        return _full_optim_state(self, optimizer, rank0_only, offload_to_cpu)

    def load_full_optim_state_dict(self, optimizer, sd):
        _load_full_optim_state(self, optimizer, sd)

    def load_state_dict(self, state_dict, strict: bool = True):
        missing = []
        rank = self.comm.rank
        used = set()
        for u in self.all_units():
            s0 = rank * u.shard_numel
            shard = torch.zeros(u.shard_numel, dtype=torch.float32, device=self.device)
            for (m, pn, fqn, shape), off, n in zip(u.params, u.offsets, u.numels):
                if fqn not in state_dict:
                    missing.append(fqn)
                    continue
                used.add(fqn)
                t = state_dict[fqn].detach().reshape(-1)
                a, b = max(off, s0), min(off + n, s0 + u.shard_numel)
                if a < b:
                    shard[a - s0:b - s0].copy_(t[a - off:b - off].to(device=self.device, dtype=torch.float32))
            for (_m, _pn, fqn, _src) in getattr(u, "ties", []):
                used.add(fqn)
            with torch.no_grad():
                u.flat_param.copy_(shard)
            u.refresh_lp(force=True)
            if self.comm.world_size > 1 and u.state == u.GATHERED and u is self.root_unit:
                u._free_full()
        rest = {k: v for k, v in state_dict.items() if k not in used}
        res = self.module.load_state_dict(rest, strict=False)
        unexpected = [k for k in res.unexpected_keys]
        if strict and (missing or unexpected):
            raise RuntimeError(f"FSDP load_state_dict: missing={missing} unexpected={unexpected}")
        return res


def _full_optim_state(fsdp, optimizer, rank0_only=False, offload_to_cpu=False):
    idx_of = {f: i for i, f in enumerate(fsdp._param_fqns)}
    keep = not rank0_only or fsdp.comm.rank == 0
    state = {}
    flat_to_idx = {}
    for u in fsdp.all_units():
        idxs = [idx_of[fqn] for (_m, _pn, fqn, _s) in u.params if fqn in idx_of]
        flat_to_idx[id(u.flat_param)] = idxs
        st = optimizer.state.get(u.flat_param)
        if not st:
            continue
        full = {}
        for k, v in st.items():       # one state key of one unit on the device at a time
            if torch.is_tensor(v) and v.dim() == 1 and v.numel() == u.shard_numel:
                g = fsdp._gather_full_fp32(u, v.detach())
                if keep:
                    full[k] = g.cpu() if offload_to_cpu else g
                del g
        if not keep:
            continue
        for (m, pn, fqn, shape), off, n in zip(u.params, u.offsets, u.numels):
            if fqn not in idx_of:
                continue
            ent = {k: v[off:off + n].view(shape).clone() for k, v in full.items()}
            for k, v in st.items():
                if k not in ent:
                    ent[k] = v.clone() if torch.is_tensor(v) else v
            state[idx_of[fqn]] = ent
    if not keep:
        return None
    groups = []
    for g in optimizer.param_groups:
        d = {k: v for k, v in g.items() if k != "params"}
        d["params"] = sorted(i for p in g["params"] for i in flat_to_idx.get(id(p), []))
        groups.append(d)
    return {"state": state, "param_groups": groups}


def _load_full_optim_state(fsdp, optimizer, sd):
    idx_of = {f: i for i, f in enumerate(fsdp._param_fqns)}
    st_all = sd["state"]
    rank = fsdp.comm.rank
    if sd.get("param_groups"):
        hp = {k: v for k, v in sd["param_groups"][0].items() if k != "params"}
        for g in optimizer.param_groups:
            g.update(hp)
    for u in fsdp.all_units():
        s0 = rank * u.shard_numel
        keys, step = None, None
        for (_m, _pn, fqn, _s) in u.params:
            e = st_all.get(idx_of.get(fqn, -1), st_all.get(str(idx_of.get(fqn, -1))))
            if e is not None:
                keys = [k for k, v in e.items() if torch.is_tensor(v) and v.dim() > 0]
                step = e.get("step")
                break
        if keys is None:
            continue
        new = {}
        for k in keys:
            shard = torch.zeros(u.shard_numel, dtype=torch.float32, device=u.flat_param.device)
            for (_m, _pn, fqn, _shape), off, n in zip(u.params, u.offsets, u.numels):
                e = st_all.get(idx_of.get(fqn, -1), st_all.get(str(idx_of.get(fqn, -1))))
                if e is None:
                    continue
                t = e[k].reshape(-1)
                a, b = max(off, s0), min(off + n, s0 + u.shard_numel)
                if a < b:
                    shard[a - s0:b - s0].copy_(t[a - off:b - off].to(shard.device, torch.float32))
            new[k] = shard
        if step is not None:
            new["step"] = step.clone() if torch.is_tensor(step) else torch.tensor(float(step))
        optimizer.state[u.flat_param] = new


def _flatten(x):
    if torch.is_tensor(x):
        return [x]
    if isinstance(x, (list, tuple)):
        out = []
        for y in x:
            out.extend(_flatten(y))
        return out
    if isinstance(x, dict):
        out = []
        for y in x.values():
            out.extend(_flatten(y))
        return out
    return []
