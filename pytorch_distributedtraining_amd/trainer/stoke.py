"""The training facade: wrap an nn.Module, get a distributed training loop with mixed precision,
gradient accumulation / clipping, sharded optimizers and checkpointing -- the capability the reference
obtains from Stoke (Stoke-DDP.py:240-254 construction; :73-86,116-118,142-145,274-301 use).

Same method names and semantics as the reference exercises them:
    model(x) / loss(out, tgt) / backward(loss) / step() / detach_and_sync_loss(loss) /
    print_ema_loss(prepend_msg) / print_on_devices(msg) / model_access / optimizer / world_size / rank /
    DataLoader(dataset, sampler, ...) / save(path, name) -> (path, tag) / load(path, tag)
* ``loss()`` divides by grad_accum_steps in training mode; ``backward()`` runs under the engine's
  ``no_sync()`` on non-boundary micro-steps; ``step()`` acts only on accumulation boundaries:
  (unscale ->) clip -> optimizer step -> zero grads.  effective batch = per-device x accum x world.
* MI355X-first execution underneath: RCCL engines from ``parallel`` (bucketed DDP, ZeRO-1 OSS,
  ZeRO-2 ShardedDDP, FSDP), the fused AdamW and fused clip/unscale kernels (gradient multiplier and
  found_inf stay on device -- no host sync between backward and update), bf16 autocast by default,
  loss/EMA synchronisation only when printed.
"""
from __future__ import annotations

import contextlib
import os
import uuid

import torch
import torch.nn as nn

from ..data.loader import DeviceDataLoader
from ..ops import picks
from ..ops.fp8 import fp8_autocast
from ..optim import FusedAdamW, GradScaler, clip_grad_norm_
from ..optim._grads import grad_of
from ..parallel.comm import Comm
from ..utils import checkpoint as ckpt
from ..utils import profiling as prof
from ..utils.dist import init_distributed
from ..utils.fault import maybe_inject_fault
from ..utils.logging import RankLogger
from .configs import (AMPConfig, ClipGradConfig, ClipGradNormConfig, DDPConfig, DeepspeedConfig, DistributedOptions,
                      FairscaleFSDPConfig, FairscaleOSSConfig, FairscaleSDDPConfig, FP16Options, StokeOptimizer,
                      find_config)
from .status import TrainerStatus


def _val(x):
    return x.value if hasattr(x, "value") else x


class SyncedLoss:
    """A rank-local device scalar whose cross-rank mean is taken lazily (``Trainer.detach_and_sync_loss(loss,
    lazy=True)`` or ``Trainer(lazy_loss_sync=True)``).

    Linear arithmetic keeps it on the device and unsynchronised: ``+``/``-`` with another SyncedLoss or a number,
    ``*``/``/`` by a number (the mean over ranks commutes with these).  Reading it -- ``float()``, ``int()``,
    ``item()``, ``bool()``, formatting, comparisons, ``==`` -- runs ONE all-reduce (AVG) and one host read, then
    caches the value.  READING IS A COLLECTIVE: every rank must read the value at the same point (a read on one rank
    only, e.g. under ``if rank == 0``, waits forever for the others); ``float(x)`` on every rank first, then use the
    float.  Not hashable and not JSON-serialisable (log ``float(x)``).  A number added to it is treated as already
    rank-uniform (e.g. the ``0.0`` a running sum starts from)."""

    __hash__ = None

    __slots__ = ("t", "comm", "_value")

    def __init__(self, t, comm):
        self.t, self.comm, self._value = t, comm, None

    # -- lazy linear arithmetic ------------------------------------------------------------------------
    def _other(self, o):
        if isinstance(o, SyncedLoss):
            return o.t
        if isinstance(o, (int, float)):
            return float(o)
        return NotImplemented

    def __add__(self, o):
        v = self._other(o)
        return NotImplemented if v is NotImplemented else SyncedLoss(self.t + v, self.comm)

    __radd__ = __add__

    def __sub__(self, o):
        v = self._other(o)
        return NotImplemented if v is NotImplemented else SyncedLoss(self.t - v, self.comm)

    def __rsub__(self, o):
        v = self._other(o)
        return NotImplemented if v is NotImplemented else SyncedLoss(v - self.t, self.comm)

    def __mul__(self, o):
        if isinstance(o, (int, float)):
            return SyncedLoss(self.t * float(o), self.comm)
        return NotImplemented

    __rmul__ = __mul__

    def __truediv__(self, o):
        if isinstance(o, (int, float)):
            return SyncedLoss(self.t / float(o), self.comm)
        return NotImplemented

    def __neg__(self):
        return SyncedLoss(-self.t, self.comm)

    # -- materialisation (collective) ------------------------------------------------------------------
    def item(self) -> float:
        if self._value is None:
            t = self.t.clone()
            self.comm.all_reduce(t, "avg")
            self._value = float(t.item())
        return self._value

    def __float__(self):
        return self.item()

    def __format__(self, spec):
        return format(self.item(), spec)

    def __repr__(self):
        return f"SyncedLoss({self.item()!r})" if self._value is not None else "SyncedLoss(<not synced>)"

    def __lt__(self, o):
        return self.item() < float(o)

    def __le__(self, o):
        return self.item() <= float(o)

    def __gt__(self, o):
        return self.item() > float(o)

    def __ge__(self, o):
        return self.item() >= float(o)

    def __eq__(self, o):
        return self.item() == float(o)

    def __ne__(self, o):
        return self.item() != float(o)

    def __bool__(self):
        return bool(self.item())

    def __int__(self):
        return int(self.item())


class Trainer:
    def __init__(self, model: nn.Module, optimizer, loss, batch_size_per_device: int, grad_accum_steps: int = 1,
                 grad_clip=None, gpu: bool = False, fp16=None, distributed=None, fairscale_oss: bool = False,
                 fairscale_sddp: bool = False, fairscale_fsdp: bool = False, configs=None, info_rank=0,
                 verbose: bool = True, ema_weight: float = 0.1, comm: Comm | None = None, fp8: bool = False,
                 lazy_loss_sync: bool = False, ema_print_every: int = 1, portable_checkpoint: bool = False):
        """``fp8=True`` (with bf16 precision on GPU): every framework ``Linear`` of the model runs its forward,
        data- and weight-gradient GEMMs in fp8 with delayed scaling (``ops.fp8.fp8_autocast``); norms,
        attention, the loss and the optimizer stay bf16 / fp32.
        ``lazy_loss_sync``: ``detach_and_sync_loss`` returns a ``SyncedLoss`` (synchronised when read) instead of
        Stoke's float (an all-reduce and a host read per call).  ``ema_print_every``: ``print_ema_loss`` acts on
        every N-th call only (Stoke prints on every call; the others then issue nothing at all).
        ``portable_checkpoint``: ``save`` writes the model in its standard layout where the model defines one
        (``to_portable_state_dict``: Llama's fused wqkv / w13 split back into Meta's wq, wk, wv / w1, w3); ``load``
        accepts either layout (``from_portable_state_dict``)."""
        self.verbose = verbose
        self.logger = RankLogger(info_rank, verbose)
        self._loss_fn = loss
        self.batch_size = int(batch_size_per_device)
        self.grad_accum = int(grad_accum_steps)
        self.grad_clip = grad_clip
        self.gpu = bool(gpu) and torch.cuda.is_available()
        fp16 = _val(fp16)
        distributed = _val(distributed)
        ds_cfg = find_config(configs, DeepspeedConfig)
        if distributed == "deepspeed" and ds_cfg is not None:
            stage = ds_cfg.zero_optimization.stage
            fairscale_oss = stage >= 1 or fairscale_oss
            fairscale_sddp = stage >= 2 or fairscale_sddp
            if stage >= 3:
                fairscale_fsdp, fairscale_oss, fairscale_sddp = True, False, False
            distributed = "ddp"
        if distributed == "fsdp":
            fairscale_fsdp = True
        self.fp16 = {"apex_O1": "amp", "apex_O2": "bf16", "deepspeed": "bf16"}.get(fp16, fp16)
        if fp8 and not (self.gpu and self.fp16 == "bf16"):
            raise ValueError("Trainer(fp8=True) needs gpu=True and fp16='bf16' (fp8 GEMMs under a bf16 compute dtype)")
        self.fp8 = bool(fp8)
        self.ddp_config = find_config(configs, DDPConfig) or DDPConfig()
        self.amp_config = find_config(configs, AMPConfig) or AMPConfig()
        self.oss_config = find_config(configs, FairscaleOSSConfig) or FairscaleOSSConfig()
        self.sddp_config = find_config(configs, FairscaleSDDPConfig) or FairscaleSDDPConfig()
        self.fsdp_config = find_config(configs, FairscaleFSDPConfig) or FairscaleFSDPConfig()

        # ---- process group / device
        self.distributed = distributed if distributed is not None or fairscale_fsdp else None
        if fairscale_fsdp and self.distributed is None:
            self.distributed = "fsdp"
        if self.distributed is not None:
            backend = self.ddp_config.backend if self.gpu else "gloo"
            if self.ddp_config.local_rank is not None and self.gpu:
                torch.cuda.set_device(int(self.ddp_config.local_rank) % torch.cuda.device_count())
            self.rank_, self.world_size_, self.device = init_distributed(backend, self.ddp_config.timeout_s)
            if not self.gpu:
                self.device = torch.device("cpu")
        else:
            self.rank_, self.world_size_ = 0, 1
            self.device = torch.device("cuda", torch.cuda.current_device()) if self.gpu else torch.device("cpu")
        self.comm = comm or Comm()
        self.status = TrainerStatus(self.gpu, self.distributed, self.fp16, fairscale_oss, fairscale_sddp,
                                    fairscale_fsdp, self.grad_accum, self.batch_size, self.world_size_).validate()

        # ---- precision
        self.scaler = None
        self.autocast_dtype = None
        if self.fp16 == "amp":
            self.autocast_dtype = torch.float16
            a = self.amp_config
            self.scaler = GradScaler(a.init_scale, a.growth_factor, a.backoff_factor, a.growth_interval,
                                     comm=self.comm, sharded=fairscale_sddp or fairscale_fsdp)
        elif self.fp16 == "bf16" and not fairscale_fsdp:
            self.autocast_dtype = torch.bfloat16

        # ---- model / engines
        if self.distributed is not None and self.ddp_config.convert_to_sync_batch_norm and not fairscale_fsdp:
            from ..parallel.syncbn import convert_sync_batchnorm
            model = convert_sync_batchnorm(model, self.comm)
        self._module = model
        opt_spec = optimizer if isinstance(optimizer, StokeOptimizer) else StokeOptimizer(**optimizer) \
            if isinstance(optimizer, dict) else StokeOptimizer(optimizer)
        opt_cls = self._fused_equivalent(opt_spec.optimizer)
        kw = dict(opt_spec.optimizer_kwargs)
        self._sharded_grads = False
        self.compute_dtype = None
        if fairscale_fsdp:
            from ..parallel.fsdp import FullyShardedDataParallel, MixedPrecision, ShardingStrategy
            c = self.fsdp_config
            mp = MixedPrecision(c.param_dtype if self.fp16 in ("bf16", None) and self.gpu else torch.float32,
                                c.reduce_dtype if self.gpu else torch.float32)
            if c.activation_checkpointing and hasattr(model, "config"):
                model.config.activation_checkpointing = True
            self._engine = FullyShardedDataParallel(
                model.to(self.device), wrap_classes=c.wrap_classes or None,
                sharding_strategy=ShardingStrategy(c.sharding_strategy), mixed_precision=mp, comm=self.comm,
                device=self.device, forward_prefetch=c.forward_prefetch, backward_prefetch=c.backward_prefetch,
                keep_low_precision_grads=opt_cls is FusedAdamW)
            self._optimizer = opt_cls(self._engine.flat_parameters(), **kw)
            self._clip_params = self._engine.flat_parameters
            self._sharded_grads = True
        else:
            model.to(self.device)
            # bf16 compute copy: with the fused optimizer the module itself runs on bf16 parameters that the
            # AdamW epilogue rewrites from fp32 masters, instead of autocast casting every fp32 weight to bf16
            # in every forward and every bf16 gradient back to fp32 (thousands of cast kernels per step)
            cdt = torch.bfloat16 if (self.gpu and self.fp16 == "bf16" and opt_cls is FusedAdamW) else None
            self.compute_dtype = cdt
            if fairscale_oss:
                from ..parallel.zero import OSS, ShardedDataParallel
                self._optimizer = OSS(model.parameters(), optim=opt_cls, comm=self.comm,
                                      broadcast_fp16=self.oss_config.broadcast_fp16, compute_dtype=cdt, **kw)
                s = self.sddp_config
                # ZeRO-2 (reduce each bucket to its owner, drop the rest) with SDDP, else ZeRO-1 gradients
                # (bucketed all-reduce over the same owner-contiguous flat) under DDP + OSS
                self._engine = ShardedDataParallel(model, self._optimizer, comm=self.comm,
                                                   broadcast_buffers=s.broadcast_buffers if fairscale_sddp else
                                                   self.ddp_config.broadcast_buffers,
                                                   sync_models_at_startup=s.sync_models_at_startup,
                                                   reduce_buffer_size=s.reduce_buffer_size if fairscale_sddp else
                                                   int(self.ddp_config.bucket_cap_mb * (1 << 20)),
                                                   reduce_fp16=s.reduce_fp16,
                                                   reduce_mode="reduce" if fairscale_sddp else "all_reduce")
                self._clip_params = self._optimizer.owned_params
                self._sharded_grads = True
            elif self.distributed is not None or cdt is not None:
                self._engine = self._make_ddp(model, rebuild=self.distributed is not None, compute_dtype=cdt)
                self._optimizer = opt_cls(self._engine.optimizer_parameters(), **kw)
                self._clip_params = self._engine.optimizer_parameters
            else:
                self._engine = model
                self._optimizer = opt_cls(model.parameters(), **kw)
                self._clip_params = lambda: list(self._module.parameters())

        # ---- counters / meters
        self._backward_steps = 0
        self._grad_accum_counter = 0
        self._optimizer_steps = 0
        self._ema_weight = ema_weight
        self._ema = None           # device tensor
        self._lazy_loss = bool(lazy_loss_sync)
        self._portable = bool(portable_checkpoint)
        self._ema_every = max(1, int(ema_print_every))
        self._ema_calls = 0
        self._ema_pending = []     # (event, pinned host scalar, message parts): EMA prints waiting for their copy
        self._last_loss = None
        self._training = True
        # PDT_COMM_DEBUG=1: cross-rank collective-sequence check every K optimizer steps
        self._verify_every = max(1, int(os.environ.get("PDT_VERIFY_EVERY", "50")))
        if verbose:
            self.logger.print(f"[Trainer] {self.status.as_dict()} device={self.device}")

    # ------------------------------------------------------------------ construction helpers
    def _fused_equivalent(self, cls):
        """torch AdamW/Adam -> the framework's fused AdamW on GPU (identical math and state layout)."""
        if self.gpu and cls in (torch.optim.AdamW, FusedAdamW):
            return FusedAdamW
        if self.gpu and cls is torch.optim.Adam:
            return lambda params, **kw: FusedAdamW(params, decoupled=False, **kw)
        return cls

    def _make_ddp(self, model, rebuild, compute_dtype=None):
        from ..parallel.ddp import DistributedDataParallel
        c = self.ddp_config
        return DistributedDataParallel(model, comm=self.comm, device=self.device, bucket_cap_mb=c.bucket_cap_mb,
                                       first_bucket_mb=c.first_bucket_mb, broadcast_buffers=c.broadcast_buffers,
                                       find_unused_parameters=c.find_unused_parameters, reduce_dtype=c.reduce_dtype,
                                       rebuild_buckets=rebuild, compute_dtype=compute_dtype)

    # ------------------------------------------------------------------ properties
    @property
    def model_access(self) -> nn.Module:
        return self._module

    @property
    def optimizer(self):
        return self._optimizer

    @property
    def world_size(self) -> int:
        return self.world_size_

    @property
    def rank(self) -> int:
        return self.rank_

    @property
    def effective_batch_size(self) -> int:
        return self.status.effective_batch_size

    @property
    def backward_steps(self) -> int:
        return self._backward_steps

    @property
    def optimizer_steps(self) -> int:
        return self._optimizer_steps

    @property
    def grad_accum_step(self) -> int:
        return self._grad_accum_counter

    @property
    def is_distributed(self) -> bool:
        return self.world_size_ > 1

    @property
    def ema_loss(self):
        return None if self._ema is None else float(self._ema)

    # ------------------------------------------------------------------ forward / loss / backward / step
    def _autocast(self):
        if self.autocast_dtype is None:
            return contextlib.nullcontext()
        return torch.autocast(self.device.type, dtype=self.autocast_dtype)

    def model(self, *args, **kwargs):
        with prof.range("pdt.forward"), self._autocast(), fp8_autocast(enabled=self.fp8):
            return self._engine(*args, **kwargs)

    __call__ = model

    def loss(self, *args, **kwargs):
        with self._autocast():
            out = self._loss_fn(*args, **kwargs)
        if isinstance(out, (list, tuple)):
            out = sum(out)
        d = out.detach().float()
        if self._ema is None:
            self._ema = d.clone()
        else:      # in place: a captured step (Trainer.graph) keeps chaining the same device scalar on replay
            self._ema.mul_(1 - self._ema_weight).add_(d, alpha=self._ema_weight)
        self._last_loss = d
        if self._module.training and self.grad_accum > 1:
            out = out / self.grad_accum
        return out

    def _is_boundary(self) -> bool:
        return (self._grad_accum_counter + 1) % self.grad_accum == 0

    def backward(self, loss):
        boundary = self._is_boundary()
        scaled = self.scaler.scale(loss) if self.scaler is not None else loss
        use_no_sync = (not boundary) and self.ddp_config.no_sync and hasattr(self._engine, "no_sync")
        with prof.range("pdt.backward"), (self._engine.no_sync() if use_no_sync else contextlib.nullcontext()):
            scaled.backward()
        self._backward_steps += 1
        self._grad_accum_counter = (self._grad_accum_counter + 1) % self.grad_accum

    def step(self):
        if self._grad_accum_counter != 0:
            return False   # not an accumulation boundary
        maybe_inject_fault(self._optimizer_steps)     # env-driven fault injection (tests of restart/resume)
        with prof.range("pdt.optimizer_step"):
            self._step()
        self._optimizer_steps += 1
        if self._optimizer_steps <= 3 and self.comm.world_size > 1 and not (
                torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()):
            # the kernel picks timed inside the first steps' forward / backward, agreed over THIS engine's group
            # at a point every rank reaches together (ops/picks.py) -- never from inside autograd
            picks.agree(self.comm)
        if self.comm.debug and self._optimizer_steps % self._verify_every == 0:
            self.comm.verify_consistency(f"after optimizer step {self._optimizer_steps}")
        return True

    def _step(self):
        params = self._clip_params() if callable(self._clip_params) else self._clip_params
        opt = self._optimizer
        fused = isinstance(opt, FusedAdamW) or (hasattr(opt, "optim") and isinstance(getattr(opt, "optim", None),
                                                                                    FusedAdamW))
        inv_scale = 1.0 / self.scaler.get_scale() if self.scaler is not None else 1.0
        max_norm = self.grad_clip.max_norm if isinstance(self.grad_clip, ClipGradNormConfig) else 0.0
        norm_type = self.grad_clip.norm_type if isinstance(self.grad_clip, ClipGradNormConfig) else 2.0
        if isinstance(self.grad_clip, ClipGradConfig):
            for p in params:
                g = grad_of(p)         # a compute-dtype master's gradient is its engine's flat (_pdt_grad)
                if g is not None:
                    if self.scaler is not None:
                        g.mul_(inv_scale)
                    g.clamp_(-self.grad_clip.clip_value, self.grad_clip.clip_value)
            inv_scale = 1.0
        need_stats = self.scaler is not None or max_norm > 0
        coef = found = None
        if need_stats:
            _, coef, found = clip_grad_norm_(params, max_norm, norm_type=norm_type, comm=self.comm,
                                             sharded=self._sharded_grads, inv_scale=inv_scale, apply=not fused)
            if self.scaler is not None:
                self.scaler._pending = (coef, found)
        if fused:
            opt.step(grad_scale=coef, found_inf=found)
        else:
            if found is None or int(found.item()) == 0:
                opt.step()
        if self.scaler is not None:
            self.scaler.update()
        self.zero_grads()

    def graph(self, step_fn, *static_inputs: torch.Tensor, warmup: int = 2):
        """Capture ``step_fn(*static_inputs)`` -- one or more WHOLE optimizer steps written against this Trainer
        (``model`` / ``loss`` / ``backward`` / ``step`` calls over the accumulation micro-batches) -- into a HIP
        graph (utils.graphs.GraphedStep) and return a callable that copies its arguments into the static
        buffers and replays the graph, advancing the Trainer's step counters exactly as the eager call does.
        Removes the per-launch host cost of many-small-kernel steps (SwinIR: ~3,500 launches per step).

        Needs the fused optimizer (switched to its capturable device step count here; under OSS the wrapped
        one) and no fp16 GradScaler (its scale update is host logic).  At world > 1 the collectives are
        captured with the step: RCCL (``nccl``) process group, DDP or ShardedDDP engine (their bucket
        readiness is switched to capture-safe hooks: ``prepare_capture``), and the xGMI mesh is bypassed
        while capturing (its epochs are host arguments).  FSDP's unit hooks are not capture-safe."""
        from ..utils.graphs import GraphedStep
        opt = self._optimizer
        inner = opt.optim if isinstance(getattr(opt, "optim", None), FusedAdamW) else opt
        fused = isinstance(inner, FusedAdamW)
        if not (self.gpu and fused and self.scaler is None):
            raise RuntimeError("Trainer.graph needs a GPU, FusedAdamW and no fp16 GradScaler")
        if self.world_size_ > 1:
            if self.comm.backend != "nccl" or not hasattr(self._engine, "prepare_capture"):
                raise RuntimeError("Trainer.graph at world > 1 needs the RCCL (nccl) backend and a DDP or "
                                   f"ShardedDDP engine (backend {self.comm.backend}, engine "
                                   f"{type(self._engine).__name__})")
            self._engine.prepare_capture()
        for g in list(inner.param_groups) + (list(opt.param_groups) if inner is not opt else []):
            g["capturable"] = True      # OSS copies its groups' hyper-parameters into the wrapped optimizer
        gs = GraphedStep(step_fn, *static_inputs, warmup=warmup)
        tr = self
        state = {"delta": None}

        def run(*inputs):
            before = (tr._backward_steps, tr._optimizer_steps)
            first = gs.graph is None
            out = gs(*inputs)
            if first:      # python ran warmup + 1 times (warm-up + capture); the device ran warmup + 1 (+ replay)
                n = gs.warmup + 1
                state["delta"] = ((tr._backward_steps - before[0]) // n, (tr._optimizer_steps - before[1]) // n)
            else:
                tr._backward_steps += state["delta"][0]
                tr._optimizer_steps += state["delta"][1]
            return out
        run.graphed = gs
        return run

    def zero_grads(self):
        if hasattr(self._engine, "zero_grad") and self._engine is not self._module:
            self._engine.zero_grad()
        self._optimizer.zero_grad(set_to_none=True)

    # ------------------------------------------------------------------ loss sync / printing
    def detach_and_sync_loss(self, loss, device=None, lazy: bool | None = None):
        """The loss averaged over ranks (Stoke-DDP.py:86).  Default: a float, as Stoke returns -- one all-reduce
        and one host read per call, a collective every rank makes.  ``lazy=True`` (or ``Trainer(lazy_loss_sync=
        True)``): a ``SyncedLoss`` device scalar that is NOT synchronised yet -- ``sum_loss += t.detach_and_sync_loss(
        loss, lazy=True)`` stays on the device, and the one all-reduce + host read happen when the sum is read (on
        log steps only); reading it is then the collective."""
        s = SyncedLoss(loss.detach().float().reshape(1).clone(), self.comm)
        if lazy if lazy is not None else self._lazy_loss:
            return s
        return s.item()

    def print_ema_loss(self, prepend_msg: str = "Current EMA Loss", postpend_msg: str = ""):
        """Print the EMA of the loss averaged over ranks (Stoke-DDP.py:76).  Every rank calls it (on a print call
        the ranks reduce their EMAs to the printing rank -- a device-side collective, no host wait on any rank).  The
        printing rank copies the value to pinned host memory asynchronously and prints it once the copy has
        landed (usually at its next call; ``flush_prints`` waits for the rest), so no call blocks the host on the
        device.  With ``ema_print_every=N`` only every N-th call does anything."""
        self._ema_calls += 1
        if self._ema is None or (self._ema_calls - 1) % self._ema_every:
            return
        t = self._ema.reshape(1).clone()
        if self.world_size_ > 1:
            ir = self.logger.info_rank
            if isinstance(ir, int) or (isinstance(ir, (list, tuple)) and len(ir) == 1):
                # one printing rank: reduce to it only
                self.comm.reduce(t, dst=int(ir if isinstance(ir, int) else ir[0]), op="avg")
            else:
                # several printing ranks ('all', a list, or None = every rank's logger decides): each needs the mean
                self.comm.all_reduce(t, "avg")
        if not self.logger.will_print():
            return
        parts = (prepend_msg, postpend_msg)
        if t.is_cuda:
            host = torch.empty(1, dtype=torch.float32, pin_memory=True)
            host.copy_(t, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._ema_pending.append((ev, host, parts))
            self._flush_ema(block=False)
        else:
            self._print_ema(float(t), parts)

    def _print_ema(self, v, parts):
        self.logger.print(f"{parts[0]}: {v:.5f} {parts[1]}".rstrip())

    def _flush_ema(self, block: bool):
        while self._ema_pending and (block or self._ema_pending[0][0].query()):
            ev, host, parts = self._ema_pending.pop(0)
            ev.synchronize()
            self._print_ema(float(host), parts)

    def flush_prints(self):
        """Print every EMA line still waiting for its device-to-host copy (waits for those copies)."""
        self._flush_ema(block=True)

    def print_on_devices(self, msg, rank=None):
        self.logger.print(msg, ranks=None if rank is None else (rank if isinstance(rank, (list, tuple)) else [rank]))

    def print(self, msg):
        self.logger.print(msg)

    def barrier(self):
        self.comm.barrier()

    def reset_ema(self):
        self._ema = None

    def train(self):
        self._module.train()

    def eval(self):
        self._module.eval()

    # ------------------------------------------------------------------ data
    def DataLoader(self, dataset, **kwargs):
        kwargs.setdefault("batch_size", self.batch_size)
        return DeviceDataLoader(dataset, device=self.device, **kwargs)

    # ------------------------------------------------------------------ checkpointing
    def _model_state(self):
        sd = self._model_state_native()
        fn = getattr(self._module, "to_portable_state_dict", None)
        if self._portable and fn is not None and sd:
            sd = fn(sd)
        return sd

    def _model_state_native(self):
        eng = self._engine
        if hasattr(eng, "sharding_strategy"):           # FSDP: full unflattened fp32 state dict, unit by
            return eng.state_dict(rank0_only=True, offload_to_cpu=True)   # unit to rank 0's host memory
        if hasattr(eng, "full_state_dict"):
            return eng.full_state_dict()
        return self._module.state_dict()

    def _optimizer_state(self):
        opt = self._optimizer
        if hasattr(opt, "consolidate_state_dict"):
            opt.consolidate_state_dict(recipient_rank=0)
            return opt.state_dict() if self.rank_ == 0 else None
        if hasattr(self._engine, "sharding_strategy"):
            return self._engine.full_optim_state_dict(opt, rank0_only=True, offload_to_cpu=True)
        if hasattr(self._engine, "full_optim_state_dict"):
            return self._engine.full_optim_state_dict(opt)
        return opt.state_dict()

    def save(self, path: str, name: str | None = None, extension: str = "pt", create_directory: bool = True,
             extras: dict | None = None):
        name = name or uuid.uuid4().hex[:8]
        self.flush_prints()
        model_state = self._model_state()
        opt_state = self._optimizer_state()
        return ckpt.save_checkpoint(
            path, name, model_state=model_state, optimizer_state=opt_state,
            scaler_state=self.scaler.state_dict() if self.scaler is not None else None,
            backward_step=self._backward_steps, grad_accum_step=self._grad_accum_counter,
            optimizer_step=self._optimizer_steps, status=self.status.as_dict(), extras=extras, extension=extension,
            rank=self.rank_, barrier=self.barrier if self.is_distributed else None, create_directory=create_directory)

    def load(self, path: str, tag: str, strict: bool = True, extension: str = "pt"):
        payload = ckpt.load_checkpoint(path, tag, extension=extension,
                                       map_location=self.device if self.device.type == "cpu" else "cpu")
        fn = getattr(self._module, "from_portable_state_dict", None)
        if fn is not None:
            payload["model_state_dict"] = fn(payload["model_state_dict"])
        eng = self._engine
        if hasattr(eng, "sharding_strategy"):
            eng.load_state_dict(payload["model_state_dict"], strict=strict)
        elif hasattr(eng, "load_full_state_dict"):
            eng.load_full_state_dict(payload["model_state_dict"], strict=strict)
        else:
            self._module.load_state_dict(payload["model_state_dict"], strict=strict)
        if payload.get("optimizer_state_dict") is not None:
            if hasattr(eng, "load_full_optim_state_dict"):
                eng.load_full_optim_state_dict(self._optimizer, payload["optimizer_state_dict"])
            else:
                self._optimizer.load_state_dict(payload["optimizer_state_dict"])
        if self.scaler is not None and payload.get("scaler_state_dict"):
            self.scaler.load_state_dict(payload["scaler_state_dict"])
        self._backward_steps = payload["backward_step"]
        self._grad_accum_counter = payload["grad_accum_step"]
        self._optimizer_steps = payload["optimizer_step"]
        return payload.get("extras")


Stoke = Trainer
