"""Uniform collective layer used by every engine (DDP bucketer, ZeRO-1/2, FSDP, SyncBN, facade).

Backends
  * ``nccl`` -- on ROCm this IS RCCL over xGMI (one process per GPU).  Collectives are enqueued on
    c10d's internal communication stream after an event wait on the caller's stream, so issuing them
    with ``async_op=True`` from autograd hooks overlaps them with backward compute; ``Handle.wait()``
    makes the *current* stream wait (no host sync).
  * ``gloo`` -- CPU bootstrap / CPU tests (reduce-scatter and AVG emulated on top of all-reduce).

Every call can be recorded in the native ``CollectiveTracer`` (sequence number + shape hash); in
debug mode (``PDT_COMM_DEBUG=1`` or ``TORCH_DISTRIBUTED_DEBUG=DETAIL``) ``verify_consistency()``
compares the rolling hash across ranks -- the mismatch detector of SURVEY.md §5.2.

Reference: the collectives the reference triggers through torch/Fairscale,
re-issued here as few, large, bucketed operations.  The bucket / window sizes are chosen from link arithmetic
for 7 xGMI links per GPU and are defaults UNMEASURED on a multi-GPU node: no sweep against RCCL
has run yet (every run so far had one GPU).
"""
from __future__ import annotations

import os
from contextlib import contextmanager

import torch
import torch.distributed as dist

from ..utils.native import runtime

_DT_CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int64: 3, torch.int32: 4,
            torch.uint8: 5, torch.float64: 6}


# Exposed-communication probe (bench.py / StepTimer users): while a list is installed, every device-side
# wait records an event pair on the WAITING stream; the GPU time between them is the time that stream
# stalled on communication (zero when the collective already finished under earlier compute).
_WAIT_EVENTS = None


def start_wait_timing():
    global _WAIT_EVENTS
    _WAIT_EVENTS = []


def stop_wait_timing() -> float:
    """Stop recording; return the summed compute-stream stall (ms) of the waits seen (synchronises)."""
    global _WAIT_EVENTS
    evs, _WAIT_EVENTS = _WAIT_EVENTS or [], None
    if not evs:
        return 0.0
    torch.cuda.synchronize()
    return float(sum(a.elapsed_time(b) for a, b in evs))


class Handle:
    """Async work handle; ``wait()`` orders the current stream after the collective (no host sync for
    device collectives: a c10d work's wait, or a stream wait on the xGMI comm stream's event)."""

    def __init__(self, work=None, post=None, event=None):
        self._work = work
        self._post = post
        self._event = event
        self._done = work is None and post is None and event is None

    def wait(self):
        if self._done:
            return
        timed = _WAIT_EVENTS is not None and (self._work is not None or self._event is not None) \
            and torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing()
        if timed:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        if self._work is not None:
            self._work.wait()
        if self._event is not None:
            torch.cuda.current_stream().wait_event(self._event)
        if timed:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            _WAIT_EVENTS.append((e0, e1))
        if self._post is not None:
            self._post()
        self._done = True

    def is_completed(self) -> bool:
        if self._done:
            return True
        if self._event is not None:
            return self._event.query()
        return self._work is not None and self._work.is_completed()


def _xgmi_handle(ev, async_op: bool) -> Handle:
    h = Handle(event=ev)
    if not async_op:
        h.wait()          # stream-ordered for the caller, still no host sync
    return h


class Comm:
    def __init__(self, group=None, debug: bool | None = None, xgmi: bool | None = None):
        self.group = group
        self.initialized = dist.is_available() and dist.is_initialized()
        if self.initialized:
            self.rank = dist.get_rank(group)
            self.world_size = dist.get_world_size(group)
            self.backend = str(dist.get_backend(group))
        else:
            self.rank, self.world_size, self.backend = 0, 1, "none"
        if debug is None:
            debug = os.environ.get("PDT_COMM_DEBUG", "0") == "1" or \
                os.environ.get("TORCH_DISTRIBUTED_DEBUG", "").upper() == "DETAIL"
        self.debug = debug
        self.stats = {"calls": 0, "bytes": 0}
        self.op_log = None       # list of (op, numel, dtype, device) while recording (bench comm-only replay)
        rt = runtime()
        self.tracer = rt.CollectiveTracer(4096) if rt is not None else None
        self.xgmi = None
        if xgmi is None:
            from ..run_config import xgmi_mode
            xgmi = xgmi_mode() != "off"
        if xgmi and self.world_size > 1 and torch.cuda.is_available():
            from ..run_config import xgmi_kwargs
            self.enable_xgmi(**xgmi_kwargs())

    def enable_xgmi(self, **kw):
        """Route eligible CUDA all_reduce / all_gather / reduce_scatter through the peer-mapped xGMI
        kernels (parallel/xgmi.py).  Collective: every rank must call it."""
        from .xgmi import XGMIComm
        if self.xgmi is None and self.world_size > 1:
            self.xgmi = XGMIComm(self, **kw)
        return self.xgmi

    def _xgmi_ok(self, t, kind="all_reduce") -> bool:
        x = self.xgmi
        # not under HIP-graph capture: the mesh's epochs are host-issued kernel arguments, and a replayed
        # epoch would match the flags of the previous replay -- captured steps take RCCL, which captures
        return (x is not None and t.is_cuda and t.is_contiguous()
                and x.eligible(t.numel() * t.element_size(), kind, t.dtype)
                and not torch.cuda.is_current_stream_capturing())

    # ------------------------------------------------------------------ helpers
    @property
    def is_gloo(self) -> bool:
        return self.backend == "gloo"

    def _trace(self, op, t, nbytes=None):
        """Sequence/shape record for the consistency checker plus per-process traffic counters
        (``stats``: collective calls and full-payload bytes, read by bench.py per step)."""
        self.stats["calls"] += 1
        self.stats["bytes"] += t.numel() * t.element_size() if nbytes is None else nbytes
        if self.op_log is not None:
            self.op_log.append((op, t.numel(), t.dtype, t.device))
        if self.tracer is not None:
            self.tracer.record(op, list(t.shape), _DT_CODE.get(t.dtype, 99))

    def reset_stats(self):
        self.stats = {"calls": 0, "bytes": 0}

    # ------------------------------------------------------------------ collectives
    def all_reduce(self, t: torch.Tensor, op: str = "sum", async_op: bool = False) -> Handle:
        self._trace("all_reduce:" + op, t)
        if self.world_size == 1:
            return Handle()
        if op in ("sum", "avg") and self._xgmi_ok(t):
            return _xgmi_handle(self.xgmi.all_reduce(t, op, async_op=True), async_op)
        if op == "avg" and self.is_gloo:
            w = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)
            ws = self.world_size

            def post():
                t.div_(ws)
            if not async_op:
                post()
                return Handle()
            return Handle(w, post)
        rop = {"sum": dist.ReduceOp.SUM, "avg": dist.ReduceOp.AVG, "max": dist.ReduceOp.MAX,
               "min": dist.ReduceOp.MIN}[op]
        w = dist.all_reduce(t, op=rop, group=self.group, async_op=async_op)
        return Handle(w) if async_op else Handle()

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum", async_op: bool = False) -> Handle:
        """out = op over ranks of inp.chunk(world)[rank] (inp numel = world * out numel)."""
        self._trace("reduce_scatter:" + op, inp)
        if self.world_size == 1:
            if out.data_ptr() != inp.data_ptr():
                out.copy_(inp.view_as(out))
            return Handle()
        if op in ("sum", "avg") and out.dtype == inp.dtype and self._xgmi_ok(inp, "reduce_scatter") \
                and out.is_contiguous():
            return _xgmi_handle(self.xgmi.reduce_scatter(out, inp, op, async_op=True), async_op)
        if self.is_gloo:
            buf = inp.clone()
            w = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)
            n, r, ws = out.numel(), self.rank, self.world_size

            def post():
                out.copy_(buf.view(-1)[r * n:(r + 1) * n].view_as(out))
                if op == "avg":
                    out.div_(ws)
            if not async_op:
                post()
                return Handle()
            return Handle(w, post)
        rop = dist.ReduceOp.AVG if op == "avg" else dist.ReduceOp.SUM
        w = dist.reduce_scatter_tensor(out, inp, op=rop, group=self.group, async_op=async_op)
        return Handle(w) if async_op else Handle()

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False) -> Handle:
        """out (world * inp numel) = concat over ranks of inp."""
        self._trace("all_gather", inp, out.numel() * out.element_size())
        if self.world_size == 1:
            if out.data_ptr() != inp.data_ptr():
                out.view(-1).copy_(inp.view(-1))
            return Handle()
        if out.dtype == inp.dtype and out.is_contiguous() and self._xgmi_ok(inp, "all_gather"):
            return _xgmi_handle(self.xgmi.all_gather(out, inp, async_op=True), async_op)
        if self.is_gloo:
            parts = list(out.view(self.world_size, -1).unbind(0))
            w = dist.all_gather(parts, inp.view(-1).contiguous(), group=self.group, async_op=async_op)
            return Handle(w) if async_op else Handle()
        w = dist.all_gather_into_tensor(out, inp, group=self.group, async_op=async_op)
        return Handle(w) if async_op else Handle()

    def broadcast(self, t: torch.Tensor, src: int = 0, async_op: bool = False) -> Handle:
        self._trace("broadcast", t)
        if self.world_size == 1:
            return Handle()
        gsrc = dist.get_global_rank(self.group, src) if self.group is not None else src
        w = dist.broadcast(t, src=gsrc, group=self.group, async_op=async_op)
        return Handle(w) if async_op else Handle()

    def reduce(self, t: torch.Tensor, dst: int, op: str = "sum", async_op: bool = False) -> Handle:
        self._trace("reduce", t)
        if self.world_size == 1:
            return Handle()
        if op in ("sum", "avg") and self._xgmi_ok(t, "reduce"):
            return _xgmi_handle(self.xgmi.reduce(t, dst, op, async_op=True), async_op)
        gdst = dist.get_global_rank(self.group, dst) if self.group is not None else dst
        w = dist.reduce(t, dst=gdst, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)
        if op == "avg":
            ws, r = self.world_size, self.rank

            def post():
                if r == dst:
                    t.div_(ws)
            if not async_op:
                post()
                return Handle()
            return Handle(w, post)
        return Handle(w) if async_op else Handle()

    def barrier(self):
        if self.world_size > 1:
            if self.backend == "nccl" and torch.cuda.is_available():
                dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
            else:
                dist.barrier(group=self.group)

    def broadcast_object(self, obj, src: int = 0):
        if self.world_size == 1:
            return obj
        lst = [obj if self.rank == src else None]
        gsrc = dist.get_global_rank(self.group, src) if self.group is not None else src
        dist.broadcast_object_list(lst, src=gsrc, group=self.group)
        return lst[0]

    def all_gather_object(self, obj):
        if self.world_size == 1:
            return [obj]
        out = [None] * self.world_size
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def broadcast_coalesced(self, tensors, src: int = 0, bucket_bytes: int = 256 << 20):
        """Broadcast a list of tensors with one collective per (dtype, bucket)."""
        if self.world_size == 1 or not tensors:
            return
        by_dt = {}
        for t in tensors:
            by_dt.setdefault((t.dtype, t.device), []).append(t)
        for (_dt, _dev), ts in by_dt.items():
            i = 0
            while i < len(ts):
                chunk, nbytes = [], 0
                while i < len(ts) and (not chunk or nbytes + ts[i].numel() * ts[i].element_size() <= bucket_bytes):
                    chunk.append(ts[i])
                    nbytes += ts[i].numel() * ts[i].element_size()
                    i += 1
                flat = torch.cat([t.detach().reshape(-1) for t in chunk])
                self.broadcast(flat, src)
                off = 0
                for t in chunk:
                    n = t.numel()
                    with torch.no_grad():
                        t.copy_(flat[off:off + n].view_as(t))
                    off += n

    # ------------------------------------------------------------------ failure detection / debug
    def check_errors(self):
        """Raise if a device collective of this rank failed (xGMI timeout word, read without a device sync).
        Called by the engines at their end-of-backward sync points."""
        if self.xgmi is not None:
            self.xgmi.raise_if_failed()

    def verify_consistency(self, tag: str = "") -> None:
        """Cross-rank check that every rank issued the same collective sequence (debug mode)."""
        if self.tracer is None or self.world_size == 1:
            return
        mine = (int(self.tracer.seq), int(self.tracer.rolling_hash))
        allv = self.all_gather_object(mine)
        if any(v != allv[0] for v in allv):
            raise RuntimeError(f"collective mismatch across ranks {tag}: (seq, hash) per rank = {allv}")


_default = None


def default_comm() -> Comm:
    global _default
    if _default is None or (_default.initialized != (dist.is_available() and dist.is_initialized())):
        _default = Comm()
    return _default


@contextmanager
def comm_debug(comm: Comm):
    old = comm.debug
    comm.debug = True
    try:
        yield comm
    finally:
        comm.debug = old
