"""Multi-tensor launches: fused AdamW, fused L2 norm (+ non-finite check), clip coefficient, scale.

One HIP launch covers an arbitrary list of tensors through a device-resident table
(``csrc/kernels/multi_tensor.hip``).  The engines keep parameters/gradients in flat buffers so their
tables have a single entry; user parameter lists get one table per (dtype, group).

Reference parity: AdamW as configured in Stoke-DDP.py:226-235 / Fairscale-DDP.py:78-86 (math order
of torch/optim/adam.py:419-547), clip_grad_norm_ as configured by Stoke-DDP.py:253
(torch/nn/utils/clip_grad.py:50-186).
"""
from __future__ import annotations

import math
from typing import Sequence

import torch

from . import _lib

META = 6
DEFAULT_CHUNK = 32768


def _dense(t: torch.Tensor) -> bool:
    return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last)) or \
        (t.dim() == 5 and t.is_contiguous(memory_format=torch.channels_last_3d))


class TensorTable:
    """Device table describing up to 5 aligned tensor lists (+ numel) for a multi-tensor kernel.

    ``cols`` is a list of columns, each a list of tensors (or None) of equal length; column 0 defines
    the numel.  The table holds raw pointers, so the caller must keep the tensors alive and must
    rebuild the table if any storage is reallocated (``key()`` changes).
    """

    def __init__(self, cols: Sequence[Sequence[torch.Tensor | None]], chunk: int = DEFAULT_CHUNK):
        assert 1 <= len(cols) <= 5
        n = len(cols[0])
        for c in cols:
            assert len(c) == n
        self.chunk = int(chunk)
        self.cols = [list(c) for c in cols]
        self.numels = [t.numel() for t in cols[0]]
        dev = cols[0][0].device if n else torch.device("cpu")
        rows = max(n, 1)
        counts = torch.tensor([(m + self.chunk - 1) // self.chunk for m in self.numels] or [0], dtype=torch.int64)
        self.nblocks = int(counts.sum())
        nb = max(self.nblocks, 1)
        # ONE host buffer = meta rows (int64) followed by the (tensor, chunk) int32 pairs packed two per int64
        # word, filled without a per-chunk Python loop and uploaded with ONE asynchronous copy from pinned
        # memory: a pageable copy blocks the host until the stream drains (the whole backward, before the
        # clip norm) and the per-chunk loop cost ~4 ms per 1.3B-parameter table -- both idle GPU time
        # (profiles/r3_s4g_gpt2_1.3b_fsdp1_mb96_kernel_table.txt).
        host = torch.zeros(rows * META + nb, dtype=torch.int64, pin_memory=dev.type == "cuda")
        meta = host[:rows * META].view(rows, META)
        for i in range(n):
            ref = cols[0][i]
            for j, col in enumerate(cols):
                t = col[i]
                if t is not None:
                    # elementwise over the storage: any dense layout works if every column shares it
                    assert _dense(t), "multi-tensor kernels need dense (non-overlapping) tensors"
                    assert t.numel() == self.numels[i]
                    assert t.dim() <= 1 or all(a == b for a, b, k in zip(t.stride(), ref.stride(), ref.shape) if k != 1), \
                        "multi-tensor columns must share a layout"   # (a size-1 dimension's stride is arbitrary)
                    meta[i, j] = t.data_ptr()
            meta[i, 5] = self.numels[i]
        if self.nblocks:
            tid = torch.repeat_interleave(torch.arange(len(counts), dtype=torch.int64), counts)
            first = torch.cumsum(counts, 0) - counts
            cid = torch.arange(self.nblocks, dtype=torch.int64) - torch.repeat_interleave(first, counts)
            host[rows * META:] = tid | (cid << 32)           # little-endian: int32 pair (tensor, chunk)
        if dev.type == "cuda":
            buf = host.to(dev, non_blocking=True)
            self._host = host                                 # pinned source stays alive with the table
        else:
            buf = host
        self.meta = buf[:rows * META].view(rows, META)
        self.blk = buf[rows * META:].view(torch.int32).view(nb, 2)
        self._key = self.make_key(cols)
        self.device = dev

    @staticmethod
    def make_key(cols) -> tuple:
        return tuple((t.data_ptr(), t.numel()) if t is not None else None for c in cols for t in c)

    def key(self) -> tuple:
        return self._key


class TableCache:
    """Rebuilds a TensorTable only when the pointer set changes."""

    def __init__(self):
        self._tables = {}

    def get(self, name, cols, chunk=DEFAULT_CHUNK) -> TensorTable:
        key = TensorTable.make_key(cols)
        t = self._tables.get(name)
        if t is None or t.key() != key:
            t = TensorTable(cols, chunk)
            self._tables[name] = t
        return t

    def retain(self, keep) -> None:
        """Drop every cached table whose name fails ``keep(name)`` (its device table is freed with it)."""
        for n in [n for n in self._tables if not keep(n)]:
            del self._tables[n]

    def __len__(self):
        return len(self._tables)


_cache = TableCache()


def l2norm_sq(tensors: Sequence[torch.Tensor], out: torch.Tensor | None = None, accumulate=False,
              table: TensorTable | None = None) -> torch.Tensor:
    """Sum of squares over all tensors as a 1-element fp32 device tensor (no host sync)."""
    tensors = [t for t in tensors if t is not None and t.numel() > 0]
    if not tensors:
        o = out if out is not None else torch.zeros(1, dtype=torch.float32)
        if not accumulate:
            o.zero_()
        return o
    dev = tensors[0].device
    if out is None:
        out = torch.zeros(1, dtype=torch.float32, device=dev)
    if dev.type != "cuda":
        s = torch.zeros((), dtype=torch.float32)
        for t in tensors:
            s = s + t.detach().float().pow(2).sum()
        if accumulate:
            out.add_(s)
        else:
            out.copy_(s.reshape(1))
        return out
    by_dt = {}
    for t in tensors:
        by_dt.setdefault(t.dtype, []).append(t)
    first = True
    for dt, ts in by_dt.items():
        tab = table if (table is not None and len(by_dt) == 1) else _cache.get(("l2", dt, len(ts)), [ts])
        partial = torch.empty(max(tab.nblocks, 1), dtype=torch.float32, device=dev)
        _lib.call("pdt_l2norm_mt", tab.meta.data_ptr(), tab.blk.data_ptr(), tab.nblocks, tab.chunk,
                  _lib.dtype_code(dt), partial.data_ptr(), out.data_ptr(), 1 if (accumulate or not first) else 0,
                  _lib.stream_handle(dev))
        first = False
    return out


def clip_coef(total_sq: torch.Tensor, max_norm: float, inv_scale: torch.Tensor | float = 1.0):
    """From an (all-reduced) sum of squares: (norm, grad_multiplier, found_inf) device tensors.

    grad_multiplier = min(1, max_norm/(norm+1e-6)) * inv_scale; max_norm<=0 disables clipping."""
    dev = total_sq.device
    norm = torch.empty(1, dtype=torch.float32, device=dev)
    coef = torch.empty(1, dtype=torch.float32, device=dev)
    found = torch.empty(1, dtype=torch.int32, device=dev)
    if dev.type != "cuda":
        inv = float(inv_scale) if not torch.is_tensor(inv_scale) else float(inv_scale.reshape(-1)[0])
        sq = float(total_sq.reshape(-1)[0])
        fin = math.isfinite(sq)
        nrm = math.sqrt(sq) * inv if fin else float("nan") if sq != sq else float("inf")
        c = min(max_norm / (nrm + 1e-6), 1.0) if (max_norm > 0 and fin) else 1.0
        norm.fill_(nrm)
        coef.fill_(c * inv)
        found.fill_(0 if fin else 1)
        return norm, coef, found
    if torch.is_tensor(inv_scale):
        inv_ptr, inv_val = inv_scale.data_ptr(), 1.0
    else:
        inv_ptr, inv_val = 0, float(inv_scale)
    _lib.call("pdt_clip_coef", total_sq.data_ptr(), float(max_norm), inv_ptr, inv_val, norm.data_ptr(),
              coef.data_ptr(), found.data_ptr(), _lib.stream_handle(dev))
    return norm, coef, found


def scale_(tensors: Sequence[torch.Tensor], s: torch.Tensor) -> None:
    """In-place multiply every tensor by the device scalar ``s``."""
    tensors = [t for t in tensors if t is not None and t.numel() > 0]
    if not tensors:
        return
    dev = tensors[0].device
    if dev.type != "cuda":
        for t in tensors:
            t.mul_(s.to(t.dtype))
        return
    by_dt = {}
    for t in tensors:
        by_dt.setdefault(t.dtype, []).append(t)
    for dt, ts in by_dt.items():
        tab = _cache.get(("scale", dt, len(ts)), [ts])
        _lib.call("pdt_scale_mt", tab.meta.data_ptr(), tab.blk.data_ptr(), tab.nblocks, tab.chunk,
                  _lib.dtype_code(dt), s.data_ptr(), _lib.stream_handle(dev))


def adamw_step(params, grads, exp_avgs, exp_avg_sqs, *, lr: float, beta1: float, beta2: float, eps: float,
               weight_decay: float, step: int, decoupled: bool = True, grad_scale: torch.Tensor | None = None,
               found_inf: torch.Tensor | None = None, out_bf16=None, table: TensorTable | None = None,
               dstep: torch.Tensor | None = None) -> None:
    """One fused (multi-tensor) AdamW update.  fp32 params/state; grads fp32 or bf16.

    grad_scale: optional device scalar multiplied into every gradient (unscale x clip coefficient).
    found_inf: optional device int32 flag; non-zero skips the update (GradScaler semantics).
    out_bf16: optional list of bf16 tensors receiving the updated params (low-precision compute copy /
    all-gather input for the sharded engines).
    dstep: optional device fp32 step count (already incremented): the kernel derives the bias corrections
    from it, so the launch replays correctly inside a captured HIP graph (``step`` is then ignored)."""
    if dstep is not None and params and params[0].device.type != "cuda":
        step = int(dstep.item())
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    step_size = lr / bc1
    bc2_sqrt = math.sqrt(bc2)
    if len(params) == 0:
        return
    dev = params[0].device
    if dev.type != "cuda":
        if found_inf is not None and int(found_inf.reshape(-1)[0]) != 0:
            return
        gs = None if grad_scale is None else grad_scale.reshape(())
        for i, p in enumerate(params):
            g = grads[i].float()
            if gs is not None:
                g = g * gs
            m, v = exp_avgs[i], exp_avg_sqs[i]
            if decoupled:
                p.mul_(1 - lr * weight_decay)
            elif weight_decay != 0:
                g = g + weight_decay * p
            m.mul_(beta1).add_(g, alpha=1 - beta1)
            v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
            denom = v.sqrt() / bc2_sqrt + eps
            p.addcdiv_(m, denom, value=-step_size)
            if out_bf16 is not None and out_bf16[i] is not None:
                out_bf16[i].copy_(p)
        return
    gdt = grads[0].dtype
    if table is None:
        cols = [list(params), list(grads), list(exp_avgs), list(exp_avg_sqs)]
        cols.append(list(out_bf16) if out_bf16 is not None else [None] * len(params))
        table = _cache.get(("adamw", gdt, len(params), id(params[0])), cols)
    _lib.call("pdt_adamw_mt", table.meta.data_ptr(), table.blk.data_ptr(), table.nblocks, table.chunk,
              _lib.dtype_code(gdt), float(lr), float(beta1), float(beta2), float(eps), float(weight_decay),
              float(step_size), float(bc2_sqrt), 1 if decoupled else 0, _lib.ptr(grad_scale), _lib.ptr(found_inf),
              _lib.ptr(dstep), _lib.stream_handle(dev))


def step_inc_(dstep: torch.Tensor, found_inf: torch.Tensor | None = None) -> None:
    """dstep += 1 unless ``found_inf`` (device int32 flag) is set -- on the device, no host sync."""
    if dstep.device.type != "cuda":
        if found_inf is None or int(found_inf.reshape(-1)[0]) == 0:
            dstep.add_(1.0)
        return
    _lib.call("pdt_step_inc", dstep.data_ptr(), _lib.ptr(found_inf), _lib.stream_handle(dstep.device))


def cast_f32_to_bf16(src: torch.Tensor, dst: torch.Tensor) -> None:
    assert src.dtype == torch.float32 and dst.dtype == torch.bfloat16 and src.numel() == dst.numel()
    if src.device.type != "cuda":
        dst.copy_(src)
        return
    _lib.call("pdt_cast_f32_bf16", src.data_ptr(), dst.data_ptr(), src.numel(), _lib.stream_handle(src.device))


def add_(dsts: Sequence[torch.Tensor], srcs: Sequence[torch.Tensor | None], name: str = "add") -> None:
    """dst += src for every pair (same dtype, same element order; a None src adds nothing) in ONE launch on CUDA
    (bf16 / fp32) -- per-parameter gradients accumulated into a flat buffer."""
    pairs = [(d, s) for d, s in zip(dsts, srcs) if s is not None]
    if not pairs:
        return
    dev = pairs[0][0].device
    if dev.type != "cuda" or pairs[0][0].dtype not in (torch.bfloat16, torch.float32) or \
            torch.cuda.is_current_stream_capturing():
        torch._foreach_add_([d for d, _ in pairs], [s for _, s in pairs])
        return
    for d, s in pairs:
        assert s.dtype == d.dtype and s.numel() == d.numel()
    t = _cache.get(name, [[d for d, _ in pairs], [s for _, s in pairs]])
    _lib.call("pdt_add_mt", t.meta.data_ptr(), t.blk.data_ptr(), t.nblocks, t.chunk, _lib.dtype_code(pairs[0][0].dtype),
              _lib.stream_handle(dev))


def copy_(dsts: Sequence[torch.Tensor], srcs: Sequence[torch.Tensor | None], name: str = "copy") -> None:
    """dst.copy_(src) for every pair (same dtype, same element order; a None src zero-fills its dst) in ONE
    launch on CUDA -- e.g. per-parameter gradients gathered into a flat buffer."""
    if not dsts:
        return
    dev = dsts[0].device
    if dev.type != "cuda":
        for d, s in zip(dsts, srcs):
            d.zero_() if s is None else d.copy_(s)
        return
    for d, s in zip(dsts, srcs):
        assert s is None or (s.dtype == d.dtype and s.numel() == d.numel())
    key = TensorTable.make_key([list(dsts), list(srcs)])
    cached = _cache._tables.get(name)
    if torch.cuda.is_current_stream_capturing() and (cached is None or cached.key() != key):
        # a new pointer set while a HIP graph is captured: no table upload is allowed -- torch's foreach copy
        pairs = [(d, s) for d, s in zip(dsts, srcs) if s is not None]
        if pairs:
            torch._foreach_copy_([d for d, _ in pairs], [s for _, s in pairs])
        zs = [d for d, s in zip(dsts, srcs) if s is None]
        if zs:
            torch._foreach_zero_(zs)
        return
    t = _cache.get(name, [list(dsts), list(srcs)])
    _lib.call("pdt_copy_mt", t.meta.data_ptr(), t.blk.data_ptr(), t.nblocks, t.chunk, dsts[0].element_size(),
              _lib.stream_handle(dev))
