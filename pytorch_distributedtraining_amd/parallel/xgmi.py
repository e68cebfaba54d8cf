"""Direct peer-to-peer collectives over the xGMI mesh of one MI355X node.

Every rank allocates ONE symmetric HBM buffer ([4 KB signals][staging slot 0][staging slot 1]), exports
it with ``hipIpcGetMemHandle`` and maps every peer's buffer with ``hipIpcOpenMemHandle`` -- the handles
are exchanged once through the existing c10d process group (TCPStore bootstrap).  The
collectives are HIP kernels in ``csrc/kernels/xgmi_comm.hip`` that read peers' staging slots directly
(system-scope, cache-bypassing loads) after a bounded mesh barrier:

  * ``all_reduce``   one-shot (<= ``oneshot_max_bytes``: grad-norm / found_inf scalars, loss sync,
                     SyncBN statistics -- latency class) or two-shot (reduce-scatter + all-gather phases:
                     2(W-1)/W of the payload over all 7 links at once -- bandwidth class);
  * ``all_gather`` / ``reduce_scatter`` of one staging slot.

They run on the caller's current HIP stream (stream-ordered like every other kernel: no host sync, no
separate communication stream), so a ``Handle`` returned to the engines is already complete from the
host's point of view.  A wait that exceeds ``spin_limit`` never hangs the queue: the kernel records an
error bit that ``check()`` raises on.

``Comm(xgmi=True)`` (or ``PDT_XGMI=1``) routes eligible CUDA collectives here (sizes that are a multiple
of 16 B, world <= 8, payload <= one staging slot); everything else stays on RCCL.  Ranks must issue
collectives in the same order (the same contract as RCCL).
"""
from __future__ import annotations

import ctypes

import torch

from ..ops import _lib

_KIND = {"allreduce1": 0, "allreduce2": 1, "all_gather": 2, "reduce_scatter": 3, "barrier": 4}
SIG_BYTES = 4096
MAX_WORLD = 8


class XGMIComm:
    """Peer-mapped collectives for ``comm``'s ranks (one process per GPU of one node)."""

    def __init__(self, comm, slot_bytes: int = 64 << 20, oneshot_max_bytes: int = 256 << 10,
                 spin_limit: int = 1 << 24, uncached: bool = True):
        if comm.world_size > MAX_WORLD:
            raise ValueError(f"XGMIComm spans one node (<= {MAX_WORLD} GPUs), got world_size={comm.world_size}")
        self.comm = comm
        self.rank, self.world = comm.rank, comm.world_size
        self.slot_bytes = int(slot_bytes)
        self.oneshot_max_bytes = int(oneshot_max_bytes)
        self.spin_limit = int(spin_limit)
        self.device = torch.device("cuda", torch.cuda.current_device())
        lib = _lib.require()   # ctypes signatures: ops/_lib.py _SIGS (checked against the C sources)
        self._lib = lib
        nbytes = SIG_BYTES + 2 * self.slot_bytes
        own = ctypes.c_void_p()
        _lib.check(lib.pdt_xgmi_alloc(nbytes, 1 if uncached else 0, ctypes.byref(own)), "pdt_xgmi_alloc")
        self._own = own
        hb = lib.pdt_xgmi_ipc_handle_bytes()
        handle = ctypes.create_string_buffer(hb)
        _lib.check(lib.pdt_xgmi_ipc_get(own, handle), "pdt_xgmi_ipc_get")
        handles = comm.all_gather_object(bytes(handle.raw))
        ptrs, self._opened = [], []
        for p, h in enumerate(handles):
            if p == self.rank:
                ptrs.append(own.value)
                continue
            q = ctypes.c_void_p()
            _lib.check(lib.pdt_xgmi_ipc_open(ctypes.create_string_buffer(h, hb), ctypes.byref(q)), "pdt_xgmi_ipc_open")
            self._opened.append(q)
            ptrs.append(q.value)
        self._bufs = (ctypes.c_void_p * MAX_WORLD)(*(ptrs + [None] * (MAX_WORLD - len(ptrs))))
        self.epoch = 0
        comm.barrier()

    # ------------------------------------------------------------------ eligibility
    def eligible(self, nbytes: int, kind: str = "all_reduce") -> bool:
        if nbytes <= 0 or nbytes % 16 or nbytes > self.slot_bytes:
            return False
        if kind in ("reduce_scatter", "allreduce2") and nbytes % (16 * self.world):
            return False
        return True

    # ------------------------------------------------------------------ launch
    def _run(self, kind: str, inp, out, in_bytes: int, dtype: torch.dtype, scale: float):
        self.epoch += 1
        if self.epoch >= 1 << 32:
            self.epoch = 1
        code = _lib.dtype_code(dtype) if dtype is not None else 0
        err = self._lib.pdt_xgmi_collective(_KIND[kind], _lib.ptr(inp), _lib.ptr(out), int(in_bytes), code,
                                            float(scale), self._bufs, self.rank, self.world, self.epoch,
                                            self.slot_bytes, self.spin_limit, _lib.stream_handle(self.device))
        _lib.check(err, f"pdt_xgmi_collective[{kind}]")

    @staticmethod
    def _flat(t):
        if not t.is_contiguous():
            raise ValueError("xGMI collectives need contiguous tensors")
        return t.view(-1)

    def all_reduce(self, t: torch.Tensor, op: str = "sum", out: torch.Tensor | None = None) -> torch.Tensor:
        """In place (or into ``out``): sum / avg over ranks.  fp32 or bf16 (fp32 accumulation)."""
        if op not in ("sum", "avg"):
            raise ValueError(f"xGMI all_reduce supports sum/avg, got {op}")
        nbytes = t.numel() * t.element_size()
        if not self.eligible(nbytes):
            raise ValueError(f"xGMI all_reduce: {nbytes} B not eligible")
        out = t if out is None else out
        scale = 1.0 / self.world if op == "avg" else 1.0
        two_shot = nbytes > self.oneshot_max_bytes and nbytes % (16 * self.world) == 0
        self._run("allreduce2" if two_shot else "allreduce1", self._flat(t), self._flat(out), nbytes, t.dtype, scale)
        return out

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        nbytes = inp.numel() * inp.element_size()
        if out.numel() != inp.numel() * self.world or not self.eligible(nbytes):
            raise ValueError("xGMI all_gather: bad sizes")
        self._run("all_gather", self._flat(inp), self._flat(out), nbytes, inp.dtype, 1.0)
        return out

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum") -> torch.Tensor:
        nbytes = inp.numel() * inp.element_size()
        if inp.numel() != out.numel() * self.world or not self.eligible(nbytes, "reduce_scatter"):
            raise ValueError("xGMI reduce_scatter: bad sizes")
        scale = 1.0 / self.world if op == "avg" else 1.0
        self._run("reduce_scatter", self._flat(inp), self._flat(out), nbytes, inp.dtype, scale)
        return out

    def barrier(self):
        self._run("barrier", None, None, 0, None, 1.0)

    def check(self):
        """Raise if any mesh wait on this rank timed out since the last check (synchronises the device)."""
        torch.cuda.synchronize(self.device)
        v = ctypes.c_uint(0)
        _lib.check(self._lib.pdt_xgmi_error(self._own, ctypes.byref(v)), "pdt_xgmi_error")
        if v.value:
            raise RuntimeError(f"xGMI collective timed out on rank {self.rank} (barrier bits {v.value:#x}): "
                               "a peer did not reach the same collective")

    def close(self):
        if getattr(self, "_own", None) is None:
            return
        torch.cuda.synchronize(self.device)
        self.comm.barrier()          # no peer may still read our buffer
        for q in self._opened:
            self._lib.pdt_xgmi_ipc_close(q)
        self._opened = []
        self._lib.pdt_xgmi_free(self._own)
        self._own = None
