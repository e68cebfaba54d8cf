"""Direct peer-to-peer collectives over the xGMI mesh of one MI355X node.

Every rank allocates ONE symmetric HBM buffer ([4 KB signals][staging slot 0][staging slot 1]), exports
it with ``hipIpcGetMemHandle`` and maps every peer's buffer with ``hipIpcOpenMemHandle`` -- the handles
are exchanged once through the existing c10d process group (TCPStore bootstrap).  The
collectives are HIP kernels in ``csrc/kernels/xgmi_comm.hip`` that read peers' staging slots directly
(system-scope, cache-bypassing loads) after a bounded mesh barrier that ONE workgroup per rank waits in (the
last block of the copy-in kernel; the payload kernels read its published result and never spin):

  * ``all_reduce``   one-shot (<= ``oneshot_max_bytes``: grad-norm / found_inf scalars, loss sync,
                     SyncBN statistics -- latency class) or two-shot (reduce-scatter + all-gather phases:
                     2(W-1)/W of the payload over all 7 links at once -- bandwidth class);
  * ``all_gather`` / ``reduce_scatter`` of flat shards (FSDP units, ZeRO-2 buckets).

Asynchronous like c10d: each collective runs on this rank's dedicated communication stream after an
event wait on the caller's stream, the tensors are ``record_stream``-ed so the caching allocator cannot
recycle them early, and the returned event is what ``Handle.wait()`` makes the *waiting* stream wait on
(no host sync).  FSDP prefetch all-gathers and DDP / ZeRO-2 bucket reductions therefore overlap the GEMMs
of the compute stream.  Payloads larger than a staging slot are chunked (one epoch per chunk); the
kernels address reduce-scatter inputs and all-gather outputs with a per-peer pitch, so a chunk is a
strided window of the caller's tensor (no extra copy).

Failure is loud: a mesh wait longer than ``timeout_us`` (wall clock, s_memrealtime; default 60 s) makes the
kernel poison its output with NaN and set a host-mapped error word; ``raise_if_failed()`` (called by every engine at its end-of-backward and
optimizer sync points through ``Comm.check_errors``) reads that word without synchronising and raises.

``Comm(xgmi=True)`` (or ``PDT_XGMI=1``) routes every eligible CUDA collective here (all_reduce / reduce: fp32,
bf16 or fp64 of any size; all_gather / reduce_scatter: fp32 / bf16 pieces of a multiple of 16 B; world <= 8); ``PDT_XGMI=auto`` routes by SIZE CLASS: payloads in
[``min_bytes``, ``max_bytes``] -- by default the latency class up to 1 MiB (grad-norm / found_inf scalars,
SyncBN statistics, loss sync, small first buckets), where the one-shot mesh kernel is one barrier and one
read of every peer -- go to the mesh, everything else stays on RCCL's pipelined rings
(``PDT_XGMI_MIN_KB`` / ``PDT_XGMI_MAX_KB`` move the window; parity of the default window on a real 8-GPU node
is unpinned: it has only run with several ranks on one GPU).  Ranks must issue collectives in the same order
(the same contract as RCCL); the routing depends only on the payload size, so every rank routes alike.
"""
from __future__ import annotations

import ctypes

import torch

from ..ops import _lib

_KIND = {"allreduce1": 0, "allreduce2": 1, "all_gather": 2, "reduce_scatter": 3, "barrier": 4, "reduce": 5}
SIG_BYTES = 4096
MAX_WORLD = 8


class SizeClass:
    """Which payloads the mesh takes: [min_bytes, max_bytes] (None = unbounded).  Pure function of the size, so
    every rank of a collective routes it the same way."""

    def __init__(self, min_bytes: int = 0, max_bytes: int | None = None):
        if min_bytes < 0 or (max_bytes is not None and max_bytes < min_bytes):
            raise ValueError(f"bad xGMI size class [{min_bytes}, {max_bytes}]")
        self.min_bytes, self.max_bytes = int(min_bytes), max_bytes

    def __call__(self, nbytes: int) -> bool:
        return nbytes > 0 and nbytes >= self.min_bytes and (self.max_bytes is None or nbytes <= self.max_bytes)

    def __repr__(self):
        return f"SizeClass({self.min_bytes}, {self.max_bytes})"


class XGMIComm:
    """Peer-mapped collectives for ``comm``'s ranks (one process per GPU of one node)."""

    def __init__(self, comm, slot_bytes: int = 256 << 20, oneshot_max_bytes: int = 256 << 10,
                 timeout_us: int = 60_000_000, uncached: bool = True, min_bytes: int = 0,
                 max_bytes: int | None = None):
        if comm.world_size > MAX_WORLD:
            raise ValueError(f"XGMIComm spans one node (<= {MAX_WORLD} GPUs), got world_size={comm.world_size}")
        self.comm = comm
        self.rank, self.world = comm.rank, comm.world_size
        self.slot_bytes = int(slot_bytes)
        if not 0 < self.slot_bytes < (1 << 31) or self.slot_bytes % 4096:
            # the kernels address a slot with 32-bit buffer-resource offsets
            raise ValueError(f"xGMI slot_bytes must be a positive multiple of 4 KiB below 2 GiB, got {slot_bytes}")
        self.oneshot_max_bytes = int(oneshot_max_bytes)
        self.size_class = SizeClass(min_bytes, max_bytes)
        self.timeout_us = max(1, min(int(timeout_us), (1 << 32) - 1))
        self.wallclock_khz = int(_lib.require().pdt_xgmi_wallclock_khz())   # s_memrealtime rate (budget unit)
        self.device = torch.device("cuda", torch.cuda.current_device())
        lib = _lib.require()   # ctypes signatures: ops/_lib.py _SIGS (checked against the C sources)
        self._lib = lib
        nbytes = SIG_BYTES + 2 * self.slot_bytes
        own = ctypes.c_void_p()
        _lib.check(lib.pdt_xgmi_alloc(nbytes, 1 if uncached else 0, ctypes.byref(own)), "pdt_xgmi_alloc")
        self._own = own
        hp, dp = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(lib.pdt_xgmi_host_flag_alloc(ctypes.byref(hp), ctypes.byref(dp)), "pdt_xgmi_host_flag_alloc")
        self._host_flag, self._dev_flag = hp, dp
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
        self.calls = 0           # collectives issued through the mesh (tests assert the engines used it)
        # high priority: a collective that peers are spinning on should not queue behind GEMMs
        self.stream = torch.cuda.Stream(device=self.device, priority=-1)
        comm.barrier()

    # ------------------------------------------------------------------ eligibility
    def eligible(self, nbytes: int, kind: str = "all_reduce", dtype=None) -> bool:
        """Payloads inside the size class (larger than a slot: chunked).  all_reduce / reduce: fp32, bf16 or fp64,
        any size (a 4-byte grad-norm scalar, fp64 SyncBN statistics); all_gather / reduce_scatter: fp32 / bf16
        pieces that are a multiple of 16 B."""
        if dtype is not None and dtype not in (torch.float32, torch.bfloat16, torch.float64):
            return False
        if kind in ("all_gather", "reduce_scatter") and (nbytes % 16 or dtype == torch.float64):
            return False
        return self.size_class(nbytes)

    # ------------------------------------------------------------------ launch
    def _run(self, kind: str, inp: int, out: int, nbytes: int, pitch: int, dtype, scale: float):
        self.epoch += 1
        if self.epoch >= 1 << 32:
            self.epoch = 1
        code = _lib.dtype_code(dtype) if dtype is not None else 0
        err = self._lib.pdt_xgmi_collective(_KIND[kind], inp, out, int(nbytes), int(pitch), code, float(scale),
                                            self._bufs, self.rank, self.world, self.epoch, self.slot_bytes,
                                            self.timeout_us, self._dev_flag, self.stream.cuda_stream)
        _lib.check(err, f"pdt_xgmi_collective[{kind}]")

    def _issue(self, tensors, launch, async_op: bool = False) -> torch.cuda.Event:
        """Run ``launch`` on the comm stream after the caller's pending work; return the completion event
        (``async_op=False``: the caller's stream also waits for it -- stream-ordered, no host sync)."""
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        self.calls += 1
        launch()
        for t in tensors:
            t.record_stream(self.stream)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        if not async_op:
            cur.wait_event(ev)
        return ev

    @staticmethod
    def _flat(t):
        if not t.is_contiguous():
            raise ValueError("xGMI collectives need contiguous tensors")
        return t.view(-1)

    def _two_shot_chunk(self) -> int:
        q = 16 * self.world
        return (self.slot_bytes // q) * q

    def all_reduce(self, t: torch.Tensor, op: str = "sum", async_op: bool = False) -> torch.cuda.Event:
        """In place: sum / avg over ranks.  fp32 or bf16 (fp32 accumulation).  Returns the completion event."""
        if op not in ("sum", "avg"):
            raise ValueError(f"xGMI all_reduce supports sum/avg, got {op}")
        t = self._flat(t)
        nbytes = t.numel() * t.element_size()
        if not self.eligible(nbytes, "all_reduce", t.dtype):
            raise ValueError(f"xGMI all_reduce: {nbytes} B of {t.dtype} not eligible")
        scale = 1.0 / self.world if op == "avg" else 1.0
        base = t.data_ptr()

        def launch():
            if nbytes <= self.oneshot_max_bytes or t.dtype == torch.float64:
                for o in range(0, nbytes, self.slot_bytes):     # fp64: one-shot windows (no two-shot kernels)
                    self._run("allreduce1", base + o, base + o, min(self.slot_bytes, nbytes - o), 0, t.dtype, scale)
                return
            q = 16 * self.world
            main = (nbytes // q) * q
            step = self._two_shot_chunk()
            for o in range(0, main, step):
                c = min(step, main - o)
                self._run("allreduce2", base + o, base + o, c, 0, t.dtype, scale)
            if main < nbytes:    # < 16 * world bytes left: latency-class one-shot (any size)
                self._run("allreduce1", base + main, base + main, nbytes - main, 0, t.dtype, scale)
        return self._issue([t], launch, async_op)

    def reduce(self, t: torch.Tensor, dst: int, op: str = "sum", async_op: bool = False) -> torch.cuda.Event:
        """In place on ``dst`` (ZeRO-2 reduce-to-owner): the owner reads every peer's slot, the others only
        stage their contribution.  Other ranks' ``t`` is left unchanged."""
        if op not in ("sum", "avg"):
            raise ValueError(f"xGMI reduce supports sum/avg, got {op}")
        t = self._flat(t)
        nbytes = t.numel() * t.element_size()
        if not self.eligible(nbytes, "reduce", t.dtype) or not 0 <= dst < self.world:
            raise ValueError(f"xGMI reduce: {nbytes} B / dst {dst} not eligible")
        scale = 1.0 / self.world if op == "avg" else 1.0
        base = t.data_ptr()

        def launch():
            for o in range(0, nbytes, self.slot_bytes):
                c = min(self.slot_bytes, nbytes - o)
                self._run("reduce", base + o, base + o, c, 16 * dst, t.dtype, scale)
        return self._issue([t], launch, async_op)

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False) -> torch.cuda.Event:
        inp, out = self._flat(inp), self._flat(out)
        nbytes = inp.numel() * inp.element_size()
        if (out.numel() != inp.numel() * self.world or out.dtype != inp.dtype
                or not self.eligible(nbytes, "all_gather", inp.dtype)):
            raise ValueError("xGMI all_gather: bad sizes")
        src, dst = inp.data_ptr(), out.data_ptr()

        def launch():
            for o in range(0, nbytes, self.slot_bytes):
                c = min(self.slot_bytes, nbytes - o)
                self._run("all_gather", src + o, dst + o, c, nbytes, inp.dtype, 1.0)
        return self._issue([inp, out], launch, async_op)

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum",
                       async_op: bool = False) -> torch.cuda.Event:
        inp, out = self._flat(inp), self._flat(out)
        nbytes = out.numel() * out.element_size()          # one rank's piece
        if (inp.numel() != out.numel() * self.world or out.dtype != inp.dtype
                or not self.eligible(nbytes, "reduce_scatter", inp.dtype)):
            raise ValueError("xGMI reduce_scatter: bad sizes")
        scale = 1.0 / self.world if op == "avg" else 1.0
        src, dst = inp.data_ptr(), out.data_ptr()
        step = (self.slot_bytes // self.world) // 16 * 16

        def launch():
            for o in range(0, nbytes, step):
                c = min(step, nbytes - o)
                self._run("reduce_scatter", src + o, dst + o, c, nbytes, inp.dtype, scale)
        return self._issue([inp, out], launch, async_op)

    def barrier(self) -> torch.cuda.Event:
        return self._issue([], lambda: self._run("barrier", 0, 0, 0, 0, None, 1.0), False)

    # ------------------------------------------------------------------ failure detection
    def failed(self) -> int:
        """Timeout bits recorded by the kernels so far (host-mapped word: no device sync)."""
        return ctypes.c_uint.from_address(self._host_flag.value).value

    def diagnosis(self) -> dict:
        """What the last timed-out wait saw: the epoch it waited for, the barrier, the late peer and that
        peer's last signalled epoch (host-mapped words written by the kernel; no device sync)."""
        w = (ctypes.c_uint * 4).from_address(self._host_flag.value)
        return {"flag": w[0], "epoch": w[1], "barrier": w[2] >> 8, "peer": w[2] & 0xFF, "peer_epoch": w[3],
                "issued_epoch": self.epoch}

    def raise_if_failed(self):
        v = self.failed()
        if v:
            d = self.diagnosis()
            raise RuntimeError(f"xGMI collective timed out on rank {self.rank} (flag {v:#x}): a peer did not reach "
                               f"the same collective in time; its outputs were poisoned with NaN -- waited at "
                               f"barrier {d['barrier']} for epoch {d['epoch']}, peer {d['peer']} had signalled "
                               f"{d['peer_epoch']}; this rank has issued up to epoch {d['issued_epoch']}")

    def check(self):
        """Synchronise the comm stream, then raise if any mesh wait timed out (tests / teardown)."""
        self.stream.synchronize()
        v = ctypes.c_uint(0)
        _lib.check(self._lib.pdt_xgmi_error(self._own, ctypes.byref(v)), "pdt_xgmi_error")
        if v.value:
            raise RuntimeError(f"xGMI collective timed out on rank {self.rank} (barrier bits {v.value:#x}): "
                               "a peer did not reach the same collective")
        self.raise_if_failed()

    def close(self):
        if getattr(self, "_own", None) is None:
            return
        torch.cuda.synchronize(self.device)
        self.comm.barrier()          # no peer may still read our buffer
        for q in self._opened:
            self._lib.pdt_xgmi_ipc_close(q)
        self._opened = []
        self._lib.pdt_xgmi_free(self._own)
        self._lib.pdt_xgmi_host_flag_free(self._host_flag)
        self._own = None
