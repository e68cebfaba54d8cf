"""Device-prefetching DataLoader (the facade's ``DataLoader``).

Wraps torch.utils.data.DataLoader (worker processes, pinned host memory) and moves every (nested)
batch to the rank's GPU on a dedicated HIP copy stream one batch AHEAD of the consumer, so the H2D
copy of batch i+1 overlaps compute on batch i; the compute stream waits on an event, never on the host.
Reference: stoke_model.DataLoader(dataset, sampler, num_workers, multiprocessing_context='spawn')
(Stoke-DDP.py:286-298) -- batch size comes from ``batch_size_per_device``.
"""
from __future__ import annotations

import torch
from torch.utils.data import DataLoader as _TorchLoader


def to_device(batch, device, non_blocking=True, dtype=None):
    if torch.is_tensor(batch):
        t = batch.to(device, non_blocking=non_blocking)
        if dtype is not None and t.is_floating_point():
            t = t.to(dtype)
        return t
    if isinstance(batch, (list, tuple)):
        out = [to_device(b, device, non_blocking, dtype) for b in batch]
        return type(batch)(out) if isinstance(batch, tuple) and not hasattr(batch, "_fields") else out
    if isinstance(batch, dict):
        return {k: to_device(v, device, non_blocking, dtype) for k, v in batch.items()}
    return batch


class DeviceDataLoader:
    def __init__(self, dataset, batch_size: int, device=None, sampler=None, num_workers: int = 0,
                 pin_memory: bool | None = None, drop_last: bool = False, prefetch: bool = True,
                 cast_dtype=None, **kwargs):
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        if pin_memory is None:
            pin_memory = self.device.type == "cuda"
        if num_workers == 0:
            kwargs.pop("multiprocessing_context", None)
            kwargs.pop("persistent_workers", None)
            kwargs.pop("prefetch_factor", None)
        self.loader = _TorchLoader(dataset, batch_size=batch_size, sampler=sampler, num_workers=num_workers,
                                   pin_memory=pin_memory, drop_last=drop_last, **kwargs)
        self.prefetch = prefetch and self.device.type == "cuda"
        self.cast_dtype = cast_dtype
        self.sampler = sampler
        self.dataset = dataset

    def __len__(self):
        return len(self.loader)

    def set_epoch(self, epoch: int):
        if hasattr(self.sampler, "set_epoch"):
            self.sampler.set_epoch(epoch)

    def __iter__(self):
        if not self.prefetch:
            for b in self.loader:
                yield to_device(b, self.device, True, self.cast_dtype)
            return
        stream = torch.cuda.Stream(device=self.device)
        it = iter(self.loader)
        nxt, ev = self._stage(it, stream)
        while nxt is not None:
            cur, cur_ev = nxt, ev
            nxt, ev = self._stage(it, stream)
            torch.cuda.current_stream(self.device).wait_event(cur_ev)
            _record(cur, torch.cuda.current_stream(self.device))
            yield cur

    def _stage(self, it, stream):
        try:
            b = next(it)
        except StopIteration:
            return None, None
        with torch.cuda.stream(stream):
            d = to_device(b, self.device, True, self.cast_dtype)
            ev = torch.cuda.Event()
            ev.record(stream)
        return d, ev


def _record(batch, stream):
    if torch.is_tensor(batch):
        batch.record_stream(stream)
    elif isinstance(batch, (list, tuple)):
        for b in batch:
            _record(b, stream)
    elif isinstance(batch, dict):
        for b in batch.values():
            _record(b, stream)
