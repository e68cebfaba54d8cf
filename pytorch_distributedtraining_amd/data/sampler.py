"""Distributed sampling and rank-consistent dataset splitting.

``DistributedSampler`` reproduces torch/utils/data/distributed.py:107-134 (shuffle with seed+epoch,
pad by repetition to ceil(N/R)*R or drop the tail, strided ``indices[rank::R]``) -- the sampler the
reference builds in Fairscale-DDP.py:45-55 and Stoke-DDP.py:272-283 -- with world size / rank taken
from the process group when not given (the reference hard-codes num_replicas=4).

``random_split`` fixes the reference quirk B12: an unseeded torch.utils.data.random_split
gives every rank a DIFFERENT train/val split (torch 2.10 seeds processes differently), so validation
samples leak into other ranks' training data.  Here the permutation comes from a generator seeded
identically on every rank.
"""
from __future__ import annotations

import math
from typing import Iterator, Optional, Sequence

import torch
import torch.distributed as dist
from torch.utils.data import Dataset, Sampler, Subset


class DistributedSampler(Sampler[int]):
    def __init__(self, dataset, num_replicas: Optional[int] = None, rank: Optional[int] = None,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False):
        if num_replicas is None:
            num_replicas = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        if rank is None:
            rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"invalid rank {rank} for num_replicas {num_replicas}")
        self.dataset, self.num_replicas, self.rank = dataset, num_replicas, rank
        self.shuffle, self.seed, self.drop_last, self.epoch = shuffle, seed, drop_last, 0
        n = len(dataset)
        if drop_last and n % num_replicas:
            self.num_samples = math.ceil((n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def __iter__(self) -> Iterator[int]:
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            indices = torch.randperm(n, generator=g).tolist()
        else:
            indices = list(range(n))
        if not self.drop_last:
            pad = self.total_size - len(indices)
            if pad > 0:
                if pad <= len(indices):
                    indices += indices[:pad]
                else:
                    indices += (indices * math.ceil(pad / len(indices)))[:pad]
        else:
            indices = indices[: self.total_size]
        assert len(indices) == self.total_size
        return iter(indices[self.rank:self.total_size:self.num_replicas])

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch


def random_split(dataset: Dataset, lengths: Sequence[float], seed: int = 0):
    """Split identically on every rank (fractions or absolute lengths)."""
    n = len(dataset)
    if all(0 <= x <= 1 for x in lengths) and abs(sum(lengths) - 1) < 1e-6 and not all(isinstance(x, int) for x in lengths):
        sizes = [int(math.floor(n * f)) for f in lengths]
        for i in range(n - sum(sizes)):
            sizes[i % len(sizes)] += 1
    else:
        sizes = [int(x) for x in lengths]
    if sum(sizes) != n:
        raise ValueError("sum of split lengths must equal the dataset length")
    g = torch.Generator()
    g.manual_seed(seed)
    perm = torch.randperm(n, generator=g).tolist()
    out, off = [], 0
    for s in sizes:
        out.append(Subset(dataset, perm[off:off + s]))
        off += s
    return out
