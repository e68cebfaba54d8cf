"""Data pipeline: distributed sampling, rank-consistent splits, device prefetching, synthetic data."""
from .datasets import CustomDataset, PairedImageDataset
from .loader import DeviceDataLoader, to_device
from .sampler import DistributedSampler, random_split
from .synthetic import SyntheticImageDataset, SyntheticSRDataset, SyntheticTokenDataset

__all__ = ["CustomDataset", "PairedImageDataset", "DeviceDataLoader", "to_device", "DistributedSampler",
           "random_split", "SyntheticImageDataset", "SyntheticSRDataset", "SyntheticTokenDataset"]
