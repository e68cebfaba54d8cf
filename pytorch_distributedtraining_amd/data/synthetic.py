"""Synthetic datasets (no network access: every benchmark and example runs on generated data).

* ``SyntheticSRDataset``   -- paired (LR, HR) images like the reference's Flickr2K / DIV2K patches
                              (Fairscale-DDP.py:32-33: 3x256x256 -> 3x512x512; Stoke-DDP.py:169-170:
                              3x128x128 -> 3x256x256); HR is a smooth random field, LR its bicubic downsample,
                              so super-resolution is learnable.
* ``SyntheticImageDataset`` -- ImageNet-shaped classification samples (ResNet configs).
* ``SyntheticTokenDataset`` -- LM token sequences (GPT-2 / Llama configs).
All are deterministic functions of (seed, index) so every rank / worker sees identical samples.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch.utils.data import Dataset


class SyntheticSRDataset(Dataset):
    def __init__(self, n: int = 256, lr_size: int = 128, scale: int = 2, channels: int = 3, seed: int = 0):
        self.n, self.lr, self.scale, self.c, self.seed = n, lr_size, scale, channels, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        hr_size = self.lr * self.scale
        base = torch.rand(1, self.c, hr_size // 8, hr_size // 8, generator=g)
        hr = F.interpolate(base, size=(hr_size, hr_size), mode="bicubic", align_corners=False).clamp(0, 1)
        lr = F.interpolate(hr, size=(self.lr, self.lr), mode="bicubic", align_corners=False).clamp(0, 1)
        return lr[0], hr[0]


class SyntheticImageDataset(Dataset):
    def __init__(self, n: int = 1024, size: int = 224, num_classes: int = 1000, seed: int = 0):
        self.n, self.size, self.k, self.seed = n, size, num_classes, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        y = int(torch.randint(0, self.k, (1,), generator=g))
        x = torch.randn(3, self.size, self.size, generator=g) * 0.5 + (y % 7) / 7.0
        return x, y


class SyntheticTokenDataset(Dataset):
    def __init__(self, n: int = 1024, seq_len: int = 1024, vocab: int = 50257, seed: int = 0):
        self.n, self.s, self.v, self.seed = n, seq_len, vocab, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        t = torch.randint(0, self.v, (self.s + 1,), generator=g)
        return t[:-1], t[1:]
