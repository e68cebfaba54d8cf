"""File-backed paired-image dataset (the reference's missing ``old_dataset.CustomDataset``,
SURVEY.md F2: ``CustomDataset(input_dir, target_dir)`` -> (input, target) float tensors from matching
LR/HR patch files, Fairscale-DDP.py:37 / Stoke-DDP.py:264).  Truncated images are tolerated like the
reference's ``ImageFile.LOAD_TRUNCATED_IMAGES = True`` (Fairscale-DDP.py:11-12)."""
from __future__ import annotations

import os

import numpy as np
import torch
from torch.utils.data import Dataset

_EXT = (".png", ".jpg", ".jpeg", ".bmp", ".tif", ".tiff", ".webp")


class PairedImageDataset(Dataset):
    def __init__(self, input_dir: str, target_dir: str, transform=None):
        from PIL import ImageFile

        ImageFile.LOAD_TRUNCATED_IMAGES = True
        self.input_dir, self.target_dir, self.transform = input_dir, target_dir, transform
        names = sorted(f for f in os.listdir(input_dir) if f.lower().endswith(_EXT))
        self.names = [f for f in names if os.path.exists(os.path.join(target_dir, f))]
        if not self.names:
            raise FileNotFoundError(f"no paired images in {input_dir} / {target_dir}")

    def __len__(self):
        return len(self.names)

    @staticmethod
    def _load(path):
        from PIL import Image

        with Image.open(path) as im:
            a = np.asarray(im.convert("RGB"), dtype=np.float32) / 255.0
        return torch.from_numpy(a).permute(2, 0, 1).contiguous()

    def __getitem__(self, i):
        n = self.names[i]
        x = self._load(os.path.join(self.input_dir, n))
        y = self._load(os.path.join(self.target_dir, n))
        if self.transform is not None:
            x, y = self.transform(x, y)
        return x, y


CustomDataset = PairedImageDataset
