"""Image-restoration metrics used by the reference's validate() (Stoke-DDP.py:120-121; module ``metrics``
absent from the reference): MAE = mean|x - y|, PSNR = 10 log10(range^2 / MSE) for
``img_range=1.`` images.  Returned as Python floats (the reference sums them per batch)."""
import math

import torch


def mae(outputs: torch.Tensor, targets: torch.Tensor) -> float:
    return float((outputs.detach().float() - targets.detach().float()).abs().mean())


def psnr(outputs: torch.Tensor, targets: torch.Tensor, data_range: float = 1.0) -> float:
    mse = float((outputs.detach().float().clamp(0, data_range) - targets.detach().float()).pow(2).mean())
    return float("inf") if mse == 0 else 10.0 * math.log10(data_range ** 2 / mse)
