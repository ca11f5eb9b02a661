"""torchOptics.metrics -- the metric the reference imports as ``tm`` (env.py:25).

get_PSNR(x, y) = 10 log10(peak^2 / mean((x - y)^2)), peak 1 (the reference
always passes intensities scaled by tt.relativeLoss against [0, 1] targets).
Returns a Python float: the reference only compares, subtracts and formats it
(env.py:184-214, DBS_1024_24.py:355-378)."""
from __future__ import annotations

import math

import torch

__all__ = ["get_PSNR", "get_MSE"]


def get_MSE(x: torch.Tensor, y: torch.Tensor) -> float:
    d = x.double() - y.double()
    return float(torch.mean(d * d).item())


def get_PSNR(x: torch.Tensor, y: torch.Tensor, peak: float = 1.0) -> float:
    mse = get_MSE(x, y)
    return float("inf") if mse <= 0 else 10.0 * math.log10(peak * peak / mse)
