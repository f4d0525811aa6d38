"""Weighted DMC energy estimate (drop-in for AIQMCrelease3/DMC/estimate_energy.py:4-5):
jnp.average(energy, weights=weights) over all axes."""
from __future__ import annotations

import torch


def estimate_energy(energy: torch.Tensor, weights: torch.Tensor) -> torch.Tensor:
    e = torch.as_tensor(energy)
    w = torch.as_tensor(weights, device=e.device).to(e.real.dtype if e.is_complex() else e.dtype)
    return (e * w).sum() / w.sum()
