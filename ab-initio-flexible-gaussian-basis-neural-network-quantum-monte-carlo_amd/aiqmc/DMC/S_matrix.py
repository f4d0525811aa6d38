"""DMC S factor (drop-in for AIQMCrelease3/DMC/S_matrix.py:4-24), on device tensors.

Quirk kept: e_cut = min(|e_est - eloc| over the WHOLE batch and branchcut) * sign(e_est - eloc)
(jnp.min over the stacked array).  ``e_trial`` / ``e_est`` may be scalars or per-walker arrays
(the first DMC block passes the per-walker total_e energies, main_dmc.py:115-124); ``branchcut``
likewise.  The fused weight update used by dmc_propagate runs in the HIP kernel of
aiqmc_dmc_weights."""
from __future__ import annotations

import torch


def _real(x, like: torch.Tensor) -> torch.Tensor:
    """jnp.real of a Python/NumPy scalar or array, or a tensor, on eloc's device and dtype."""
    if isinstance(x, complex):
        x = x.real
    if isinstance(x, (int, float)):
        return torch.tensor(float(x), dtype=like.dtype, device=like.device)
    t = torch.as_tensor(x, device=like.device)
    if torch.is_complex(t):
        t = t.real
    return t.to(like.dtype)


def comput_S(e_trial, e_est, branchcut, v2: torch.Tensor, tau: float, eloc: torch.Tensor, nelec: int):
    v2 = torch.sum(v2, dim=-1)
    eloc = eloc.real if torch.is_complex(eloc) else eloc
    e_est = _real(e_est, eloc)
    e_trial = _real(e_trial, eloc)
    e_cut = e_est - eloc
    bc = torch.as_tensor(branchcut, dtype=e_cut.dtype, device=e_cut.device).reshape(-1)
    cut = torch.min(torch.cat([torch.abs(e_cut).reshape(-1), bc]))
    return e_trial - e_est + cut * torch.sign(e_cut) / (1 + (v2 * tau / nelec) ** 2)
