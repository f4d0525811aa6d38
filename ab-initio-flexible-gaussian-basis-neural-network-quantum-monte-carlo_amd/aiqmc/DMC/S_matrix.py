"""DMC S factor (drop-in for AIQMCrelease3/DMC/S_matrix.py:4-24), on device tensors.

Quirk kept: e_cut = min(|e_est - eloc| over the WHOLE batch and branchcut) * sign(e_est - eloc)
(jnp.min over the stacked array).  The fused weight update used by dmc_propagate runs in the
HIP kernel of aiqmc_dmc_weights."""
from __future__ import annotations

import torch


def comput_S(e_trial, e_est, branchcut, v2: torch.Tensor, tau: float, eloc: torch.Tensor, nelec: int):
    v2 = torch.sum(v2, dim=-1)
    eloc = eloc.real if torch.is_complex(eloc) else eloc
    e_est = float(e_est.real if isinstance(e_est, complex) else e_est)
    e_trial = float(e_trial.real if isinstance(e_trial, complex) else e_trial)
    e_cut = e_est - eloc
    bc = torch.as_tensor(branchcut, dtype=e_cut.dtype, device=e_cut.device).reshape(-1)
    cut = torch.min(torch.cat([torch.abs(e_cut).reshape(-1), bc]))
    return e_trial - e_est + cut * torch.sign(e_cut) / (1 + (v2 * tau / nelec) ** 2)
