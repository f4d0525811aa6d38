"""Stochastic comb (drop-in for AIQMCrelease3/DMC/branch.py:10-33) on the GPU (aiqmc_dmc_branch).

``branch(data, weights, key)`` -> (weights, newinds): newinds = searchsorted(cumsum(w),
(u wtot + linspace(0, wtot, n, endpoint=False)) % wtot), weights -> wtot / n.  ``key`` is the
uniform draw u in [0, 1) (parity mode) or an int seed for numpy's generator.  The driver's
re-indexing of the positions (main_dmc.py:208-242: unique() plus ad-hoc extra walkers) is
``DMC.main_dmc.reindex_walkers``; ``apply_branch`` is the plain comb gather x[newinds]."""
from __future__ import annotations

import numpy as np
import torch

from ..Energy.hamiltonian import _network_of


def branch(data, weights: torch.Tensor, key, network=None, params=None):
    u = float(key) if isinstance(key, float) else float(np.random.default_rng(int(key)).uniform())
    net = _network_of(network) if network is not None else None
    if net is None:
        raise TypeError("branch needs the aiqmc network (network=apply function) for its HIP context")
    ctx = net.context(data.atoms, weights.dtype if weights.dtype in (torch.float32, torch.float64) else torch.float32)
    w, idx = ctx.dmc_branch(weights, u)
    return w, idx


def apply_branch(positions: torch.Tensor, newinds: torch.Tensor) -> torch.Tensor:
    return positions.reshape(positions.shape[0], -1)[newinds.long()].reshape(positions.shape)
