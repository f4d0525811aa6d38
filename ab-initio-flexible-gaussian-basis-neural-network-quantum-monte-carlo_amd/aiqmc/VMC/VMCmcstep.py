"""Drift-diffusion Metropolis step (drop-in for AIQMCrelease3/VMC/VMCmcstep.py).

``main_monte_carlo(f, tstep, ndim, nelectrons, nsteps, batch_size)`` returns
``mc_step(params, data, key) -> data`` (VMCmcstep.py:121-140).  Each of the
``nsteps`` updates (walkers_update, :28-111) is five stream-ordered launches:
gradient at the walkers, device-batch limdrift reduction, value+gradient at the
B*N single-electron proposals, the second limdrift reduction, acceptance.

``key`` selects the random draws:
  * ``PhiloxKey(seed, offset)`` or a plain int seed: on-device Philox4x32-10;
  * ``HostDraws(gauss1, gauss2, u)``: caller-supplied draws (parity mode, Q7),
    shapes [nsteps,B,3N], [nsteps,B,N,3N] (the reference's shape; only the
    electron-diagonal 3-blocks are read) or [nsteps,B,N,3], and [nsteps,B,N].
``batch_size`` is the per-device walker count; limdrift's v2 is reduced over
exactly those walkers (Q8).  Positions are updated in place when they already
are a contiguous device tensor of the compute dtype (donate_argnums analogue).
"""
from __future__ import annotations

import dataclasses
from typing import Union

import numpy as np
import torch

from ..wavefunction_Ynlm.nn import AINetData


def limdrift(g: torch.Tensor, tau: float, acyrus: float) -> torch.Tensor:
    """VMCmcstep.py:11-14 (v2 summed over ALL entries of g)."""
    v2 = torch.sum(g ** 2)
    taueff = (torch.sqrt(1 + 2 * tau * acyrus * v2) - 1) / (acyrus * v2)
    return g * taueff


@dataclasses.dataclass
class PhiloxKey:
    seed: int = 0
    offset: int = 0


@dataclasses.dataclass
class HostDraws:
    gauss1: torch.Tensor
    gauss2: torch.Tensor
    u: torch.Tensor


def diag_gauss2(gauss2: torch.Tensor, nelectrons: int) -> torch.Tensor:
    """[..., N, 3N] -> [..., N, 3]: the blocks the reference reads (VMCmcstep.py:87-94)."""
    if gauss2.shape[-1] == 3:
        return gauss2
    n = nelectrons
    g = gauss2.reshape(*gauss2.shape[:-2], n, n, 3)
    idx = torch.arange(n, device=g.device)
    return g[..., idx, idx, :]


def main_monte_carlo(f, tstep: float, ndim: int, nelectrons: int, nsteps: int, batch_size: int):
    net = getattr(f, "_aiqmc_network", None)
    if net is None:
        raise TypeError("main_monte_carlo: f must be the apply function of an aiqmc make_ai_net Network")
    if ndim != 3 or nelectrons != net.nelectrons:
        raise ValueError("ndim/nelectrons do not match the network")

    def mc_step(params, data: AINetData, key: Union[int, PhiloxKey, HostDraws] = 0) -> AINetData:
        pos = data.positions if isinstance(data.positions, torch.Tensor) else torch.as_tensor(
            np.asarray(data.positions))
        dtype = pos.dtype if pos.dtype in (torch.float32, torch.float64) else torch.float32
        ctx = net.bind(params, data.atoms, dtype)
        shape = pos.shape
        p = pos.reshape(-1, 3 * nelectrons)
        if p.shape[0] != batch_size:
            raise ValueError(f"expected {batch_size} walkers per device, got {p.shape[0]}")
        inplace = p.is_cuda and p.dtype == dtype and p.is_contiguous() and p.device == ctx.device
        work = p if inplace else p.to(ctx.device, dtype).contiguous()
        if isinstance(key, HostDraws):
            g2 = diag_gauss2(torch.as_tensor(key.gauss2), nelectrons)
            ctx.mc_step(work, nsteps, tstep, gauss1=torch.as_tensor(key.gauss1), gauss2=g2,
                        u=torch.as_tensor(key.u))
        else:
            k = key if isinstance(key, PhiloxKey) else PhiloxKey(int(key), 0)
            ctx.mc_step(work, nsteps, tstep, seed=k.seed, offset=k.offset)
        out = work.reshape(shape) if inplace else work.to(pos.device, pos.dtype).reshape(shape)
        return AINetData(positions=out, spins=data.spins, atoms=data.atoms, charges=data.charges)

    return mc_step
