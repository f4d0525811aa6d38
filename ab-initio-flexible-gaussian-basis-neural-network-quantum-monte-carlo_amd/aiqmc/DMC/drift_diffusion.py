"""DMC drift-diffusion (drop-in for AIQMCrelease3/DMC/drift_diffusion.py:25-107).

``propose_drift_diffusion(logabs_f, tstep, ndim, nelectrons, batch_size)`` returns
``drift_diffusion(params, key, data) -> (new_data, key, tdamp, grad_eff_old, grad_new_eff_s)``.
One HIP sweep (aiqmc_dmc_drift_diffusion): the VMC one-electron-move Metropolis step (same
draws and quirks) plus tdamp = sum(x_new)/sum(x_proposed) and the limdrift'ed gradients at
the old and new positions.  key: PhiloxKey / int seed, or VMCmcstep.HostDraws (parity mode).
"""
from __future__ import annotations

import numpy as np
import torch

from ..VMC.VMCmcstep import HostDraws, PhiloxKey, diag_gauss2
from ..wavefunction_Ynlm.nn import AINetData


def propose_drift_diffusion(logabs_f, tstep: float, ndim: int, nelectrons: int, batch_size: int):
    net = getattr(logabs_f, "_aiqmc_network", None)
    if net is None:
        raise TypeError("propose_drift_diffusion: logabs_f must come from an aiqmc make_ai_net Network")
    if ndim != 3 or nelectrons != net.nelectrons:
        raise ValueError("ndim/nelectrons do not match the network")

    def drift_diffusion(params, key, data: AINetData):
        pos = data.positions if isinstance(data.positions, torch.Tensor) else torch.as_tensor(
            np.asarray(data.positions))
        dtype = pos.dtype if pos.dtype in (torch.float32, torch.float64) else torch.float32
        ctx = net.bind(params, data.atoms, dtype)
        p = pos.reshape(-1, 3 * nelectrons)
        if p.shape[0] != batch_size:
            raise ValueError(f"expected {batch_size} walkers per device, got {p.shape[0]}")
        work = p.to(ctx.device, dtype).contiguous().clone()
        if isinstance(key, HostDraws):
            g1 = torch.as_tensor(key.gauss1).reshape(1, batch_size, -1)
            g2 = diag_gauss2(torch.as_tensor(key.gauss2), nelectrons).reshape(1, batch_size, nelectrons, 3)
            go, gn, td = ctx.dmc_drift_diffusion(work, tstep, gauss1=g1, gauss2=g2,
                                                 u=torch.as_tensor(key.u).reshape(1, batch_size, -1))
            newkey = key
        else:
            k = key if isinstance(key, PhiloxKey) else PhiloxKey(int(key), 0)
            go, gn, td = ctx.dmc_drift_diffusion(work, tstep, seed=k.seed, offset=k.offset)
            newkey = PhiloxKey(k.seed, k.offset + 1)
        new = AINetData(positions=work.reshape(pos.shape), spins=data.spins, atoms=data.atoms, charges=data.charges)
        return new, newkey, td[2], go, gn

    return drift_diffusion
