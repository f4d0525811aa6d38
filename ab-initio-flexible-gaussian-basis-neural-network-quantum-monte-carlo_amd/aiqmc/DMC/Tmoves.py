"""T-moves (drop-in for AIQMCrelease3/DMC/Tmoves.py:32-225).

``compute_tmoves(list_l, tstep, nelectrons, natoms, ndim, lognetwork, Rn_non_local,
Non_local_coes, Non_local_exps)`` returns ``calculate_ratio_weight_tmoves(data, params, key)
-> (positions, acceptance)``.  The reference function handles one walker and is vmapped by
dmc.py:42-43; this one takes the device batch data.positions [B, 3N] and returns the new
positions [B, 3N] and the acceptance [B, N] (the reference's per-walker [N, 1]).

The whole batch runs on the GPU (aiqmc_dmc_tmoves): the pp quadrature configurations of every
electron through the walker cache (the machinery of aiqmc_local_energy_ecp), then one wave per
walker for amplitudes, the cdf / searchsorted selection and the acceptance, with the
reference's quirks T1-T8 (oracle/dmc.py).

``key``: ``HostTmoveDraws(rot[B,3,3], u_sel[B], u_acc[B,N])`` injects the draws (parity mode;
the reference shares ONE device key across the vmapped walkers, so a faithful replay passes
the same rotation and uniforms for every walker), a ``PhiloxKey`` / int seed draws them per
walker on the device.  ``lognetwork`` must carry the aiqmc network (``nn.make_log_network``
or any function with an ``_aiqmc_network`` attribute); it is not called.
"""
from __future__ import annotations

import dataclasses
from typing import Union

import numpy as np
import torch

from ..VMC.VMCmcstep import PhiloxKey
from ..wavefunction_Ynlm.nn import AINetData


@dataclasses.dataclass
class HostTmoveDraws:
    rot: torch.Tensor     # [B, 3, 3] get_rot's matrix (Tmoves.py:70)
    u_sel: torch.Tensor   # [B] select_walker's uniform (:146)
    u_acc: torch.Tensor   # [B, N] acceptance uniforms (:216-217)


def _np64(t):
    return np.asarray(t.detach().cpu() if isinstance(t, torch.Tensor) else t, dtype=np.float64)


def attach_nonlocal(ctx, natoms: int, list_l: int, rn_non_local, non_local_coes, non_local_exps):
    """Give `ctx` the nonlocal tables unless its pp tables already hold the same ones."""
    nl = tuple(_np64(t) for t in (rn_non_local, non_local_coes, non_local_exps))
    if nl[0].reshape(natoms, -1).shape[1] % (int(list_l) + 1):
        raise ValueError("non-local tables must have list_l + 1 angular channels per atom")
    tok = getattr(ctx, "_ecp_token", None)
    want = (int(list_l),) + tuple(t.tobytes() for t in nl)
    if tok is not None and (tok[0],) + tok[4:] == want:
        return
    zero = np.zeros((natoms, 1))
    ctx.set_ecp(zero, zero, zero + 1.0, *nl, list_l=int(list_l))   # local part unused by T-moves
    ctx._ecp_token = (int(list_l),) + tuple(t.tobytes() for t in (zero, zero, zero + 1.0)) + want[1:]


def compute_tmoves(list_l: int, tstep: float, nelectrons: int, natoms: int, ndim: int, lognetwork,
                   Rn_non_local, Non_local_coes, Non_local_exps):
    net = getattr(lognetwork, "_aiqmc_network", None)
    if net is None:
        raise TypeError("compute_tmoves: lognetwork must carry an aiqmc make_ai_net Network "
                        "(use aiqmc.wavefunction_Ynlm.nn.make_log_network)")
    if ndim != 3 or nelectrons != net.nelectrons or natoms != net.natoms:
        raise ValueError("ndim / nelectrons / natoms do not match the network")
    if not tstep > 0:
        raise ValueError("tstep must be > 0")

    def calculate_ratio_weight_tmoves(data: AINetData, params, key: Union[int, PhiloxKey, HostTmoveDraws]):
        pos = data.positions if isinstance(data.positions, torch.Tensor) else torch.as_tensor(
            np.asarray(data.positions))
        dtype = pos.dtype if pos.dtype in (torch.float32, torch.float64) else torch.float32
        ctx = net.bind(params, data.atoms, dtype)
        attach_nonlocal(ctx, natoms, list_l, Rn_non_local, Non_local_coes, Non_local_exps)
        work = pos.reshape(-1, 3 * nelectrons).to(ctx.device, dtype).contiguous().clone()
        if isinstance(key, HostTmoveDraws):
            acc = ctx.dmc_tmoves(work, tstep, rot=key.rot, u_sel=key.u_sel, u_acc=key.u_acc)
        else:
            k = key if isinstance(key, PhiloxKey) else PhiloxKey(int(key or 0), 0)
            acc = ctx.dmc_tmoves(work, tstep, seed=k.seed, offset=k.offset)
        return work.reshape(pos.shape), acc

    calculate_ratio_weight_tmoves._aiqmc_network = net
    return calculate_ratio_weight_tmoves
