"""One DMC propagation step (drop-in for AIQMCrelease3/DMC/dmc.py:13-93).

``dmc_propagate(signed_network, log_network, logabs_f, list_l, nelectrons, natoms, ndim,
batch_size, tstep, nsteps, charges, spins, Rn_local, ...)`` returns
``dmc_propagate_run(params, key, data, weights, branchcut_start, e_trial, e_est) ->
(eloc_new, weights, new_data)``, in the reference's order (dmc.py:79-93): T-moves
(aiqmc_dmc_tmoves, DMC/Tmoves.py with its quirks T1-T8), drift-diffusion of the T-moved
walkers (aiqmc_dmc_drift_diffusion), the complex pseudopotential local energies of the
walkers before the T-moves and after the drift-diffusion (aiqmc_local_energy_ecp), and the
weight update with the S factors (aiqmc_dmc_weights_ex).  Every stage is a batched GPU launch
sequence; the draws come from one PhiloxKey per call (the reference reuses one device key for
all stages and walkers; threefry bits are out of scope).

``e_trial`` / ``e_est`` are scalars or per-walker [B] arrays: the driver's first block passes
the per-walker pp energies (main_dmc.py:115-116), later blocks the scalar estimate.  comput_S's
energy cut is ONE jnp.min over the stacked arrays of every device (S_matrix.py:21-22): with
more than one rank the per-rank minima are all-reduced with MIN (RCCL) before the update.
"""
from __future__ import annotations

import dataclasses

import torch
import torch.distributed as dist

from ..Energy import pphamiltonian
from ..Energy.pphamiltonian import HostRotations
from ..VMC.VMCmcstep import HostDraws, PhiloxKey
from ..wavefunction_Ynlm.nn import AINetData
from .Tmoves import HostTmoveDraws, compute_tmoves
from .drift_diffusion import propose_drift_diffusion


@dataclasses.dataclass
class HostDmcDraws:
    """Injected draws of one dmc_propagate_run step (parity mode): the T-moves' draws, the
    drift-diffusion sweep's gauss1 [B,3N] / gauss2 [B,N,3N] or [B,N,3] / u [B,N], and the grid
    rotations [B,3,3] of the pp energies before (rot_old) and after (rot_new) the move."""
    tmoves: HostTmoveDraws
    drift: HostDraws
    rot_old: torch.Tensor
    rot_new: torch.Tensor


def dmc_propagate(signed_network, log_network, logabs_f, list_l: int, nelectrons: int, natoms: int, ndim: int,
                  batch_size: int, tstep: float, nsteps: int, charges, spins, Rn_local, Local_coes, Local_exps,
                  Rn_non_local, Non_local_coes, Non_local_exps):
    del nsteps
    dd = propose_drift_diffusion(signed_network, tstep, ndim, nelectrons, batch_size)
    le = pphamiltonian.local_energy(f=signed_network, lognetwork=log_network, charges=charges, nspins=spins,
                                    rn_local=Rn_local, local_coes=Local_coes, local_exps=Local_exps,
                                    rn_non_local=Rn_non_local, non_local_coes=Non_local_coes,
                                    non_local_exps=Non_local_exps, natoms=natoms, nelectrons=nelectrons, ndim=ndim,
                                    list_l=list_l)
    net = signed_network._aiqmc_network
    tm = compute_tmoves(list_l, tstep, nelectrons, natoms, ndim, signed_network, Rn_non_local, Non_local_coes,
                        Non_local_exps)

    def dmc_propagate_run(params, key, data, weights: torch.Tensor, branchcut_start, e_trial, e_est):
        if isinstance(key, HostDmcDraws):
            k_tm, k_eo, k_dd, k_en = key.tmoves, HostRotations(key.rot_old), key.drift, HostRotations(key.rot_new)
        else:
            k = key if isinstance(key, PhiloxKey) else PhiloxKey(int(key), 0)
            k_tm, k_eo, k_dd, k_en = (PhiloxKey(k.seed + 3, k.offset), PhiloxKey(k.seed + 1, k.offset), k,
                                      PhiloxKey(k.seed + 2, k.offset))
        pos_t, _ = tm(data, params, k_tm)
        t_move_data = AINetData(positions=pos_t, spins=data.spins, atoms=data.atoms, charges=data.charges)
        eloc_old, _ = le(params, k_eo, data)
        new_data, _, tdamp_scalar, go, gn = dd(params, k_dd, t_move_data)
        eloc_new, _ = le(params, k_en, new_data)
        ctx = net.bind(params, data.atoms, go.dtype)
        td = torch.zeros(3, dtype=torch.float64, device=go.device)
        td[2] = tdamp_scalar
        bc = float(torch.as_tensor(branchcut_start).reshape(-1)[0].real)
        w = weights.to(go.device, go.dtype).contiguous().clone()
        if w.numel() == 1:
            w = w.expand(go.shape[0]).contiguous()
        cuts = None
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            cuts = ctx.dmc_cut_minima(eloc_old, eloc_new, e_est, bc)
            dist.all_reduce(cuts, op=dist.ReduceOp.MIN)
        ctx.dmc_weights(w, eloc_old, eloc_new, go, gn, td, tstep, e_trial, e_est, bc, cut_minima=cuts)
        return eloc_new, w, new_data

    return dmc_propagate_run
