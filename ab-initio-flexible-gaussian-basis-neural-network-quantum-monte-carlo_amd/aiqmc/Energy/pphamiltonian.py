"""Pseudopotential local energy (drop-in for AIQMCrelease3/Energy/pphamiltonian.py).

``local_energy(f, lognetwork, charges, nspins, rn_local, local_coes, local_exps,
rn_non_local, non_local_coes, non_local_exps, natoms, nelectrons, ndim, list_l,
use_scan=False, complex_output=False)`` returns ``_e_l(params, key, data) ->
(E_L, None)`` (pphamiltonian.py:130-190) with E_L complex [B]:
V_ee + V_nn + KE + local pp + nonlocal pp (complex_output=True adds the kinetic energy's phase
terms, pphamiltonian.py:84-104, from aiqmc_local_energy_complex).  The whole batch runs on the GPU
(aiqmc_local_energy_ecp): the all-electron local-energy kernels, then the
N*A*50 quadrature configurations of every walker as value-only single-electron
moves through the walker cache, then one reduction wave per walker.

``key`` selects the grid rotations (the reference draws one
jax.random.orthogonal matrix per walker key, pseudopotential.py:233-241,
loss.py:203-204): a ``HostRotations(rot[B,3,3])`` injects them (parity mode),
a ``PhiloxKey(seed, offset)`` or an int seed draws Haar O(3) matrices on the
device.  ``lognetwork`` must be the complex log of the same network
(log|psi| + i phase, main_pp_adam_muti_GPU.py:119-121); it is not called.
"""
from __future__ import annotations

import dataclasses
from typing import Optional, Tuple, Union

import numpy as np
import torch

from ..VMC.VMCmcstep import PhiloxKey
from .hamiltonian import _network_of


@dataclasses.dataclass
class HostRotations:
    rot: torch.Tensor   # [B, 3, 3], row-major, as jax.random.orthogonal returns


def local_energy(f, lognetwork, charges, nspins, rn_local, local_coes, local_exps, rn_non_local,
                 non_local_coes, non_local_exps, natoms: int, nelectrons: int, ndim: int, list_l: int,
                 use_scan: bool = False, complex_output: bool = False):
    del nspins, use_scan, lognetwork
    if ndim != 3:
        raise NotImplementedError("ndim must be 3")
    net = _network_of(f)
    if natoms != net.natoms or nelectrons != net.nelectrons:
        raise ValueError("natoms / nelectrons do not match the network")
    c = np.asarray(charges.detach().cpu() if isinstance(charges, torch.Tensor) else charges, dtype=np.float64)
    if c.shape != net.charges.shape or not np.allclose(c, net.charges):
        raise ValueError("local_energy charges differ from the network's charges")
    tables = tuple(np.asarray(t.detach().cpu() if isinstance(t, torch.Tensor) else t, dtype=np.float64)
                   for t in (rn_local, local_coes, local_exps, rn_non_local, non_local_coes, non_local_exps))
    if tables[3].reshape(natoms, -1).shape[1] % (int(list_l) + 1):
        raise ValueError("non-local tables must have list_l + 1 angular channels per atom")
    token = (int(list_l),) + tuple(t.tobytes() for t in tables)

    def _e_l(params, key: Union[int, PhiloxKey, HostRotations, None],
             data) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        pos = data.positions if isinstance(data.positions, torch.Tensor) else torch.as_tensor(
            np.asarray(data.positions))
        dtype = pos.dtype if pos.dtype in (torch.float32, torch.float64) else torch.float32
        ctx = net.bind(params, data.atoms, dtype)
        if getattr(ctx, "_ecp_token", None) != token:
            ctx.set_ecp(*tables, list_l=int(list_l))
            ctx._ecp_token = token
        # complex_output: the kinetic energy's phase terms (pphamiltonian.py:84-104 =
        # hamiltonian.py:110-130) added in the same call, from the log|psi| and theta launch pairs
        if isinstance(key, HostRotations):
            e = ctx.local_energy_ecp(pos, rot=torch.as_tensor(key.rot), complex_output=complex_output)
        else:
            k = key if isinstance(key, PhiloxKey) else PhiloxKey(int(key or 0), 0)
            e = ctx.local_energy_ecp(pos, seed=k.seed, offset=k.offset, complex_output=complex_output)
        return e.reshape(pos.shape[:-1]), None

    _e_l._aiqmc_network = net
    return _e_l
