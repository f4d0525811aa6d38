"""Local energy (drop-in for AIQMCrelease3/Energy/hamiltonian.py).

``local_energy(f, charges, nspins, use_scan=False, complex_output=False)``
returns ``_e_l(params, key, data) -> (E_L, None)`` (hamiltonian.py:236-260); with
complex_output=True E_L is complex (the phase terms of :110-130).
For an AIQMC network (``f`` produced by ``make_ai_net``) the whole local
energy -- potential + kinetic via a forward Laplacian equal to the reference's
jvp-of-grad loop (:100-131) -- runs in ONE HIP kernel launch over the batch
``data.positions[B,3N]``.  Any other ``f`` raises: this package has no
autodiff fallback.

The potential functions (:177-233) are provided as torch ops for API parity.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np
import torch


def potential_electron_electron(r_ee: torch.Tensor) -> torch.Tensor:
    """hamiltonian.py:177-187 (r_ee [..., N, N, 1])."""
    n = r_ee.shape[-2]
    iu = torch.triu_indices(n, n, 1, device=r_ee.device)
    return (1.0 / r_ee[..., iu[0], iu[1], 0]).sum(-1)


def potential_electron_nuclear(charges: torch.Tensor, r_ae: torch.Tensor) -> torch.Tensor:
    """hamiltonian.py:190-198."""
    return -torch.sum(charges / r_ae[..., 0], dim=(-2, -1))


def potential_nuclear_nuclear(charges: torch.Tensor, atoms: torch.Tensor) -> torch.Tensor:
    """hamiltonian.py:201-210."""
    r_aa = torch.linalg.norm(atoms[None, ...] - atoms[:, None], dim=-1)
    a = atoms.shape[0]
    iu = torch.triu_indices(a, a, 1, device=atoms.device)
    cc = charges[None, :] * charges[:, None]
    return (cc[iu[0], iu[1]] / r_aa[iu[0], iu[1]]).sum()


def potential_energy(r_ae, r_ee, atoms, charges) -> torch.Tensor:
    """hamiltonian.py:213-233."""
    return (potential_electron_electron(r_ee) + potential_electron_nuclear(charges, r_ae)
            + potential_nuclear_nuclear(charges, atoms))


def _network_of(f):
    net = getattr(f, "_aiqmc_network", None)
    if net is None:
        raise TypeError("local_energy: f must be the apply function of an aiqmc make_ai_net Network "
                        "(the HIP local-energy kernel is specific to that ansatz)")
    return net


def local_kinetic_energy(f, use_scan: bool = False, complex_output: bool = True):
    """hamiltonian.py:77-132: returns ke(params, data) -> -1/2 (lap log|psi| + |grad log|psi||^2), or
    with complex_output (the reference's default here, :110-130) the complex
    -1/2 [lap log|psi| + i lap theta] - 1/2 |grad log|psi||^2 + 1/2 |grad theta|^2
    - i grad log|psi| . grad theta  (theta = arg psi; aiqmc_local_energy_complex)."""
    del use_scan
    net = _network_of(f)

    def ke(params, data):
        pos = data.positions if isinstance(data.positions, torch.Tensor) else torch.as_tensor(data.positions)
        dtype = pos.dtype if pos.dtype in (torch.float32, torch.float64) else torch.float32
        ctx = net.bind(params, data.atoms, dtype)
        if complex_output:
            el = ctx.local_energy_complex(pos)
        else:
            el, _, _ = ctx.local_energy(pos)
        # E_L = V + KE  ->  KE = E_L - V  (V from the same kernel would need a second output;
        # computed here from positions with the reference potential formulas)
        p = pos.to(ctx.device, dtype).reshape(-1, net.nelectrons, 3)
        atoms = torch.as_tensor(np.asarray(ctx_atoms(data.atoms)), dtype=dtype, device=ctx.device)
        charges = torch.as_tensor(net.charges, dtype=dtype, device=ctx.device)
        ae = p[:, :, None, :] - atoms[None, None]
        r_ae = torch.linalg.norm(ae, dim=-1, keepdim=True)
        ee = p[:, None, :, :] - p[:, :, None, :]
        eye = torch.eye(net.nelectrons, dtype=dtype, device=ctx.device)
        r_ee = (torch.linalg.norm(ee + eye[..., None], dim=-1) * (1.0 - eye))[..., None]
        v = potential_energy(r_ae, r_ee, atoms, charges)
        return (el - v).reshape(pos.shape[:-1])
    return ke


def ctx_atoms(atoms):
    a = atoms.detach().cpu().numpy() if isinstance(atoms, torch.Tensor) else np.asarray(atoms)
    a = np.asarray(a, dtype=np.float64)
    return a.reshape(-1, a.shape[-2], a.shape[-1])[0] if a.ndim == 3 else a


def local_energy(f, charges, nspins: Sequence[int], use_scan: bool = False, complex_output: bool = False):
    """hamiltonian.py:236-260.  ``charges`` is the closure used for the potential.

    The HIP kernel takes the potential charges from the network's configuration
    (make_ai_net ``charges``); they must agree with the charges given here.
    complex_output=True returns the complex local energy (:110-130; the phase's Laplacian and
    gradient from a second launch pair, aiqmc_local_energy_complex).
    """
    del nspins, use_scan
    net = _network_of(f)
    c = np.asarray(charges.detach().cpu() if isinstance(charges, torch.Tensor) else charges, dtype=np.float64)
    if c.shape != net.charges.shape or not np.allclose(c, net.charges):
        raise ValueError("local_energy charges differ from the network's charges")

    def _e_l(params, key, data) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        del key
        pos = data.positions if isinstance(data.positions, torch.Tensor) else torch.as_tensor(
            np.asarray(data.positions))
        dtype = pos.dtype if pos.dtype in (torch.float32, torch.float64) else torch.float32
        ctx = net.bind(params, data.atoms, dtype)
        if complex_output:
            el = ctx.local_energy_complex(pos)
        else:
            el, _, _ = ctx.local_energy(pos)
        return el.reshape(pos.shape[:-1]), None
    _e_l._aiqmc_network = net
    return _e_l
