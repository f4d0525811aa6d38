"""Local energy oracle (TEST INFRASTRUCTURE ONLY).

Restates ``AIQMCrelease3/Energy/hamiltonian.py``:
  * potentials ``:177-233``;
  * ``local_kinetic_energy`` ``:77-132`` with ``complex_output=False`` (the N2
    driver's setting, ``main_all_electrons_adam_muti_GPU.py:143``):
    ``primal, dgrad = jax.linearize(grad(logabs), x)`` then a ``fori_loop``
    summing ``dgrad(e_i)[i]``.  ``jax.linearize`` evaluated on ``e_i`` is the
    JVP of the gradient along ``e_i``; we compute exactly that with
    ``torch.func.jvp(torch.func.grad(f), (x,), (e_i,))``, batched over walkers
    with ``torch.func.vmap``;
  * ``local_energy`` ``:236-260``: V(r_ae, r_ee, atoms, charges) + KE.
A second, independent kinetic-energy path uses the full Hessian trace (the
ferminet test pattern ``ferminet/tests/hamiltonian_test.py:41-58``).
"""
from __future__ import annotations

from typing import Callable

import torch
from torch.func import grad, jvp, vmap, hessian


def potential_electron_electron(r_ee):
    """hamiltonian.py:177-187 (r_ee [N,N,1])."""
    n = r_ee.shape[0]
    iu = torch.triu_indices(n, n, 1)
    return (1.0 / r_ee[iu[0], iu[1], 0]).sum()


def potential_electron_nuclear(charges, r_ae):
    """hamiltonian.py:190-198."""
    return -torch.sum(charges / r_ae[..., 0])


def potential_nuclear_nuclear(charges, atoms):
    """hamiltonian.py:201-210."""
    r_aa = torch.linalg.norm(atoms[None, ...] - atoms[:, None], dim=-1)
    cc = charges[None, ...] * charges[..., None]
    a = atoms.shape[0]
    iu = torch.triu_indices(a, a, 1)
    return (cc[iu[0], iu[1]] / r_aa[iu[0], iu[1]]).sum()


def potential_energy(r_ae, r_ee, atoms, charges):
    """hamiltonian.py:213-233."""
    return (potential_electron_electron(r_ee) + potential_electron_nuclear(charges, r_ae)
            + potential_nuclear_nuclear(charges, atoms))


def construct_r(pos, atoms):
    x = pos.reshape(-1, 1, 3)
    ae = x - atoms[None]
    r_ae = torch.linalg.norm(ae, dim=2, keepdim=True)
    ee = pos.reshape(1, -1, 3) - pos.reshape(-1, 1, 3)
    n = ee.shape[0]
    eye = torch.eye(n, dtype=pos.dtype)
    r_ee = torch.linalg.norm(ee + eye[..., None], dim=-1) * (1.0 - eye)
    return r_ae, r_ee[..., None]


def kinetic_jvp_of_grad(logabs: Callable[[torch.Tensor], torch.Tensor]):
    """hamiltonian.py:100-131, complex_output=False: single walker x[3N] -> KE."""
    g = grad(logabs)

    def ke(x):
        n = x.shape[0]
        eye = torch.eye(n, dtype=x.dtype)
        primal = g(x)
        diag = torch.zeros((), dtype=x.dtype)
        for i in range(n):                                   # lax.fori_loop(0, n, ...)
            _, t = jvp(g, (x,), (eye[i],))
            diag = diag + t[i]
        return -0.5 * diag - 0.5 * torch.sum(primal ** 2)
    return ke


def kinetic_complex_jvp_of_grad(logabs: Callable[[torch.Tensor], torch.Tensor],
                                phase: Callable[[torch.Tensor], torch.Tensor]):
    """hamiltonian.py:100-131 with complex_output=True (:110-130): single walker x[3N] ->
    [Re KE, Im KE] of -1/2 sum_i (d_i grad log|psi| + i d_i grad theta)_i - 1/2 |grad log|psi||^2
    + 1/2 |grad theta|^2 - i grad log|psi| . grad theta  (theta = the phase output of f)."""
    g = grad(logabs)
    gp = grad(phase)

    def ke(x):
        n = x.shape[0]
        eye = torch.eye(n, dtype=x.dtype)
        primal = g(x)
        pprimal = gp(x)
        d_re = torch.zeros((), dtype=x.dtype)
        d_im = torch.zeros((), dtype=x.dtype)
        for i in range(n):                                   # lax.fori_loop(0, n, ...)
            _, t = jvp(g, (x,), (eye[i],))
            _, tp = jvp(gp, (x,), (eye[i],))
            d_re = d_re + t[i]
            d_im = d_im + tp[i]
        re = -0.5 * d_re - 0.5 * torch.sum(primal ** 2) + 0.5 * torch.sum(pprimal ** 2)
        im = -0.5 * d_im - torch.sum(primal * pprimal)
        return torch.stack([re, im])
    return ke


def batch_local_energy_complex(net, params, pos: torch.Tensor, chunk: int = 32) -> torch.Tensor:
    """complex_output=True local energy (hamiltonian.py:236-260 with :110-130) of a batch pos[B,3N]:
    a complex tensor [B] (potential real)."""
    atoms = net.atoms.to(pos.dtype)
    charges = net.charges.to(pos.dtype)
    ke = kinetic_complex_jvp_of_grad(lambda x: net.logabs(params, x), lambda x: net.apply(params, x)[0])

    def e_l(x):
        r_ae, r_ee = construct_r(x, atoms)
        k = ke(x)
        return torch.stack([potential_energy(r_ae, r_ee, atoms, charges) + k[0], k[1]])
    f = vmap(e_l)
    out = torch.cat([f(pos[s:s + chunk]) for s in range(0, pos.shape[0], chunk)])
    return torch.complex(out[:, 0], out[:, 1])


def kinetic_hessian(logabs: Callable[[torch.Tensor], torch.Tensor]):
    """ferminet/tests/hamiltonian_test.py:50-58 (kinetic_from_hessian_log)."""
    def ke(x):
        gr = grad(logabs)(x)
        h = hessian(logabs)(x)
        return -0.5 * (torch.trace(h) + torch.sum(gr ** 2))
    return ke


def local_energy(logabs: Callable[[torch.Tensor], torch.Tensor], atoms, charges,
                 method: str = "jvp"):
    """hamiltonian.py:236-260 for one walker; returns E_L."""
    ke = kinetic_jvp_of_grad(logabs) if method == "jvp" else kinetic_hessian(logabs)

    def e_l(x):
        r_ae, r_ee = construct_r(x, atoms)
        return potential_energy(r_ae, r_ee, atoms, charges) + ke(x)
    return e_l


def batch_local_energy(net, params, pos: torch.Tensor, method: str = "jvp", chunk: int = 64):
    """E_L, log|psi|, grad log|psi| for a batch pos[B,3N], in the dtype of pos (float64, or
    float32/complex64 -- the reference's own arithmetic)."""
    atoms = net.atoms.to(pos.dtype)
    charges = net.charges.to(pos.dtype)
    f = lambda x: net.logabs(params, x)
    if method == "jvp":
        el_fn = vmap(local_energy(f, atoms, charges, method))
    else:
        # vmap(hessian) through complex slogdet gives wrong batched results in
        # torch 2.10 (walkers past the first); the Hessian path loops instead.
        el1 = local_energy(f, atoms, charges, method)
        el_fn = lambda p: torch.stack([el1(p[i]) for i in range(p.shape[0])])
    g_fn = vmap(grad(f))
    l_fn = vmap(f)
    outs_e, outs_l, outs_g = [], [], []
    for s in range(0, pos.shape[0], chunk):
        p = pos[s:s + chunk]
        outs_e.append(el_fn(p))
        outs_l.append(l_fn(p))
        outs_g.append(g_fn(p))
    return torch.cat(outs_e), torch.cat(outs_l), torch.cat(outs_g)
