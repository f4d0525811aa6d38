"""ECP local-energy oracle (TEST INFRASTRUCTURE ONLY, float64, CPU).

Restates the reference's pseudopotential Hamiltonian
(``AIQMCrelease3/Energy/pphamiltonian.py:130-190``,
``pseudopotential/pseudopotential.py:86-318``,
``pseudopotential/pp_energy_test.py:45-105``) with the random rotation of
the quadrature grid injected by the caller (``get_rot`` draws it with
``jax.random.orthogonal``, pseudopotential.py:233-241; threefry bits are out of
scope, as for the Metropolis draws).

Quirks kept (SURVEY 8f-1 and the source):
* E1  the local radial terms use r**(n-2) (pseudopotential.py:95), the nonlocal
      ones r**n (:150);
* E2  the rotated electron sits at r_ia * p_q, NOT at R_a + r_ia * p_q
      (:275-276, :288-291): correct only for an atom at the origin;
* E3  cos(theta) divides by the Frobenius norm of ALL rotated points of the
      grid group (:281-283, jnp.linalg.norm of a [npts,3] array), i.e. it is the
      true cosine / sqrt(npts) for unit points;
* E4  "ratio" = (log psi(rotated) / log psi(x)) * w with the COMPLEX log
      (log|psi| + i phase, main_pp_adam_muti_GPU.py:119-121) (:307, :314-315);
* E5  P_l carries 1/(4 pi) on top of weights that already sum to 1 (:256-269);
* E6  every (l, electron, atom) term is multiplied by v_l(r_ia) and summed
      (pp_energy_test.py:85-98), so the result is complex;
* E7  the local part carries -Z/r_ia with data.charges (pseudopotential.py:111);
      the pp Hamiltonian's potential_energy has V_ee + V_nn only
      (pphamiltonian.py:124-127).
The grid constants are the reference's own 8-digit literals (:197-224).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import hamiltonian as ham

_S2 = 0.70710678
_S3 = 0.57735027
OA = np.array([[-1, 0, 0], [0, -1, 0], [0, 0, -1], [0, 0, 1], [0, 1, 0], [1, 0, 0]], dtype=np.float64)
OB = np.array([[-_S2, -_S2, 0.], [-_S2, 0., -_S2], [-_S2, 0., _S2], [-_S2, _S2, 0.],
               [0., -_S2, -_S2], [0., -_S2, _S2], [0., _S2, -_S2], [0., _S2, _S2],
               [_S2, -_S2, 0.], [_S2, 0., -_S2], [_S2, 0., _S2], [_S2, _S2, 0.]])
OC = np.array([[-_S3, -_S3, -_S3], [-_S3, -_S3, _S3], [-_S3, _S3, -_S3], [-_S3, _S3, _S3],
               [_S3, -_S3, -_S3], [_S3, -_S3, _S3], [_S3, _S3, -_S3], [_S3, _S3, _S3]])


def quadrature_grids():
    """generate_quadrature_grids (pseudopotential.py:181-225): [OA, OB, OC, OD], weights."""
    d1 = OC * math.sqrt(3 / 11)
    od1 = np.stack([d1[:, 0], d1[:, 1], d1[:, 2] * 3], axis=1)
    od2 = np.stack([d1[:, 0], d1[:, 1] * 3, d1[:, 2]], axis=1)
    od3 = np.stack([d1[:, 0] * 3, d1[:, 1], d1[:, 2]], axis=1)
    od = np.concatenate([od1, od2, od3], axis=0)
    weights = np.array([4 / 315, 64 / 2835, 27 / 1280, 14641 / 725760])
    return [OA, OB, OC, od], weights


def rotate_points(rot: np.ndarray, pts: np.ndarray) -> np.ndarray:
    """einsum('jkl,ik->jil', rot, P) for one rotation (pseudopotential.py:237-240)."""
    return np.einsum("kl,ik->il", rot, pts)


def p_l(x, list_l: int):
    """P_l (pseudopotential.py:250-269), 1/(4 pi) included (E5); list of list_l+1 arrays."""
    c = 1.0 / (4 * math.pi)
    out = [c * torch.ones_like(x)]
    if list_l >= 1:
        out.append(3 * c * x)
    if list_l >= 2:
        out.append(5 * c * 0.5 * (3 * x * x - 1))
    if list_l >= 3:
        out.append(7 * c * 0.5 * (5 * x * x * x - 3 * x))
    return out


class ECP:
    """Pseudopotential tables as the reference drivers pass them (single_atom_C.py:13-23)."""

    def __init__(self, rn_local, local_coes, local_exps, rn_non_local, non_local_coes, non_local_exps,
                 list_l: int):
        self.rn_local = np.asarray(rn_local, np.float64)            # [A, KL]
        self.local_coes = np.asarray(local_coes, np.float64)
        self.local_exps = np.asarray(local_exps, np.float64)
        self.rn_non_local = np.asarray(rn_non_local, np.float64)    # [A, L, KN]
        self.non_local_coes = np.asarray(non_local_coes, np.float64)
        self.non_local_exps = np.asarray(non_local_exps, np.float64)
        self.list_l = int(list_l)


def c_atom_ccecp() -> ECP:
    """example/single_atom_C/single_atom_C.py:13-36 (list_l = 2)."""
    return ECP([[1.0, 3.0, 2.0]], [[4.00000, 57.74008, -25.81955]], [[14.43502, 8.39889, 7.38188]],
               [[[2.0, 2.0], [2.0, 2.0], [2.0, 2.0]]], [[[52.13345, 0], [0, 0], [0, 0]]],
               [[[7.76079, 0], [0, 0], [0, 0]]], 2)


def c2_ccecp() -> ECP:
    """example/C2/C2.py:12-27: the carbon ccECP block on each of the two atoms (list_l = 2)."""
    c = c_atom_ccecp()
    two = lambda a: np.concatenate([a, a], axis=0)
    return ECP(two(c.rn_local), two(c.local_coes), two(c.local_exps), two(c.rn_non_local), two(c.non_local_coes),
               two(c.non_local_exps), 2)


def co2_ccecp() -> ECP:
    """The CO2 example (AIQMCrelease2/example/CO2/co2_test.py:7-19; atoms C, O, O): the carbon
    block and the oxygen ccECP (Z_eff 6: local 6.0 / 73.85984 / -47.87600 at exponents 12.30997 /
    14.76962 / 13.71419, one l = 0 projector 85.86406 at 13.65512), in release 3's [A, 3, 2]
    nonlocal layout (the l = 0 term first, as c_atom_ccecp)."""
    c = c_atom_ccecp()
    o_loc = ([1.0, 3.0, 2.0], [6.0, 73.85984, -47.87600], [12.30997, 14.76962, 13.71419])
    o_nl = ([[2.0, 2.0], [2.0, 2.0], [2.0, 2.0]], [[85.86406, 0], [0, 0], [0, 0]], [[13.65512, 0], [0, 0], [0, 0]])
    st = lambda a, o: np.concatenate([a, [o], [o]], axis=0)
    return ECP(st(c.rn_local, o_loc[0]), st(c.local_coes, o_loc[1]), st(c.local_exps, o_loc[2]),
               st(c.rn_non_local, o_nl[0]), st(c.non_local_coes, o_nl[1]), st(c.non_local_exps, o_nl[2]), 2)


def local_pp_energy(ecp: ECP, pos: torch.Tensor, atoms: torch.Tensor, charges: torch.Tensor):
    """local_pp_energy (pseudopotential.py:86-117) summed over electrons and atoms."""
    N = pos.shape[0] // 3
    ae = pos.reshape(N, 1, 3) - atoms[None]
    r = torch.linalg.norm(ae, dim=-1)                                        # [N, A]
    part1 = -charges[None] / r
    rn = torch.as_tensor(ecp.rn_local) - 2                                   # E1
    co = torch.as_tensor(ecp.local_coes)
    ex = torch.as_tensor(ecp.local_exps)
    part2 = (co[None] * r[..., None] ** rn[None] * torch.exp(-ex[None] * r[..., None] ** 2)).sum(-1)
    return (part1 + part2).sum()


def non_local_coefficients(ecp: ECP, pos: torch.Tensor, atoms: torch.Tensor):
    """get_non_v_l (pseudopotential.py:134-165): v[N, A, L] with r**n (E1)."""
    N = pos.shape[0] // 3
    r = torch.linalg.norm(pos.reshape(N, 1, 3) - atoms[None], dim=-1)       # [N, A]
    rn = torch.as_tensor(ecp.rn_non_local)
    co = torch.as_tensor(ecp.non_local_coes)
    ex = torch.as_tensor(ecp.non_local_exps)
    rr = r[..., None, None]
    return (co[None] * rr ** rn[None] * torch.exp(-ex[None] * rr ** 2)).sum(-1)


def rotated_configurations(pos: torch.Tensor, atoms: torch.Tensor, pts: np.ndarray):
    """get_P_l.generate_points_information geometry (pseudopotential.py:303-313).

    Returns cos_theta [N, A, P] (E3) and the configurations [N, A, P, 3N] (E2)."""
    N = pos.shape[0] // 3
    A = atoms.shape[0]
    x2 = pos.reshape(N, 3)
    ae = x2[:, None, :] - atoms[None]                                        # [N, A, 3]
    r = torch.linalg.norm(ae, dim=-1)                                        # [N, A]
    p = torch.as_tensor(pts)
    rc = r[..., None, None] * p[None, None]                                  # [N, A, P, 3]
    fro = torch.sqrt((rc ** 2).sum(dim=(-1, -2)))                            # [N, A]
    cos = (ae[:, :, None, :] * rc).sum(-1) / (torch.linalg.norm(ae, dim=-1)[..., None] * fro[..., None])
    P = p.shape[0]
    cfg = x2[None, None, None].expand(N, A, P, N, 3).clone()
    for i in range(N):
        cfg[i, :, :, i, :] = rc[i]
    return cos, cfg.reshape(N, A, P, 3 * N)


def nonlocal_pp_energy(net, params, ecp: ECP, pos: torch.Tensor, rot: np.ndarray):
    """total_energy_pseudopotential's nonlocal sum (pp_energy_test.py:73-98), complex.

    Also returns the complex log psi of every rotated configuration [N, A, 50], the
    groups OA, OB, OC, OD concatenated along the last axis."""
    atoms = net.atoms.to(pos.dtype)
    N, A = net.N, net.A
    ph0, la0 = net.apply(params, pos)
    den = la0 + 1j * ph0                                                     # E4
    vnl = non_local_coefficients(ecp, pos, atoms)                            # [N, A, L]
    groups, weights = quadrature_grids()
    total = torch.zeros((), dtype=torch.complex128)
    logs = []
    for g, w in zip(groups, weights):
        pts = rotate_points(rot, g)
        cos, cfg = rotated_configurations(pos, atoms, pts)
        P = pts.shape[0]
        flat = cfg.reshape(N * A * P, 3 * N)
        vals = [net.apply(params, flat[k]) for k in range(flat.shape[0])]
        ph = torch.stack([v[0] for v in vals])
        la = torch.stack([v[1] for v in vals])
        num = (la + 1j * ph).reshape(N, A, P)
        logs.append(num)
        ratios = num / den * w
        pl = p_l(cos, ecp.list_l)
        out = torch.stack([(q * ratios).sum(-1) for q in pl])                # [L, N, A]
        total = total + (out * vnl.permute(2, 0, 1)).sum()                   # E6
    return total, torch.cat(logs, dim=-1)


def local_energy_pp(net, params, ecp: ECP, pos: torch.Tensor, rot: np.ndarray):
    """pphamiltonian.local_energy._e_l (pphamiltonian.py:177-188), one walker: complex E_L."""
    atoms = net.atoms.to(pos.dtype)
    charges = net.charges.to(pos.dtype)
    f = lambda x: net.logabs(params, x)
    ke = ham.kinetic_jvp_of_grad(f)(pos)
    r_ae, r_ee = ham.construct_r(pos, atoms)
    pot = ham.potential_electron_electron(r_ee) + ham.potential_nuclear_nuclear(charges, atoms)
    loc = local_pp_energy(ecp, pos, atoms, charges)
    nl, logs = nonlocal_pp_energy(net, params, ecp, pos, rot)
    return pot + ke + loc + nl, nl, loc, logs


def batch_local_energy_pp(net, params, ecp: ECP, pos: torch.Tensor, rots: np.ndarray):
    """Complex local energies of pos[B,3N] with rots[B,3,3] (one rotation per walker key,
    loss.py:203-204).  Returns (E_L, nonlocal part, local pp part, complex log psi [B,N,A,50])."""
    out = [local_energy_pp(net, params, ecp, pos[b], rots[b]) for b in range(pos.shape[0])]
    return tuple(torch.stack([o[k] for o in out]) for k in range(4))


def haar_rotations(rng: np.random.Generator, B: int) -> np.ndarray:
    """Haar-distributed O(3) matrices (the distribution of jax.random.orthogonal)."""
    z = rng.standard_normal((B, 3, 3))
    q, r = np.linalg.qr(z)
    d = np.sign(np.einsum("bii->bi", r))
    return q * d[:, None, :]
