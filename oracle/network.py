"""torch float64 restatement of the AIQMC wavefunction (TEST INFRASTRUCTURE ONLY).

Single-walker functional form, differentiable with ``torch.func`` so that the
reference's derivative algorithms (``jax.grad``, ``jax.linearize`` + loop) can
be restated directly.  Every block cites the reference line it follows.
Quirks reproduced: Q1 row/feature mismatch, Q2 position-order
groups, Q3 ``x[3]`` clamped to ``x[2]``, Q4 unit-vector Ylm inputs, Q10 one
determinant, Q11 Jastrow multiplies every matrix element.
"""
from __future__ import annotations

import math
from typing import Any, Dict, Tuple

import numpy as np
import torch

from .system import System

PI = math.pi


def to_torch(tree, dtype=torch.float64):
    if isinstance(tree, dict):
        return {k: to_torch(v, dtype) for k, v in tree.items()}
    if isinstance(tree, list):
        return [to_torch(v, dtype) for v in tree]
    return torch.as_tensor(np.asarray(tree), dtype=dtype)


def construct_input_features(pos: torch.Tensor, atoms: torch.Tensor):
    """nn.py:106-116."""
    x = pos.reshape(-1, 1, 3)
    ae = x - atoms[None, ...]
    ee = pos.reshape(1, -1, 3) - pos.reshape(-1, 1, 3)        # ee[i,j] = x_j - x_i
    r_ae = torch.linalg.norm(ae, dim=2, keepdim=True)
    n = ee.shape[0]
    eye = torch.eye(n, dtype=pos.dtype)
    r_ee = torch.linalg.norm(ee + eye[..., None], dim=-1) * (1.0 - eye)
    return ae, ee, r_ae, r_ee[..., None]


def y_l_real(t):
    """nn.py:156-167 on the last axis of t (unit vectors)."""
    c0 = 0.5 * math.sqrt(1.0 / PI)
    c1 = math.sqrt(3.0 / (4.0 * PI))
    return torch.stack([torch.full_like(t[..., 0], c0), c1 * t[..., 0], c1 * t[..., 1], c1 * t[..., 2]], -1)


def y_l_real_high(x, y):
    """nn.py:169-193.  x = unit vector t [...,3], y = r [...,1] -> [...,12,1].

    Q3: ``x[3]`` on a length-3 vector; JAX clamps out-of-bounds gathers, so it
    reads ``x[2]``.
    """
    x0, x1, x2 = x[..., 0:1], x[..., 1:2], x[..., 2:3]
    x3 = x2
    terms = [
        1 / 2 * math.sqrt(15 / PI) * (x0 * x1 / y ** 2),
        1 / 2 * math.sqrt(15 / PI) * (x1 * x2 / y ** 2),
        1 / 4 * math.sqrt(5 / PI) * ((3 * x2 ** 2 - y ** 2) / y ** 2),
        1 / 2 * math.sqrt(15 / PI) * (x0 * x2 / y ** 2),
        1 / 4 * math.sqrt(15 / PI) * ((x0 ** 2 - x1 ** 2) / y ** 2),
        1 / 4 * math.sqrt(35 / (2 * PI)) * ((x1 * (3 * x0 ** 2 - x1 ** 2)) / y ** 3),
        1 / 2 * math.sqrt(105 / PI) * (x0 * x1 * x2 / y ** 3),
        1 / 4 * math.sqrt(21 / (2 * PI)) * ((x1 * (5 * x2 ** 2 - y ** 2)) / y ** 3),
        1 / 4 * math.sqrt(7 / PI) * ((5 * x2 ** 3 - 3 * x2 * y ** 2) / y ** 3),
        1 / 4 * math.sqrt(21 / (2 * PI)) * ((x0 * (5 * x2 ** 2 - y ** 2)) / y ** 3),
        1 / 4 * math.sqrt(105 / PI) * (((x0 ** 2 - x1 ** 2) * x3) / y ** 3),
        1 / 4 * math.sqrt(35 / (2 * PI)) * ((x0 * (x0 ** 2 - 3 * x1 ** 2)) / y ** 3),
    ]
    return torch.stack(terms, -2)


def _res(x, y):
    """nn.py:284,315: (x+y)/sqrt(2) iff same shape else y."""
    return (x + y) / math.sqrt(2.0) if x.shape == y.shape else y


def construct_symmetric_features(h_one, h_two, nspins):
    """nn.py:142-153 -- groups are POSITION ranges [0:n_up], [n_up:N] (Q2)."""
    n_up = nspins[0]
    h_ones = [h_one[:n_up], h_one[n_up:]]
    h_twos = [h_two[:n_up], h_two[n_up:]]
    g_one = [h.mean(0, keepdim=True).expand(h_one.shape[0], -1) for h in h_ones if h.numel() > 0]
    g_two = [h.mean(0) for h in h_twos if h.numel() > 0]
    return torch.cat([h_one] + g_one + g_two, dim=1)


def convolu_layer(n, x, w, b):
    """network_blocks.py:106-116: mean over feature quads of x*w, plus b."""
    x = x.reshape(n, -1, 4)
    w = w.reshape(n, -1, 4)
    return (x * w).mean(-1) + b


class Network:
    """make_ai_net (nn.py:511-553) with the closure tables of a System."""

    def __init__(self, system: System, rescale_inputs: bool = False):
        self.system = system
        self.rescale_inputs = rescale_inputs
        t = system.tables()
        self.N = system.nelectrons
        self.A = system.natoms
        self.nspins = system.nspins
        self.par = torch.as_tensor(t["parallel_indices"], dtype=torch.long)
        self.anti = torch.as_tensor(t["antiparallel_indices"], dtype=torch.long)
        self.up = torch.as_tensor(t["spin_up_indices"], dtype=torch.long)
        self.dn = torch.as_tensor(t["spin_down_indices"], dtype=torch.long)
        self.charges = torch.as_tensor(system.charges, dtype=torch.float64)
        self.atoms = torch.as_tensor(system.atoms, dtype=torch.float64)

    # -- nn.py:409-506 ------------------------------------------------------
    def orbitals(self, params, pos):
        N, A = self.N, self.A
        atoms = self.atoms.to(pos.dtype)
        charges = self.charges.to(pos.dtype)
        ae, ee, r_ae, r_ee = construct_input_features(pos, atoms)
        # make_ai_net_layers.apply (nn.py:321-352)
        if self.rescale_inputs:
            # nn.py:126-131: log(1 + r) and the vector times log(1 + r)/r.  On the r_ee diagonal
            # (masked to exactly 0 at nn.py:115) that is (0 * 0)/0 = NaN, and the NaN reaches every
            # electron through the g_two means of construct_symmetric_features (nn.py:151).
            lr_ae = torch.log(1 + r_ae)
            ae_features = torch.cat([lr_ae, ae * lr_ae / r_ae], dim=2).reshape(N, -1)
            lr_ee = torch.log(1 + r_ee)
            ee_features = torch.cat([lr_ee, ee * lr_ee / r_ee], dim=2)
        else:
            ae_features = torch.cat([r_ae, ae], dim=2).reshape(N, -1)
            ee_features = torch.cat([r_ee, ee], dim=2)
        temp = ae / r_ae
        y_sp = y_l_real(temp).reshape(N, -1)
        y_df = y_l_real_high(temp, r_ae).reshape(N, -1)
        y_one = torch.cat([y_sp, y_df.mean(-1, keepdim=True), y_sp.mean(-1, keepdim=True)], -1)
        for p in params["layers"]["streams_y"]:
            q = p["single_Ynlm"]
            y_one = _res(y_one, torch.tanh(y_one @ q["w"] + q["b"]))
        h_one, h_two = ae_features, ee_features
        for p in params["layers"]["streams"]:
            h_in = construct_symmetric_features(h_one, h_two, self.nspins)
            c = torch.tanh(convolu_layer(N, h_in, p["convolutional"]["w"], p["convolutional"]["b"]))
            nxt = torch.tanh(c @ p["single"]["w"] + p["single"]["b"])
            h_one_new = _res(h_one, nxt)
            if "double" in p:
                h_two = _res(h_two, torch.tanh(h_two @ p["double"]["w"] + p["double"]["b"]))
            h_one = h_one_new
        # make_orbitals.apply
        hs = [h_one[self.up], h_one[self.dn]]
        orbs = [h @ p["w"] + p["b"] for h, p in zip(hs, params["orbitals"])]
        wy = params["y"][0]["w"]
        wy = wy / torch.linalg.norm(wy, dim=-1, keepdim=True)
        y_orb = y_one @ wy
        orbs = [o[..., ::2] + 1j * o[..., 1::2] for o in orbs]
        m0 = torch.cat(orbs, dim=0).reshape(N, N)
        # envelope.py:26-30 per row i with electron i's geometry and params (Q1)
        rows = []
        for i in range(N):
            pe = params["envelope"][i]
            env = (torch.sum(torch.exp(-pe["beta"] * r_ae[i].reshape(-1) ** 2) * pe["alpha"])
                   + torch.sum(torch.exp(-ae[i] * pe["pi"]) * pe["sigma"] * pe["xi"]))
            rows.append(env * m0[i])
        total = torch.stack(rows) * y_orb
        # Jastrow.py:23-41 (e-e) and 84-93 (e-n)
        r2 = r_ee.reshape(N, N)
        rp = r2[self.par[0], self.par[1]]
        ra = r2[self.anti[0], self.anti[1]]
        jee = (torch.sum(rp * 0.25 / (1.0 + params["jastrow_ee"]["ee_par"] * rp))
               + torch.sum(ra * 0.5 / (1.0 + params["jastrow_ee"]["ee_anti"] * ra)))
        ra_e = r_ae.reshape(N, -1)
        beta = params["jastrow_ae"]["ae"]
        z2 = 2.0 * charges
        jae = torch.sum(-1 * z2 ** 0.75 * (1.0 - torch.exp(-1.0 * z2 ** 0.25 * ra_e * beta)) / (2.0 * beta))
        return total * torch.exp(jee / N) * torch.exp(jae / N)

    # -- network_blocks.py:138-206 -----------------------------------------
    def apply(self, params, pos) -> Tuple[torch.Tensor, torch.Tensor]:
        m = self.orbitals(params, pos)
        if m.shape[-1] == 1:
            x = m[..., 0, 0]
            sign = x / torch.abs(x)
            logdet = torch.log(torch.abs(x))
        else:
            sign, logdet = torch.linalg.slogdet(m)
        phase = torch.angle(sign)
        logabs = torch.log(torch.abs(sign)) + logdet
        return phase, logabs

    def logabs(self, params, pos):
        return self.apply(params, pos)[1]
