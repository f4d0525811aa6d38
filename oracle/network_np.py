"""Independent numpy float64 forward of the AIQMC wavefunction (TEST INFRA ONLY).

Written with explicit per-electron / per-pair loops (no shared code with
``oracle.network``) so the two restatements cross-check each other.  Follows
``wavefunction_Ynlm/nn.py:106-553``, ``network_blocks.py:106-206``,
``Jastrow.py:16-135``, ``envelope.py:8-32``.
"""
from __future__ import annotations

import math

import numpy as np

from .system import System


def _ylm_terms(t, r):
    """Y_sp (nn.py:156-167) and Y_hi (nn.py:169-193, Q3 clamp) for one (i, a)."""
    x0, x1, x2 = t
    x3 = x2
    y = r
    pi = math.pi
    sp = [0.5 * math.sqrt(1 / pi), math.sqrt(3 / (4 * pi)) * x0,
          math.sqrt(3 / (4 * pi)) * x1, math.sqrt(3 / (4 * pi)) * x2]
    hi = [0.5 * math.sqrt(15 / pi) * x0 * x1 / y ** 2,
          0.5 * math.sqrt(15 / pi) * x1 * x2 / y ** 2,
          0.25 * math.sqrt(5 / pi) * (3 * x2 ** 2 - y ** 2) / y ** 2,
          0.5 * math.sqrt(15 / pi) * x0 * x2 / y ** 2,
          0.25 * math.sqrt(15 / pi) * (x0 ** 2 - x1 ** 2) / y ** 2,
          0.25 * math.sqrt(35 / (2 * pi)) * x1 * (3 * x0 ** 2 - x1 ** 2) / y ** 3,
          0.5 * math.sqrt(105 / pi) * x0 * x1 * x2 / y ** 3,
          0.25 * math.sqrt(21 / (2 * pi)) * x1 * (5 * x2 ** 2 - y ** 2) / y ** 3,
          0.25 * math.sqrt(7 / pi) * (5 * x2 ** 3 - 3 * x2 * y ** 2) / y ** 3,
          0.25 * math.sqrt(21 / (2 * pi)) * x0 * (5 * x2 ** 2 - y ** 2) / y ** 3,
          0.25 * math.sqrt(105 / pi) * (x0 ** 2 - x1 ** 2) * x3 / y ** 3,
          0.25 * math.sqrt(35 / (2 * pi)) * x0 * (x0 ** 2 - 3 * x1 ** 2) / y ** 3]
    return sp, hi


def log_psi(system: System, params, pos: np.ndarray):
    """Returns (phase, log|psi|) for one walker ``pos[3N]``."""
    N, A = system.nelectrons, system.natoms
    nup = system.nspins[0]
    t = system.tables()
    R = system.atoms
    Z = system.charges
    x = pos.reshape(N, 3)
    groups = [g for g in (list(range(0, nup)), list(range(nup, N))) if len(g) > 0]
    s2 = math.sqrt(2.0)

    def res(a, b):
        return (a + b) / s2 if a.shape == b.shape else b

    # per-electron features
    h = np.zeros((N, 4 * A))
    yin = np.zeros((N, 4 * A + 2))
    for i in range(N):
        sps, his = [], []
        for a in range(A):
            d = x[i] - R[a]
            r = math.sqrt(float(d @ d))
            h[i, 4 * a] = r
            h[i, 4 * a + 1:4 * a + 4] = d
            sp, hi = _ylm_terms(d / r, r)
            sps += sp
            his += hi
        yin[i, :4 * A] = sps
        yin[i, 4 * A] = np.mean(his)
        yin[i, 4 * A + 1] = np.mean(sps)
    y = yin
    for p in params["layers"]["streams_y"]:
        q = p["single_Ynlm"]
        y = res(y, np.tanh(y @ q["w"] + q["b"]))
    # pair features: h2[i,j] = [r_ij, x_j - x_i], diagonal zero
    h2 = np.zeros((N, N, 4))
    for i in range(N):
        for j in range(N):
            if i != j:
                d = x[j] - x[i]
                h2[i, j, 0] = math.sqrt(float(d @ d))
                h2[i, j, 1:] = d
    for p in params["layers"]["streams"]:
        feats = [h]
        feats += [np.tile(h[g].mean(0), (N, 1)) for g in groups]
        feats += [h2[g].mean(0) for g in groups]
        f = np.concatenate(feats, 1)
        wc, bc = p["convolutional"]["w"], p["convolutional"]["b"]
        q = f.shape[1] // 4
        c = np.zeros((N, q))
        for i in range(N):
            for k in range(q):
                c[i, k] = np.tanh(np.mean(f[i, 4 * k:4 * k + 4] * wc[i, 4 * k:4 * k + 4]) + bc[i, k])
        nxt = np.tanh(c @ p["single"]["w"] + p["single"]["b"])
        if "double" in p:
            h2 = res(h2, np.tanh(h2 @ p["double"]["w"] + p["double"]["b"]))
        h = res(h, nxt)
    # orbitals
    rows = list(t["spin_up_indices"]) + list(t["spin_down_indices"])
    nch_up = len(t["spin_up_indices"])
    wy = params["y"][0]["w"]
    wy = wy / np.linalg.norm(wy, axis=-1, keepdims=True)
    yorb = y @ wy
    M = np.zeros((N, N), dtype=np.complex128)
    for r in range(N):
        ps = params["orbitals"][0 if r < nch_up else 1]
        o = h[rows[r]] @ ps["w"] + ps["b"]
        pe = params["envelope"][r]
        env = 0.0
        for a in range(A):
            d = x[r] - R[a]
            rr = math.sqrt(float(d @ d))
            env += math.exp(-pe["beta"][a] * rr ** 2) * pe["alpha"][0]
            for dd in range(3):
                env += math.exp(-d[dd] * pe["pi"][a, dd]) * pe["sigma"][a, dd] * pe["xi"][0]
        for c in range(N):
            M[r, c] = (o[2 * c] + 1j * o[2 * c + 1]) * env * yorb[r, c]
    # Jastrows
    jee = 0.0
    for p, (i, j) in enumerate(t["parallel_indices"].T):
        r = np.linalg.norm(x[j] - x[i])
        jee += 0.25 * r / (1.0 + params["jastrow_ee"]["ee_par"][p] * r)
    for p, (i, j) in enumerate(t["antiparallel_indices"].T):
        r = np.linalg.norm(x[j] - x[i])
        jee += 0.5 * r / (1.0 + params["jastrow_ee"]["ee_anti"][p] * r)
    jae = 0.0
    for i in range(N):
        for a in range(A):
            r = np.linalg.norm(x[i] - R[a])
            b = params["jastrow_ae"]["ae"][i, a]
            jae += -((2 * Z[a]) ** 0.75) * (1 - math.exp(-((2 * Z[a]) ** 0.25) * r * b)) / (2 * b)
    M = M * math.exp(jee / N) * math.exp(jae / N)
    sign, logdet = np.linalg.slogdet(M)
    return float(np.angle(sign)), float(np.log(np.abs(sign)) + logdet)


def potential(system: System, pos: np.ndarray) -> float:
    """hamiltonian.py:177-233."""
    N = system.nelectrons
    x = pos.reshape(N, 3)
    v = 0.0
    for i in range(N):
        for j in range(i + 1, N):
            v += 1.0 / np.linalg.norm(x[i] - x[j])
        for a in range(system.natoms):
            v -= system.charges[a] / np.linalg.norm(x[i] - system.atoms[a])
    for a in range(system.natoms):
        for b in range(a + 1, system.natoms):
            v += system.charges[a] * system.charges[b] / np.linalg.norm(system.atoms[a] - system.atoms[b])
    return v
