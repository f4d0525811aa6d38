"""DMC oracle (TEST INFRASTRUCTURE ONLY, float64, CPU).

Restates the well-defined parts of ``AIQMCrelease3/DMC``:
* ``propose_drift_diffusion`` (drift_diffusion.py:25-107): the VMC one-electron-move
  Metropolis sweep (same draws and quirks as VMCmcstep.walkers_update, Q5-Q8) plus
  tdamp = sum(x_new) / sum(x_proposed) over ALL coordinates of the device batch (:21 -- a
  ratio of coordinate sums, kept as written), grad_eff_old = limdrift(grad(x)) and
  grad_new_eff_s = limdrift(grad(x_new)) (:60-61, :103-104);
* ``comput_S`` (S_matrix.py:4-24): e_cut = min(|e_est - eloc|_all, branchcut) * sign(e_est - eloc)
  -- jnp.min over the stacked array takes ONE minimum over all walkers and the cut (D1);
* the weight update of dmc.py:88-92: w *= exp(tau tdamp (S_new + S_old) / 2);
* ``branch`` (branch.py:10-33): stochastic comb, newinds = searchsorted(cumsum(w),
  (u wtot + linspace(0, wtot, n, endpoint=False)) % wtot), weights -> wtot / n.
Random draws are injected (threefry bits are out of scope).
"""
from __future__ import annotations

import math

import numpy as np
import torch
from torch.func import grad, vmap

from .mcstep import limdrift


def drift_diffusion(net, params, x, gauss1, gauss2, u, tstep: float, chunk: int = 256):
    """One DMC drift-diffusion step for x[B,3N]; returns (x_new, tdamp, grad_eff_old, grad_new_eff_s)."""
    B, n3 = x.shape
    N = n3 // 3
    f = lambda p: net.logabs(params, p)
    gfn = vmap(grad(f))
    lfn = vmap(f)

    def chunked(fn, inp):
        return torch.cat([fn(inp[s:s + chunk]) for s in range(0, inp.shape[0], chunk)])

    g_x = chunked(gfn, x)
    g1 = math.sqrt(tstep) * gauss1
    grad_eff = limdrift(g_x, tstep, 0.25)
    g = (grad_eff * tstep + g1).reshape(B, N, 3)
    x1 = x.reshape(B, 1, N, 3).expand(B, N, N, 3)
    z = torch.zeros(B, N, N, 3, dtype=x.dtype)
    idx = torch.arange(N)
    z[:, idx, idx, :] = g
    x2 = (x1 + z).reshape(B, N, n3)
    changed = x.reshape(B, N, 3) + g                              # :66
    grad_new = chunked(gfn, x2.reshape(B * N, n3)).reshape(B, N, n3)
    grad_new_eff = limdrift(grad_new, tstep, 0.25)
    ge = grad_eff[:, None, :].expand(B, N, n3)
    g2 = math.sqrt(tstep) * gauss2
    t_prob = torch.exp((g2 ** 2 - (g2 + (ge + grad_new_eff) * tstep) ** 2) / (2 * tstep))
    t_pro = torch.diagonal(t_prob.reshape(B, N, N, 3).sum(-1), dim1=1, dim2=2)
    wave_x2 = chunked(lfn, x2.reshape(B * N, n3)).reshape(B, N)
    wave_x1 = chunked(lfn, x).reshape(B, 1).expand(B, N)
    wfratio = torch.exp(wave_x2 - wave_x1)
    ratio = torch.abs(wfratio) ** 2 * t_pro * torch.sign(wfratio)
    cond = (ratio > u).reshape(B, N, 1)
    x_new = torch.where(cond, changed, x.reshape(B, N, 3))
    tdamp = x_new.sum() / changed.sum()                            # walkers_accept :21
    x_new = x_new.reshape(B, n3)
    grad_new_eff_s = limdrift(chunked(gfn, x_new), tstep, 0.25)
    return x_new, tdamp, grad_eff, grad_new_eff_s


def comput_S(e_trial, e_est, branchcut, v2, tau, eloc, nelec):
    """S_matrix.py:4-24 (v2 = grad_eff**2 [B,3N], summed over the last axis)."""
    v2 = np.sum(v2, axis=-1)
    eloc = np.real(eloc)
    e_cut = np.real(e_est) - eloc
    e_cut = np.min(np.concatenate([np.abs(e_cut).reshape(-1), np.asarray([branchcut]).reshape(-1)])) * np.sign(e_cut)
    return np.real(e_trial) - np.real(e_est) + e_cut / (1 + (v2 * tau / nelec) ** 2)


def update_weights(weights, tau, tdamp, s_new, s_old):
    """dmc.py:88-92."""
    return np.exp(tau * tdamp * (0.5 * s_new + 0.5 * s_old)) * weights


def branch(weights, u):
    """branch.py:10-33 with the uniform draw u injected: (new weight, newinds)."""
    n = weights.shape[0]
    prob = np.cumsum(weights)
    wtot = prob[-1]
    base = u * wtot
    newinds = np.searchsorted(prob, (base + np.linspace(0, wtot, n, endpoint=False)) % wtot)
    return wtot / n, newinds
