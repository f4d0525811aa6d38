"""Metropolis step oracle (TEST INFRASTRUCTURE ONLY).

Restates ``AIQMCrelease3/VMC/VMCmcstep.py:11-111`` (limdrift, walkers_accept,
walkers_update) with the random draws injected by the host:

* ``gauss1`` [B,3N]  standard normals, scaled by sqrt(tstep)   (:58 / :318)
* ``gauss2`` [B,N,3N] standard normals, scaled by sqrt(tstep)  (:83 / :343)
* ``u``      [B,N]   uniforms in [0,1)                          (:19-20)

Quirks kept: Q5 (per-electron acceptance on single-move configurations, all
accepted electrons move together), Q6 (t_pro is a SUM over xyz and uses the
second draw), Q8 (limdrift's v2 is summed over the whole device batch).
"""
from __future__ import annotations

import math

import torch
from torch.func import grad, vmap


def limdrift(g, tau, acyrus):
    """VMCmcstep.py:11-14: v2 summed over ALL entries of g (Q8)."""
    v2 = torch.sum(g ** 2)
    taueff = (torch.sqrt(1 + 2 * tau * acyrus * v2) - 1) / (acyrus * v2)
    return g * taueff


def taueff(g, tau, acyrus):
    """The factor limdrift multiplies g by (VMCmcstep.py:12-13), in g's dtype."""
    v2 = torch.sum(g ** 2)
    return (torch.sqrt(1 + 2 * tau * acyrus * v2) - 1) / (acyrus * v2)


def walkers_update(net, params, x, gauss1, gauss2, u, tstep: float, chunk: int = 256, info=None):
    """One MH step for a device batch x[B,3N] -> new x[B,3N] (VMCmcstep.py:28-111).

    info: optional dict, filled with the step's intermediates (limdrift factors of the walker and
    proposal gradients, the acceptance decisions) for the fp32 Metropolis parity fixture."""
    B, n3 = x.shape
    N = n3 // 3
    f = lambda p: net.logabs(params, p)
    gfn = vmap(grad(f))
    lfn = vmap(f)

    def chunked(fn, inp):
        return torch.cat([fn(inp[s:s + chunk]) for s in range(0, inp.shape[0], chunk)])

    grad_x = chunked(gfn, x)                                     # :41-53
    g1 = math.sqrt(tstep) * gauss1                               # :58
    grad_eff = limdrift(grad_x, tstep, 0.25)                     # :60
    g = (grad_eff * tstep + g1).reshape(B, N, 3)                 # :62-63
    x1 = x.reshape(B, 1, N, 3).expand(B, N, N, 3)
    z = torch.zeros(B, N, N, 3, dtype=x.dtype)
    idx = torch.arange(N)
    z[:, idx, idx, :] = g                                        # :64-76 change_configurations
    x2 = (x1 + z).reshape(B, N, n3)
    grad_new = chunked(gfn, x2.reshape(B * N, n3)).reshape(B, N, n3)   # :79
    grad_new_eff = limdrift(grad_new, tstep, 0.25)               # :80
    ge = grad_eff[:, None, :].expand(B, N, n3)                   # :81-82
    g2 = math.sqrt(tstep) * gauss2                               # :83
    forward = g2 ** 2
    backward = (g2 + (ge + grad_new_eff) * tstep) ** 2
    t_prob = torch.exp((forward - backward) / (2 * tstep)).reshape(B, N, N, 3).sum(-1)
    t_pro = torch.diagonal(t_prob, dim1=1, dim2=2)               # :87-94
    wave_x2 = chunked(lfn, x2.reshape(B * N, n3)).reshape(B, N)  # :95-97
    wave_x1 = chunked(lfn, x).reshape(B, 1).expand(B, N)         # :98-99 (same value N times)
    acceptance = torch.abs(torch.exp(wave_x2 - wave_x1)) ** 2 * t_pro   # :100
    cond = (acceptance > u).reshape(B, N, 1)                     # walkers_accept :18-25
    x_init = x.reshape(B, N, 3)
    x_new = torch.where(cond, x_init + g, x_init)
    if info is not None:
        info.update(taueff_walkers=taueff(grad_x, tstep, 0.25), taueff_proposals=taueff(grad_new, tstep, 0.25),
                    cond=cond.reshape(B, N), grad_x=grad_x, logabs_x=wave_x1[:, 0], logabs_x2=wave_x2)
    return x_new.reshape(B, n3), acceptance


def mc_step(net, params, x, gauss1, gauss2, u, tstep: float, nsteps: int):
    """main_monte_carlo (VMCmcstep.py:121-140): nsteps walkers_update in sequence.

    gauss1 [nsteps,B,3N], gauss2 [nsteps,B,N,3N], u [nsteps,B,N].
    """
    for s in range(nsteps):
        x, _ = walkers_update(net, params, x, gauss1[s], gauss2[s], u[s], tstep)
    return x
