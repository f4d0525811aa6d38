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


# --------------------------------------------------------------------------------------------
# T-moves (DMC/Tmoves.py:32-225), one walker, draws injected.
#
# Quirks kept, as written in the reference (all relative to Tmoves.py):
# * T1 the quadrature is the pp one (get_P_l, pseudopotential.py:272-318): E2 rotated
#      electron at r_ia p_q R (not offset by the atom), E3 Frobenius cos(theta), E4 ratio =
#      quotient of COMPLEX logs times the group weight w_g;
# * T2 t_amp = ratio * sum_l (exp(-tau v_l(r_ia)) - 1) P_l(cos)   (:54-55, :92-101), P_l with the
#      extra 1/(4 pi) (E5) and v_l with r**n (E1);
# * T3 forward amplitude = where(t_amp > 0, t_amp, 0) with JAX's LEXICOGRAPHIC complex order
#      (real part first, then imaginary) (:102-104);
# * T4 norm = 1 + sum_g w_g sum_{i,a,q} fwd  -- one norm per walker over ALL electrons, the
#      group weight applied a second time (:113-115);
# * T5 per electron row [1, fwd[i, a, q] (a-major, q in OA|OB|OC|OD order)], cdf = cumsum(row /
#      norm) (:123-141); selected = searchsorted(cdf, u + 1) with the SAME u for every electron
#      (:145-149; jnp.searchsorted's scan binary search over the complex lexicographic order,
#      side='left'); index == len(row) means "no move" (:154);
# * T6 back amplitudes index the forward table by ROW = the selected move (clamped to the
#      last electron, JAX gather semantics) times 1 / ratio_total[i, move] (:183-189, :196-198);
# * T7 back norm = 1 + sum_k W_k sum back[:, slice_k] with W = [0, w_OA, w_OB, w_OC, w_OD] and
#      the hard-coded slices [0], [1:19], [19:55], [55:79], [79:151] clipped to the row length
#      (:202-210);
# * T8 acceptance = Re(norm / back_norm) per electron, accepted iff > u_acc[i]; all electrons
#      move simultaneously, each from the ORIGINAL configuration (:212-224).
# --------------------------------------------------------------------------------------------

TMOVE_SLICES = ((0, 1), (1, 19), (19, 55), (55, 79), (79, 151))


def _lex_le(q: complex, a: complex) -> bool:
    """q <= a in JAX's complex sort order (real part, then imaginary part)."""
    return q.real < a.real or (q.real == a.real and q.imag <= a.imag)


def searchsorted_scan(arr, q) -> int:
    """jnp.searchsorted(arr, q, side='left', method='scan'): a fixed-depth binary search
    (ceil(log2(n + 1)) levels, low = 0, high = n, go_left = q <= arr[mid]) that is defined
    for unsorted arrays too."""
    n = len(arr)
    low, high = 0, n
    for _ in range(int(np.ceil(np.log2(n + 1)))):
        mid = (low + high) // 2
        if _lex_le(q, complex(arr[mid])):
            high = mid
        else:
            low = mid
    return high


def tmoves(net, params, ecp, pos, rot, u_sel: float, u_acc, tstep: float):
    """calculate_ratio_weight_tmoves (Tmoves.py:68-224) for ONE walker pos[3N].

    rot [3,3] is get_rot's orthogonal matrix, u_sel the uniform of select_walker (:146),
    u_acc [N] the acceptance uniforms (:216-217).  Returns (new positions [3N], acceptance [N])."""
    from . import pphamiltonian as pp
    atoms = net.atoms.to(pos.dtype)
    N, A = net.N, net.A
    ph0, la0 = net.apply(params, pos)
    den = complex(la0.item(), ph0.item())
    vnl = pp.non_local_coefficients(ecp, pos, atoms).numpy()                 # [N, A, L]
    x2 = pos.reshape(N, 3).numpy()
    r = np.linalg.norm(x2[:, None, :] - atoms.numpy()[None], axis=-1)      # [N, A]
    groups, gw = pp.quadrature_grids()
    fwd, rat, coords = [], [], []
    norm = 1.0 + 0j
    for g, w in zip(groups, gw):
        pts = pp.rotate_points(rot, g)
        cos, cfg = pp.rotated_configurations(pos, atoms, pts)
        P = pts.shape[0]
        flat = cfg.reshape(N * A * P, 3 * N)
        vals = [net.apply(params, flat[k]) for k in range(flat.shape[0])]
        num = np.array([complex(v[1].item(), v[0].item()) for v in vals]).reshape(N, A, P)
        ratio = num / den * w                                                # T1
        pl = [t.numpy() for t in pp.p_l(cos, ecp.list_l)]
        wts = sum((np.exp(-tstep * vnl[:, :, l]) - 1.0)[..., None] * pl[l] for l in range(ecp.list_l + 1))
        t_amp = ratio * wts                                                  # T2
        pos_part = (t_amp.real > 0) | ((t_amp.real == 0) & (t_amp.imag > 0))
        f = np.where(pos_part, t_amp, 0.0)                                   # T3
        norm = norm + w * f.sum()                                            # T4
        fwd.append(f)
        rat.append(ratio)
        coords.append(r[:, :, None, None] * pts[None, None])                 # [N, A, P, 3] (E2)
    fwd = np.concatenate(fwd, axis=-1).reshape(N, A * 50)
    rat = np.concatenate(rat, axis=-1).reshape(N, A * 50)
    coords = np.concatenate(coords, axis=2).reshape(N, A * 50, 3)
    M1 = 1 + A * 50
    row = np.concatenate([np.ones((N, 1)), fwd], axis=1)                     # T5
    rat_f = np.concatenate([np.ones((N, 1)), rat], axis=1)
    cfg_f = np.concatenate([x2[:, None, :], coords], axis=1)
    cdf = np.cumsum(row / norm, axis=-1)
    W = np.concatenate([[0.0], gw])
    new = x2.copy()
    acc = np.zeros(N)
    for i in range(N):
        sel = searchsorted_scan(cdf[i], complex(u_sel + 1.0, 0.0))
        mv = sel if sel < M1 else 0
        back = row[min(mv, N - 1)] * (1.0 / rat_f[i, mv])                   # T6
        bn = 1.0 + sum(W[k] * back[lo:min(hi, M1)].sum() for k, (lo, hi) in enumerate(TMOVE_SLICES))  # T7
        acc[i] = (norm / bn).real                                            # T8
        if acc[i] > u_acc[i]:
            new[i] = cfg_f[i, mv]
    return torch.tensor(new.reshape(-1)), acc


# --------------------------------------------------------------------------------------------
# One dmc_propagate_run step (DMC/dmc.py:72-93) and the driver's block loop (main_dmc.py:113-244),
# draws injected.  e_trial / e_est are per-walker arrays in the first block (total_e returns the
# per-walker energies, total_energy.py:32; main_dmc.py:115-116) and scalars afterwards.
# --------------------------------------------------------------------------------------------

def dmc_step(net, params, ecp, x, weights, e_trial, e_est, branchcut, draws, tstep: float):
    """Returns (eloc_new [B] complex, weights [B], x_new [B,3N], parts dict)."""
    from . import pphamiltonian as pp
    B, n3 = x.shape
    N = n3 // 3
    pos_t = torch.stack([tmoves(net, params, ecp, x[b], draws["rot_tm"][b], float(draws["u_sel"][b]),
                                draws["u_acc"][b], tstep)[0] for b in range(B)])            # dmc.py:79
    x_new, tdamp, go, gn = drift_diffusion(net, params, pos_t, torch.as_tensor(draws["gauss1"]),
                                           torch.as_tensor(draws["gauss2"]), torch.as_tensor(draws["u"]), tstep)
    eloc_old = pp.batch_local_energy_pp(net, params, ecp, x, draws["rot_old"])[0].detach().numpy()
    eloc_new = pp.batch_local_energy_pp(net, params, ecp, x_new, draws["rot_new"])[0].detach().numpy()
    s_old = comput_S(e_trial, e_est, branchcut, go.numpy() ** 2, tstep, eloc_old, N)
    s_new = comput_S(e_trial, e_est, branchcut, gn.numpy() ** 2, tstep, eloc_new, N)
    w = update_weights(np.asarray(weights), tstep, float(tdamp), s_new, s_old)
    return eloc_new, w, x_new, dict(pos_t=pos_t.numpy(), tdamp=float(tdamp), eloc_old=eloc_old)


def reindex(x, newinds, extra):
    """main_dmc.py:215-233 for one device: sorted unique comb indices, killed walkers replaced by the
    last unique walker plus U[0,1) noise."""
    unique = np.unique(newinds)
    temp = x[unique]
    n = x.shape[0] - unique.size
    if n > 0:
        temp = np.concatenate([temp, temp[-1] + extra[:n]], axis=0)
    return temp


def dmc_blocks(net, params, ecp, x0, e_l0, nblocks: int, iterations: int, tstep: float, feedback: float,
               step_draws, block_draws):
    """main_dmc.py:113-244 on one device.  e_l0: the pp energies of x0 (total_e); step_draws(k) ->
    the draws of step k; block_draws(block) -> (u_comb, extra [B,3N])."""
    B = x0.shape[0]
    x = np.asarray(x0, np.float64)
    e_trial = e_est = np.asarray(e_l0)
    esigma = float(np.std(np.asarray(e_l0)))                       # :118 (complex std)
    weights = np.ones(B)
    branchcut = 10.0 * esigma                                       # :137 branchcut_start * esigma
    energy_data = np.zeros((nblocks, iterations, B))
    weights_data = np.zeros((nblocks, iterations, B))
    trace = {"energy": [], "weights": [], "positions": [], "newinds": [], "comb_weight": [], "e_est": [],
             "e_trial": []}
    k = 0
    for block in range(nblocks):
        for t in range(iterations):
            eloc, weights, xt, _ = dmc_step(net, params, ecp, torch.tensor(x), weights, e_trial, e_est, branchcut,
                                            step_draws(k), tstep)
            k += 1
            x = xt.numpy()
            energy_data[block, t] = eloc.real
            weights_data[block, t] = weights
            trace["energy"].append(eloc)
            trace["weights"].append(weights)
            trace["positions"].append(x)
        e_est = np.average(energy_data, weights=weights_data)          # :190
        u, extra = block_draws(block)
        wn, newinds = branch(weights, u)                               # :202
        weights = np.full(B, wn)
        x = reindex(x, newinds, extra)
        e_trial = e_est - feedback * np.log(np.mean([wn])).real        # :237
        trace["newinds"].append(newinds)
        trace["comb_weight"].append(wn)
        trace["e_est"].append(e_est)
        trace["e_trial"].append(e_trial)
    return trace, x, weights


def dmc_blocks_devices(net, params, ecp, x0, e_l0, nblocks: int, iterations: int, tstep: float, feedback: float,
                       step_draws, block_draws, ndev: int):
    """main_dmc.py:113-244 with the walkers split over `ndev` devices in contiguous blocks (the
    pmapped driver, main_dmc.py:86-97): per device its own T-moves, drift-diffusion (tdamp is a
    per-device ratio, drift_diffusion.py:21) and comb (branch.py under pmap, one uniform per
    device); global over devices: esigma = jnp.std over every walker (:118), the comput_S energy
    cut = ONE min over the stacked [ndev, B] |e_est - E_L| arrays and the branch cut (S_matrix.py
    :10-12 on the gathered arrays), the block estimate (:190) and the e_trial feedback = log of
    the mean over devices of the comb weights (:237).  block_draws(block) -> [(u_comb,
    extra)] * ndev; step_draws(k) -> draws of all walkers (device d takes its rows)."""
    B = x0.shape[0]
    Bd = B // ndev
    sl = [slice(d * Bd, (d + 1) * Bd) for d in range(ndev)]
    x = np.asarray(x0, np.float64)
    N = x.shape[1] // 3
    e_trial = e_est = np.asarray(e_l0)
    esigma = float(np.std(np.asarray(e_l0)))
    branchcut = 10.0 * esigma
    weights = np.ones(B)
    energy_data = np.zeros((nblocks, iterations, B))
    weights_data = np.zeros((nblocks, iterations, B))
    trace = {"energy": [], "weights": [], "positions": [], "newinds": [], "comb_weight": [], "e_est": [],
             "e_trial": []}
    pick = lambda v, d: v[sl[d]] if np.ndim(v) else v
    k = 0
    from . import pphamiltonian as pp
    for block in range(nblocks):
        for t in range(iterations):
            dr = step_draws(k)
            k += 1
            parts = []
            for d in range(ndev):
                dd = {key: np.asarray(v)[sl[d]] for key, v in dr.items()}
                xd = torch.tensor(x[sl[d]])
                pos_t = torch.stack([tmoves(net, params, ecp, xd[b], dd["rot_tm"][b], float(dd["u_sel"][b]),
                                            dd["u_acc"][b], tstep)[0] for b in range(Bd)])
                x_new, tdamp, go, gn = drift_diffusion(net, params, pos_t, torch.as_tensor(dd["gauss1"]),
                                                       torch.as_tensor(dd["gauss2"]), torch.as_tensor(dd["u"]), tstep)
                eo = pp.batch_local_energy_pp(net, params, ecp, xd, dd["rot_old"])[0].detach().numpy()
                en = pp.batch_local_energy_pp(net, params, ecp, x_new, dd["rot_new"])[0].detach().numpy()
                parts.append((x_new.numpy(), float(tdamp), go.numpy(), gn.numpy(), eo, en))
            cut = {}
            for which, col in (("old", 4), ("new", 5)):
                m = min(float(np.min(np.abs(np.real(pick(e_est, d)) - np.real(parts[d][col])))) for d in range(ndev))
                cut[which] = min(m, branchcut)
            w_new = np.empty(B)
            eloc = np.empty(B, complex)
            xn = np.empty_like(x)
            for d in range(ndev):
                x_new, tdamp, go, gn, eo, en = parts[d]

                def S(v2, el, c):
                    v2 = np.sum(v2, axis=-1)
                    el = np.real(el)
                    e_cut = c * np.sign(np.real(pick(e_est, d)) - el)
                    return np.real(pick(e_trial, d)) - np.real(pick(e_est, d)) + e_cut / (1 + (v2 * tstep / N) ** 2)
                s_old = S(go ** 2, eo, cut["old"])
                s_new = S(gn ** 2, en, cut["new"])
                w_new[sl[d]] = update_weights(weights[sl[d]], tstep, tdamp, s_new, s_old)
                eloc[sl[d]] = en
                xn[sl[d]] = x_new
            weights = w_new
            x = xn
            energy_data[block, t] = eloc.real
            weights_data[block, t] = weights
            trace["energy"].append(eloc)
            trace["weights"].append(weights.copy())
            trace["positions"].append(x.copy())
        e_est = np.average(energy_data[:block + 1], weights=weights_data[:block + 1])
        wns, inds = [], []
        bd = block_draws(block)
        for d in range(ndev):
            u, extra = bd[d]
            wn, newinds = branch(weights[sl[d]], u)
            wns.append(wn)
            inds.append(newinds)
            x[sl[d]] = reindex(x[sl[d]], newinds, extra)
            weights[sl[d]] = wn
        e_trial = e_est - feedback * np.log(np.mean(wns)).real
        trace["newinds"].append(np.stack(inds))
        trace["comb_weight"].append(np.array(wns))
        trace["e_est"].append(e_est)
        trace["e_trial"].append(e_trial)
    return trace, x, weights
