"""Energy loss with the unbiased energy gradient (drop-in for AIQMCrelease3/Loss/loss.py:73-272).

``make_loss(network, local_energy, clip_local_energy, clip_from_median,
center_at_clipped_energy, complex_output)`` returns ``total_energy(params, key, data) ->
(loss, AuxiliaryLossData)``; the reference differentiates it with ``jax.value_and_grad``
through a custom JVP (:220-270).  Here the derivative is explicit:
``total_energy.value_and_grad(params, key, data) -> ((loss, aux), grad_tree)``, with

    grad = (2 / B) sum_b [ Re(diff_b) d log|psi_b| / d theta + Im(cl_b) d phase_b / d theta ]

the custom-JVP tangent (term1 - 2 term2).real / B of :256-265 with psi_tangent = d(log|psi| +
i phase) (complex_output=True; diff = clipped local energy minus its centre, :73-135;
cl = diff + aux.clipped_energy, which is the clip centre when clipping and E_L itself when
not -- kept as written).  For real E_L the phase term vanishes.  complex_output=False uses the
reference's dot(psi_tangent, diff) / B (factor 1/B, not 2/B).  Both terms are weighted
device reductions of the per-walker parameter gradients (aiqmc_logpsi_param_grad,
aiqmc_phase_param_grad).  The optimizer pmeans the result over ranks (adam.py:55).

``total_energy.value_and_pmean_grad`` returns the gradient already pmean'd over ranks.  With
several ranks its statistics, clipping and the gradient pmean take THREE packed all-reduces per
step (``fused_levels``: [Chan 6-vector] -> [TV sums] -> [clipped sums, G, G0]) instead of the
reference's chain of pmeans (loss.py:107 twice, :206, :208, adam.py:55), with no host
synchronisation.
"""
from __future__ import annotations

import dataclasses
from typing import Any, Optional

import numpy as np
import torch

from .. import constants


# diagnostics: False routes every step through the torch statistics path (the A/B of the fused
# single-rank path, tools/adam_only.py AIQMC_LOSS_TORCH=1)
FUSED_ONE_RANK = True


@dataclasses.dataclass
class AuxiliaryLossData:
    """loss.py:28-41.  imag_check (not in the reference): a device count of local energies with a
    nonzero imaginary part when complex energies met complex_output=False; checked (one host
    read) by check_real_energies, which make_training_step calls after its NaN check."""
    variance: Any
    local_energy: Any
    clipped_energy: Any
    grad_local_energy: Any = None
    local_energy_mat: Any = None
    imag_check: Any = None


def check_real_energies(aux: AuxiliaryLossData) -> None:
    """Raise if complex local energies with a nonzero imaginary part met complex_output=False
    (the deferred form of the reference's shape/dtype error, loss.py:256-265)."""
    chk = getattr(aux, "imag_check", None)
    if chk is not None and int(chk) > 0:
        raise NotImplementedError("complex local energies need complex_output=True (loss.py:256-265)")


def _host_level(level, er, ei, L1=None, L2=None, clip=0.0, wscale=1.0, g0=False, want_phase=False):
    """The level vectors of aiqmc_loss_level restated in torch float64 (host/gloo ranks; the
    device path runs the HIP kernels).  Same formulas, csrc/aiqmc.hip k_lossr_*."""
    x = er.to(torch.float64)
    y = ei.to(torch.float64) if ei is not None else torch.zeros_like(x)
    n = float(x.numel())
    if level == 1:
        mr, mi = x.mean(), y.mean()
        m2 = ((x - mr) ** 2 + (y - mi) ** 2).sum()
        nz = (y != 0).sum().to(torch.float64)
        return torch.stack([m2, n * mr, n * mi, n * mr * mr + n * mi * mi,
                            torch.full((), n, dtype=torch.float64, device=x.device), nz])
    mr, mi, _ = _mean_var(L1)
    if level == 2:
        return torch.stack([(x - mr).abs().sum(), (y - mi).abs().sum()])
    if clip > 0.0:
        ntot = L1[4]
        tvr, tvi = L2[0] / ntot, L2[1] / ntot
        xc = torch.minimum(torch.maximum(x, mr - clip * tvr), mr + clip * tvr)
        yc = torch.minimum(torch.maximum(y, mi - clip * tvi), mi + clip * tvi)
        wp = wscale * yc
    else:
        xc, yc = x, y
        wp = wscale * ((y - mi) + y)
    w = [wscale * (xc - mr)]
    if g0:
        w.append(torch.full_like(x, wscale))
    dt = er.dtype
    return (torch.stack(w).to(dt), wp.to(dt) if want_phase else None, xc.to(dt),
            yc.to(dt) if ei is not None else None, torch.stack([xc.sum(), yc.sum()]))


def _mean_var(L1):
    ntot = L1[4]
    mr, mi = L1[1] / ntot, L1[2] / ntot
    between = torch.clamp(L1[3] - ntot * mr * mr - ntot * mi * mi, min=0.0)
    return mr, mi, (L1[0] + between) / ntot


def fused_levels(e_l: torch.Tensor, grad_fn, clip_local_energy: float, center_at_clipped_energy: bool,
                 complex_output: bool):
    """Energy statistics, clipping and the pmean'd energy gradient over all ranks with one packed
    all-reduce per dependency level (loss.py:73-135,206-208,256-265; adam.py:55):

      L1 = [sum |e - m_r|^2, n m_r (re, im), n |m_r|^2, n, #Im!=0]   -> E, variance (Chan)
      L2 = [sum |Re e - Re E|, sum |Im e - Im E|]                     -> TV window (clipping only)
      L3 = [sum xc (re, im), G, G0]                                   -> dc, grad
      grad = (G - (Re dc - Re E) G0) / world,  G = sum_b wscale (Re xc_b - Re E) dlog|psi_b|
             + sum_b wp_b dphase_b,  G0 = sum_b wscale dlog|psi_b|   (G0 only when centring at
             the clipped mean: the reference's weights wscale Re(xc_b - dc) = G's minus the constant
             Re dc - Re E, so the clipped mean rides in the gradient's all-reduce).

    grad_fn(w [K, B], wp [B] or None) -> (G [K, P], Gp [P] or None): the weighted parameter
    gradients of this rank's walkers.  Returns (loss, variance, clipped_energy, grad, imag_count).
    Device energies run the HIP level kernels (aiqmc_loss_level / _pack / _final); host energies
    the same formulas in torch.
    """
    cplx = torch.is_complex(e_l)
    er = (e_l.real if cplx else e_l).contiguous().reshape(-1)
    ei = e_l.imag.contiguous().reshape(-1) if cplx else None
    phase = cplx and complex_output
    B = er.numel()
    wscale = (2.0 if complex_output else 1.0) / B
    clipping = clip_local_energy > 0.0
    g0 = clipping and center_at_clipped_energy
    world = constants.world_size()
    dev = er.is_cuda and er.dtype in (torch.float32, torch.float64)
    if dev:
        from .. import _lib
        level = lambda *a, **k: _lib.loss_level(*a, **k)
    else:
        level = _host_level
    L1 = constants.all_reduce_(level(1, er, ei))
    L2 = constants.all_reduce_(level(2, er, ei, L1)) if clipping else None
    w, wp, cr, ci, head = level(3, er, ei, L1, L2, clip_local_energy, wscale, g0, phase)
    G, Gp = grad_fn(w, wp if phase else None)
    P = G.shape[1]
    if dev:
        L3 = constants.all_reduce_(_lib.loss_pack(G[0], Gp, G[1] if g0 else None, head))
        grad, stats = _lib.loss_final(L1, L3, P, g0, center_at_clipped_energy and clipping, world, G.dtype)
        mr, mi, var, imag = stats[0], stats[1], stats[2], stats[5]
    else:
        Gs = G[0].to(torch.float64) + (Gp.to(torch.float64) if Gp is not None else 0.0)
        parts = [head, Gs] + ([G[1].to(torch.float64)] if g0 else [])
        L3 = constants.all_reduce_(torch.cat(parts))
        mr, mi, var = _mean_var(L1)
        imag = L1[5]
        shift = (L3[0] / L1[4] - mr) if g0 else 0.0
        g = L3[2:2 + P] - (shift * L3[2 + P:2 + 2 * P] if g0 else 0.0)
        grad = (g / world).to(G.dtype)
    rdt = er.dtype
    loss = torch.complex(mr.to(rdt), mi.to(rdt)) if cplx else mr.to(rdt)
    clipped = (torch.complex(cr, ci) if cplx else cr).reshape(e_l.shape)
    return loss, var.to(rdt), clipped, grad, imag


def clip_local_values(local_values: torch.Tensor, mean_local_values: torch.Tensor, clip_scale: float,
                      clip_from_median: bool, center_at_clipped_value: bool, complex_output: bool = False):
    """loss.py:73-135: (diff_center, diff) with the total-variation window (pmean'd)."""
    batch_mean = lambda v: constants.pmean(torch.mean(v))

    def clip_at_total_variation(values, center, scale):
        tv = batch_mean(torch.abs(values - center))
        return torch.clamp(values, center - scale * tv, center + scale * tv)

    if clip_from_median:
        # jnp.median: the mean of the two middle values for an even count (torch.median would
        # return the lower one)
        center = torch.quantile(constants.all_gather(local_values).real.reshape(-1), 0.5)
    else:
        center = mean_local_values
    if torch.is_complex(local_values):
        # the median centre is real (.real before the median); JAX's .imag of a real array is 0
        c_re = center.real if torch.is_complex(center) else center
        c_im = center.imag if torch.is_complex(center) else torch.zeros_like(center)
        clipped = torch.complex(clip_at_total_variation(local_values.real, c_re, clip_scale),
                                clip_at_total_variation(local_values.imag, c_im, clip_scale))
    else:
        clipped = clip_at_total_variation(local_values, center, clip_scale)
    diff_center = batch_mean(clipped) if center_at_clipped_value else mean_local_values
    return diff_center, clipped - diff_center


def _unflatten_like(template, flat):
    """The tree of `template` with leaves cut from `flat` (numpy -> numpy leaves; a device tensor
    -> views of it on the device, so an optimiser step never leaves the GPU)."""
    shapes = []

    def collect(tree):
        if isinstance(tree, dict):
            for k in sorted(tree.keys()):
                collect(tree[k])
        elif isinstance(tree, (list, tuple)):
            for v in tree:
                collect(v)
        else:
            shapes.append(tuple(tree.shape) if hasattr(tree, "shape") else np.shape(tree))
    collect(template)
    sizes = [int(np.prod(sh)) if sh else 1 for sh in shapes]
    if isinstance(flat, torch.Tensor):
        # one split (views) + a view per leaf; each stays a view of `flat`, which nn.bind and the
        # optimiser recognise and use whole (no gather)
        pieces = iter([p.view(sh) for p, sh in zip(torch.split(flat, sizes), shapes)])
    else:
        offs = np.cumsum([0] + sizes)
        pieces = iter([flat[offs[i]:offs[i + 1]].reshape(sh) for i, sh in enumerate(shapes)])

    def build(tree):
        if isinstance(tree, dict):
            return {k: build(tree[k]) for k in sorted(tree.keys())}
        if isinstance(tree, (list, tuple)):
            return [build(v) for v in tree]
        return next(pieces)
    return build(template)


def make_loss(network, local_energy, clip_local_energy: float = 0.0, clip_from_median: bool = True,
              center_at_clipped_energy: bool = True, complex_output: bool = False):
    """loss.py:138-272.  `network` is the (log) network closure of the driver; the AIQMC
    network whose parameters are differentiated is taken from it or from `local_energy`."""
    net = getattr(network, "_aiqmc_network", None) or getattr(local_energy, "_aiqmc_network", None)
    if net is None:
        raise TypeError("make_loss: local_energy must come from aiqmc.Energy (it carries the HIP network)")

    def _energy(params, key, data):
        e_l, e_mat = local_energy(params, key, data)
        loss = constants.pmean(torch.mean(e_l))
        d = e_l - loss
        variance = constants.pmean(torch.mean(d * torch.conj(d))).real
        return e_l, e_mat, loss, variance

    def total_energy(params, key, data):
        e_l, e_mat, loss, variance = _energy(params, key, data)
        return loss, AuxiliaryLossData(variance=variance, local_energy=e_l, clipped_energy=e_l,
                                       local_energy_mat=e_mat)

    def value_and_grad_fused(params, data, e_l, e_mat):
        """One rank, device energies: the statistics, the clipping and the two weight vectors in
        one launch (aiqmc_loss_weights, the same formulas in double), then the parameter
        gradients -- no host synchronisation and ~25 small torch launches fewer per step."""
        from .. import _lib
        cplx = torch.is_complex(e_l)
        # checked after the step (check_real_energies): no host read here
        imag_check = torch.count_nonzero(e_l.imag) if cplx and not complex_output else None
        phase = cplx and complex_output
        B = e_l.numel()
        wscale = (2.0 if complex_output else 1.0) / B
        w, wp, clipped, st = _lib.loss_weights(e_l, clip_local_energy, center_at_clipped_energy, wscale, phase)
        rdt = e_l.real.dtype if cplx else e_l.dtype
        loss = torch.complex(st[0], st[1]).to(e_l.dtype) if cplx else st[0].to(rdt)
        variance = st[2].to(rdt)
        pos = data.positions if isinstance(data.positions, torch.Tensor) else torch.as_tensor(
            np.asarray(data.positions))
        dtype = pos.dtype if pos.dtype in (torch.float32, torch.float64) else torch.float32
        ctx = net.bind(params, data.atoms, dtype)
        g = ctx.logpsi_param_grad(pos.reshape(B, -1), weights=w.to(ctx.device, dtype))
        if phase:
            g = g + ctx.phase_param_grad(pos.reshape(B, -1), weights=wp.to(ctx.device, dtype))
        aux = AuxiliaryLossData(variance=variance, local_energy=e_l, clipped_energy=clipped, local_energy_mat=e_mat,
                                imag_check=imag_check)
        return (loss, aux), g

    def _device_energies(e_l):
        return (isinstance(e_l, torch.Tensor) and e_l.is_cuda
                and (e_l.real if torch.is_complex(e_l) else e_l).dtype in (torch.float32, torch.float64))

    # the median centre needs an all_gather (loss.py:118-121); without clipping it is never used
    _mean_centre = clip_local_energy <= 0.0 or not clip_from_median

    def value_and_grad(params, key, data):
        e_l, e_mat = local_energy(params, key, data)
        return _value_and_grad(params, data, e_l, e_mat)

    def _value_and_grad(params, data, e_l, e_mat):
        if FUSED_ONE_RANK and not constants._active() and _mean_centre and _device_energies(e_l):
            return value_and_grad_fused(params, data, e_l, e_mat)
        loss = constants.pmean(torch.mean(e_l))
        d = e_l - loss
        variance = constants.pmean(torch.mean(d * torch.conj(d))).real
        # complex energies with complex_output=False: the imaginary parts must vanish (checked after
        # the step, check_real_energies); the real parts carry the loss
        imag_check = torch.count_nonzero(e_l.imag) if torch.is_complex(e_l) and not complex_output else None
        cplx = torch.is_complex(e_l) and complex_output
        e_c = e_l if cplx else (e_l.real if torch.is_complex(e_l) else e_l)
        loss_c = loss if cplx else (loss.real if torch.is_complex(loss) else loss)
        if clip_local_energy > 0.0:
            center, diff = clip_local_values(e_c, loss_c, clip_local_energy, clip_from_median,
                                             center_at_clipped_energy)
            aux_clipped = center                      # aux_data.clipped_energy (loss.py:240-246)
        else:
            center, diff = loss_c, e_c - loss_c
            aux_clipped = e_c                         # total_energy's clipped_energy = e_l
        pos = data.positions if isinstance(data.positions, torch.Tensor) else torch.as_tensor(
            np.asarray(data.positions))
        dtype = pos.dtype if pos.dtype in (torch.float32, torch.float64) else torch.float32
        ctx = net.bind(params, data.atoms, dtype)
        B = diff.numel()
        scale = (2.0 if complex_output else 1.0) / B
        d_re = diff.real if torch.is_complex(diff) else diff
        w = scale * d_re.reshape(-1).to(ctx.device, dtype)
        g = ctx.logpsi_param_grad(pos.reshape(B, -1), weights=w)     # loss.py:256-265
        if cplx:
            cl = diff + aux_clipped
            wp = scale * cl.imag.reshape(-1).to(ctx.device, dtype)
            g = g + ctx.phase_param_grad(pos.reshape(B, -1), weights=wp)
        aux = AuxiliaryLossData(variance=variance, local_energy=e_l, clipped_energy=center + diff,
                                local_energy_mat=e_mat, imag_check=imag_check)
        return (loss, aux), g

    def value_and_pmean_grad(params, key, data):
        """value_and_grad followed by the optimizer's gradient pmean (adam.py:55).  Several ranks
        (or forced collectives) with a mean clip centre: fused_levels, 3 all-reduces per step."""
        e_l, e_mat = local_energy(params, key, data)
        if not (constants._active() and _mean_centre and isinstance(e_l, torch.Tensor)):
            (loss, aux), g = _value_and_grad(params, data, e_l, e_mat)
            return (loss, aux), constants.pmean(g)
        pos = data.positions if isinstance(data.positions, torch.Tensor) else torch.as_tensor(
            np.asarray(data.positions))
        dtype = pos.dtype if pos.dtype in (torch.float32, torch.float64) else torch.float32
        ctx = net.bind(params, data.atoms, dtype)
        B = e_l.numel()
        x = pos.reshape(B, -1)

        def grad_fn(w, wp):
            G = ctx.param_grad_weighted(x, w)
            Gp = ctx.param_grad_weighted(x, wp[None], phase=True)[0] if wp is not None else None
            return G, Gp

        loss, variance, clipped, g, imag = fused_levels(e_l, grad_fn, clip_local_energy, center_at_clipped_energy,
                                                        complex_output)
        imag_check = imag if torch.is_complex(e_l) and not complex_output else None
        aux = AuxiliaryLossData(variance=variance, local_energy=e_l, clipped_energy=clipped, local_energy_mat=e_mat,
                                imag_check=imag_check)
        return (loss, aux), g

    total_energy.value_and_grad = value_and_grad
    total_energy.value_and_pmean_grad = value_and_pmean_grad
    total_energy.unflatten = lambda params, flat: _unflatten_like(params, flat)
    total_energy._aiqmc_network = net
    return total_energy
