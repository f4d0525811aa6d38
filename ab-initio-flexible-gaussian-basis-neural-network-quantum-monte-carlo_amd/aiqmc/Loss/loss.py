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
    """loss.py:28-41."""
    variance: Any
    local_energy: Any
    clipped_energy: Any
    grad_local_energy: Any = None
    local_energy_mat: Any = None


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
        if cplx and not complex_output and bool(torch.any(e_l.imag != 0)):
            raise NotImplementedError("complex local energies need complex_output=True (loss.py:256-265)")
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
        aux = AuxiliaryLossData(variance=variance, local_energy=e_l, clipped_energy=clipped, local_energy_mat=e_mat)
        return (loss, aux), g

    def value_and_grad(params, key, data):
        e_l, e_mat = local_energy(params, key, data)
        if (FUSED_ONE_RANK and not constants._active() and not clip_from_median and isinstance(e_l, torch.Tensor)
                and e_l.is_cuda
                and (e_l.real if torch.is_complex(e_l) else e_l).dtype in (torch.float32, torch.float64)):
            return value_and_grad_fused(params, data, e_l, e_mat)
        loss = constants.pmean(torch.mean(e_l))
        d = e_l - loss
        variance = constants.pmean(torch.mean(d * torch.conj(d))).real
        cplx = torch.is_complex(e_l) and bool(torch.any(e_l.imag != 0))
        if cplx and not complex_output:
            raise NotImplementedError("complex local energies need complex_output=True (loss.py:256-265)")
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
                                local_energy_mat=e_mat)
        return (loss, aux), g

    total_energy.value_and_grad = value_and_grad
    total_energy.unflatten = lambda params, flat: _unflatten_like(params, flat)
    total_energy._aiqmc_network = net
    return total_energy
