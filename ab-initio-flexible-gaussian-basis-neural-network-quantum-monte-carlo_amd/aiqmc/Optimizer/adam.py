"""Adam training step (drop-in for AIQMCrelease3/Optimizer/adam.py:49-81).

``make_opt_update_step(evaluate_loss, optimizer)`` -> ``opt_update(params, data, opt_state,
key) -> (params, opt_state, loss, aux)``: the energy gradient of ``evaluate_loss`` (aiqmc
Loss.make_loss, computed on the GPU), pmean'd over ranks (adam.py:55: in the last of the loss
statistics' three packed RCCL all-reduces, Loss.loss.fused_levels), then the optimizer
(Optimizer.optax_like).
``make_training_step(opt_update)`` adds the NaN rollback of adam.py:74-79.  Parameters stay a
reference-shaped pytree; the optimizer runs on the flat device vector and the new leaves are
device tensors (views of it), so a training step makes no host round trip of the parameters
(the next bind repacks them on the device, aiqmc_set_params_device).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..Loss.loss import check_real_energies
from ..wavefunction_Ynlm.nn import flatten_params_device


def make_opt_update_step(evaluate_loss, optimizer):
    vg = getattr(evaluate_loss, "value_and_pmean_grad", None)
    if vg is None:
        raise TypeError("evaluate_loss must come from aiqmc.Loss.loss.make_loss")

    def opt_update(params, data, opt_state, key):
        # the gradient comes back pmean'd (adam.py:55): with several ranks it rides in the loss
        # statistics' last all-reduce (Loss.loss.fused_levels)
        (loss, aux), grad = vg(params, key, data)
        flat = flatten_params_device(params, grad.device).to(grad.dtype)
        if opt_state is None:
            opt_state = optimizer.init(flat)
        updates, opt_state = optimizer.update(grad, opt_state, flat)
        # the new parameters stay on the device as views of one float64 vector (the reference's
        # params are device arrays): the next bind repacks them there (aiqmc_set_params_device)
        new_flat = (flat + updates).detach().to(torch.float64)
        return evaluate_loss.unflatten(params, new_flat), opt_state, loss, aux
    return opt_update


def make_training_step(optimizer_step):
    """adam.py:62-81: one optimisation step; parameters/state roll back if the loss is NaN."""

    def step(data, params, state, key):
        new_params, new_state, loss, aux = optimizer_step(params, data, state, key)
        if math.isnan(float(loss.real if torch.is_complex(loss) else loss)):
            return data, params, state, loss, aux
        check_real_energies(aux)
        return data, new_params, new_state, loss, aux
    return step
