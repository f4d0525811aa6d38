"""Energy-gradient and Adam oracle (TEST INFRASTRUCTURE ONLY, float64, CPU).

Restates ``AIQMCrelease3/Loss/loss.py:73-272`` (total_energy, clip_local_values, the
custom-JVP energy gradient) and ``Optimizer/adam.py:49-81`` with the optax chain of
``main/main_all_electrons_adam_muti_GPU.py:152-158`` (scale_by_adam(b1=0.9, b2=0.999,
eps=1e-8, eps_root=0), scale_by_schedule(0.05 (1 + t)^-10000), scale(-1)).  optax is absent
here; its scale_by_adam / scale_by_schedule are restated from their published algorithm
(bias-corrected first/second moments with count+1; the schedule evaluated at the pre-update
count).  pmean over one device is the identity.

Parameter derivatives: ``torch.func.grad`` of the oracle network's log|psi| wrt the
parameter tree (the reference differentiates the same function with jax.jvp inside the
custom JVP, loss.py:256-258).
"""
from __future__ import annotations

import math

import numpy as np
import torch
from torch.func import grad

from . import network, system


def logabs_param_grad(net, params_np, pos: torch.Tensor) -> np.ndarray:
    """[B, P] d log|psi(x_b)| / d theta, canonical tree_flatten order (unused leaves 0)."""
    pt = network.to_torch(params_np)
    g = grad(lambda p, x: net.logabs(p, x))
    rows = []
    for b in range(pos.shape[0]):
        gt = g(pt, pos[b])
        rows.append(system.flatten_params(system.map_tree(lambda t: t.detach().numpy(), gt)))
    return np.stack(rows)


def clip_local_values(e, mean_e, clip_scale, clip_from_median=False, center_at_clipped_value=True):
    """loss.py:73-135 (real local energies, one device)."""
    if clip_from_median:
        center = np.median(e)
    else:
        center = mean_e
    tv = np.mean(np.abs(e - center))
    clipped = np.clip(e, center - clip_scale * tv, center + clip_scale * tv)
    diff_center = np.mean(clipped) if center_at_clipped_value else mean_e
    return diff_center, clipped - diff_center


def energy_gradient(e_l: np.ndarray, O: np.ndarray, clip_scale: float = 5.0, clip_from_median: bool = False,
                    center_at_clipped_energy: bool = True):
    """loss.py:220-270 with complex_output=True and real E_L (the all-electron driver):
    tangent = (term1 - 2 term2).real / B with term1 = 2 Re(clipped . conj(psi_t)),
    term2 = sum(diff_center * Re psi_t)  ==  (2/B) sum_b diff_b O_b."""
    loss = float(np.mean(e_l))
    variance = float(np.mean((e_l - loss) ** 2))
    if clip_scale > 0:
        center, diff = clip_local_values(e_l, loss, clip_scale, clip_from_median, center_at_clipped_energy)
    else:
        center, diff = loss, e_l - loss
    clipped = diff + center
    B = e_l.shape[0]
    term1 = 2.0 * (clipped @ O)
    term2 = center * O.sum(axis=0)
    return loss, variance, (term1 - 2.0 * term2) / B


def lr_schedule(t, rate=0.05, delay=1.0, decay=10000):
    """main_all_electrons_adam_muti_GPU.py:152-153."""
    return rate * (1.0 / (1.0 + (t / delay))) ** decay


class Adam:
    """optax.chain(scale_by_adam(0.9, 0.999, 1e-8, 0), scale_by_schedule(lr), scale(-1))."""

    def __init__(self, n, b1=0.9, b2=0.999, eps=1e-8, eps_root=0.0, schedule=lr_schedule):
        self.m = np.zeros(n)
        self.v = np.zeros(n)
        self.count = 0
        self.b1, self.b2, self.eps, self.eps_root, self.schedule = b1, b2, eps, eps_root, schedule

    def update(self, g: np.ndarray, params: np.ndarray) -> np.ndarray:
        self.m = self.b1 * self.m + (1 - self.b1) * g
        self.v = self.b2 * self.v + (1 - self.b2) * g * g
        c = self.count + 1
        mh = self.m / (1 - self.b1 ** c)
        vh = self.v / (1 - self.b2 ** c)
        u = mh / (np.sqrt(vh + self.eps_root) + self.eps)
        u = u * self.schedule(self.count)
        self.count += 1
        return params - u


def phase_param_grad(net, params_np, pos: torch.Tensor) -> np.ndarray:
    """[B, P] d phase(x_b) / d theta (phase = arg det, the imaginary part of the complex log
    the pp drivers differentiate, main_pp_adam_muti_GPU.py:119-121), canonical order."""
    pt = network.to_torch(params_np)
    g = grad(lambda p, x: net.apply(p, x)[0])
    rows = []
    for b in range(pos.shape[0]):
        gt = g(pt, pos[b])
        rows.append(system.flatten_params(system.map_tree(lambda t: t.detach().numpy(), gt)))
    return np.stack(rows)


def phase_param_grad_fd(net, params_np, pos: torch.Tensor, h: float = 1e-6) -> np.ndarray:
    """Central finite differences of the phase wrt every canonical parameter (pins the above)."""
    flat = system.flatten_params(params_np)
    rows = np.zeros((pos.shape[0], flat.size))
    for k in range(flat.size):
        for sgn in (1.0, -1.0):
            f = flat.copy()
            f[k] += sgn * h
            pt = network.to_torch(system.unflatten_params(params_np, f))
            ph = np.array([net.apply(pt, pos[b])[0].item() for b in range(pos.shape[0])])
            rows[:, k] += sgn * ph / (2 * h)
    return rows


def energy_gradient_complex(e_l: np.ndarray, O_abs: np.ndarray, O_phase: np.ndarray, clip_scale: float = 5.0,
                            clip_from_median: bool = False, center_at_clipped_energy: bool = True,
                            complex_output: bool = True):
    """loss.py:220-270 literally, for complex E_L and psi_tangent = O_abs + i O_phase
    (network = the complex log of the pp drivers): returns (loss, grad [P])."""
    e_l = np.asarray(e_l, dtype=np.complex128)
    loss = np.mean(e_l)
    if clip_scale > 0:
        center = np.median(e_l.real) if clip_from_median else loss
        tv_r = np.mean(np.abs(e_l.real - center.real))
        tv_i = np.mean(np.abs(e_l.imag - np.imag(center)))
        clipped = (np.clip(e_l.real, center.real - clip_scale * tv_r, center.real + clip_scale * tv_r)
                   + 1j * np.clip(e_l.imag, np.imag(center) - clip_scale * tv_i, np.imag(center) + clip_scale * tv_i))
        diff_center = np.mean(clipped) if center_at_clipped_energy else loss
        aux_clipped, diff = diff_center, clipped - diff_center
    else:
        aux_clipped, diff = e_l, e_l - loss
    B = e_l.shape[0]
    psi_t = O_abs + 1j * O_phase                                   # [B, P]
    if complex_output:
        clipped_el = diff + aux_clipped
        term1 = clipped_el @ np.conj(psi_t) + np.conj(clipped_el) @ psi_t
        term2 = (aux_clipped * np.ones(B)) @ psi_t.real
        return loss.real, (term1 - 2 * term2).real / B
    return loss, (diff @ psi_t) / B
