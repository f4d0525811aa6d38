"""The optax transformations the reference's Adam drivers chain
(main_all_electrons_adam_muti_GPU.py:152-158): scale_by_adam, scale_by_schedule, scale,
chain, apply_updates -- restated on flat device tensors (optax is not a dependency here).
Semantics follow optax: bias correction with count + 1; the schedule is evaluated at the
pre-update count; states count from 0."""
from __future__ import annotations

import dataclasses
from typing import Any, Callable, List

import torch


@dataclasses.dataclass
class GradientTransformation:
    init: Callable
    update: Callable


def scale_by_adam(b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8, eps_root: float = 0.0):
    def init(params: torch.Tensor):
        return {"count": 0, "mu": torch.zeros_like(params), "nu": torch.zeros_like(params)}

    def update(g, state, params=None):
        mu = b1 * state["mu"] + (1 - b1) * g
        nu = b2 * state["nu"] + (1 - b2) * g * g
        c = state["count"] + 1
        mh = mu / (1 - b1 ** c)
        vh = nu / (1 - b2 ** c)
        return mh / (torch.sqrt(vh + eps_root) + eps), {"count": c, "mu": mu, "nu": nu}
    return GradientTransformation(init, update)


def scale_by_schedule(fn: Callable[[Any], float]):
    def init(params):
        return {"count": 0}

    def update(u, state, params=None):
        return u * float(fn(state["count"])), {"count": state["count"] + 1}
    return GradientTransformation(init, update)


def scale(s: float):
    return GradientTransformation(lambda p: {}, lambda u, st, params=None: (u * s, st))


def chain(*ts: GradientTransformation):
    def init(params):
        return [t.init(params) for t in ts]

    def update(u, states: List, params=None):
        out = []
        for t, st in zip(ts, states):
            u, st = t.update(u, st, params)
            out.append(st)
        return u, out
    return GradientTransformation(init, update)


def apply_updates(params: torch.Tensor, updates: torch.Tensor) -> torch.Tensor:
    return params + updates
