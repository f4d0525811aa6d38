"""Cross-device collectives (AIQMCrelease3/constants.py:5-9) over torch.distributed.

The reference's ``pmean``/``psum``/``all_gather`` act over the JAX pmap axis
'qmc_pmap_axis' and are identities outside pmap.  Here one process drives one
GPU; the collectives run over the default process group (RCCL over xGMI when
initialised with backend "nccl", gloo on CPU) and are identities when no group
is initialised.  ``pmean_stats`` fuses the energy statistics of one iteration
(loss.py:206,208) into a single all-reduce.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

PMAP_AXIS_NAME = 'qmc_pmap_axis'


def _active() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def psum(x: torch.Tensor) -> torch.Tensor:
    if not _active():
        return x
    y = x.clone()
    dist.all_reduce(y, op=dist.ReduceOp.SUM)
    return y


def pmean(x: torch.Tensor) -> torch.Tensor:
    if not _active():
        return x
    return psum(x) / dist.get_world_size()


def all_gather(x: torch.Tensor) -> torch.Tensor:
    if not _active():
        return x[None]
    out = [torch.empty_like(x) for _ in range(dist.get_world_size())]
    dist.all_gather(out, x.contiguous())
    return torch.stack(out)


def pmean_stats(e_l: torch.Tensor):
    """(mean E, variance) over all walkers of all ranks with ONE all-reduce.

    Same quantities as loss.py:206-208 (pmean(mean(e)), pmean(mean(|e-E|^2)))
    for equal per-device batches; accumulated in float64.
    """
    e = e_l.to(torch.float64)
    v = torch.stack([e.sum(), (e * e).sum(), torch.tensor(float(e.numel()), dtype=torch.float64,
                                                          device=e.device)])
    v = psum(v)
    mean = v[0] / v[2]
    var = v[1] / v[2] - mean * mean
    return mean, var
