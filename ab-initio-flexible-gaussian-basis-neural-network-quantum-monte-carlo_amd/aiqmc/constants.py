"""Cross-device collectives (AIQMCrelease3/constants.py:5-9) over torch.distributed.

The reference's ``pmean``/``psum``/``all_gather`` act over the JAX pmap axis
'qmc_pmap_axis' and are identities outside pmap.  Here one process drives one
GPU; the collectives run over the default process group (RCCL over xGMI when
initialised with backend "nccl", gloo on CPU) and are identities when no group
is initialised.  ``pmean_stats`` fuses the energy statistics of one iteration
(loss.py:206,208) into a single all-reduce.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

PMAP_AXIS_NAME = 'qmc_pmap_axis'

# Run the collective path even at world size 1 (AIQMC_FORCE_COLLECTIVES=1 or force_collectives()):
# the all-reduces then execute on a one-rank group, e.g. RCCL under torch.distributed.run
# --nproc-per-node 1 (tests/test_gpu_rccl.py, bench.py --force-collectives).
_FORCE = os.environ.get("AIQMC_FORCE_COLLECTIVES", "") == "1"
# all-reduces issued through this module since import (the fused training step issues 3)
ALLREDUCE_CALLS = 0


def force_collectives(on: bool = True) -> None:
    global _FORCE
    _FORCE = bool(on)


def _active() -> bool:
    return (dist.is_available() and dist.is_initialized()
            and (dist.get_world_size() > 1 or _FORCE))


def world_size() -> int:
    return dist.get_world_size() if _active() else 1


def all_reduce_(x: torch.Tensor) -> torch.Tensor:
    """In-place SUM all-reduce over the default group (counted); identity when inactive."""
    global ALLREDUCE_CALLS
    if _active():
        ALLREDUCE_CALLS += 1
        dist.all_reduce(x, op=dist.ReduceOp.SUM)
    return x


def psum(x: torch.Tensor) -> torch.Tensor:
    if not _active():
        return x
    return all_reduce_(x.clone())


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

    The reference takes two dependent pmeans (loss.py:206-208): E = pmean(mean(e)), then
    var = pmean(mean(|e - E|^2)).  One all-reduce of [sum_r M2_r, sum_r n_r m_r, sum_r n_r m_r^2, n]
    (rank mean m_r, centred sum of squares M2_r = sum |e - m_r|^2) gives the same quantity by
    the pairwise combination of Chan et al.:
        var = (sum_r M2_r + sum_r n_r (m_r - E)^2) / n,   sum_r n_r (m_r - E)^2 = sum_r n_r m_r^2 - n E^2,
    in float64; the within-rank spread never meets the E^2 cancellation.  Equal to the
    reference's two-pass value (for the equal per-device batches the drivers require).

    Device tensors go through aiqmc_energy_stats (one workgroup forms the 4-vector, and the
    mean/variance when there is no collective): 2 launches per iteration instead of ~17 small
    elementwise/reduction kernels.  Host tensors (gloo ranks) and other dtypes take the same
    formulas in torch.
    """
    if e_l.is_cuda and e_l.dtype in (torch.float32, torch.float64):
        from . import _lib
        if not _active():
            v = _lib.energy_stats(e_l, finalize=True)
        else:
            v = _lib.energy_stats(e_l, finalize=False)
            all_reduce_(v)   # out[4..5] are rewritten below
            _lib.energy_stats_final(v)
        return v[4], v[5]
    e = e_l.to(torch.float64)
    n = float(e.numel())
    m = e.mean()
    m2 = ((e - m) * (e - m)).sum()
    # the count as a device fill, not a host scalar copied in: torch.tensor(n, device=...) is a
    # pageable host-to-device copy that waits for the stream (a drain per VMC iteration)
    cnt = torch.full((), n, dtype=torch.float64, device=e.device)
    v = torch.stack([m2, n * m, n * m * m, cnt])
    v = psum(v)
    mean = v[1] / v[3]
    between = torch.clamp(v[2] - v[3] * mean * mean, min=0.0)
    var = (v[0] + between) / v[3]
    return mean, var
