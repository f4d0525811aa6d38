"""DMC total energy (drop-in for AIQMCrelease3/DMC/total_energy.py:9-29).

``calculate_total_energy(local_energy)`` returns ``total_energy(params, key, data) ->
(e_l [B] complex, variance)``: the pp local energies of the batch (one GPU call,
aiqmc_local_energy_ecp; the reference vmaps with one split key per walker, our key draws
per-walker rotations on the device), mean = pmean(mean(e_l)), variance =
pmean(mean((e_l - mean) conj(e_l - mean))) over the ranks (RCCL all-reduce)."""
from __future__ import annotations

import torch

from .. import constants


def calculate_total_energy(local_energy):
    def total_energy(params, key, data):
        e_l, _ = local_energy(params, key, data)
        loss = constants.pmean(e_l.mean())
        diff = e_l - loss
        variance = constants.pmean((diff * torch.conj(diff)).mean())
        return e_l, variance
    return total_energy
