"""DMC driver (drop-in for AIQMCrelease3/DMC/main_dmc.py:22-242) over the GPU kernels.

``main(atoms, charges, spins, tstep, nelectrons, nsteps, natoms, ndim, batch_size, iterations,
nblocks, feedback, nspins, save_path, restore_path, Rn_local, Local_coes, Local_exps,
Rn_non_local, Non_local_coes, Non_local_exps, save_frequency, structure)`` with the
reference's flow: restore the VMC checkpoint (a DMC run without one raises, :66-67), e_trial =
e_est = the pp total energy (:113-116), then per block ``iterations`` dmc_propagate steps
(T-moves, drift-diffusion, pp energies, weights), the weighted block estimate (:190), a
checkpoint every ``save_frequency`` minutes (:195-200), the stochastic comb (:202) followed by
the driver's walker re-indexing (:204-233, ``reindex_walkers``), e_trial feedback (:237) and a
``DMC_states`` CSV row (:239-244).

One process per GPU (torchrun); ``batch_size`` is the global walker count, each rank owns
batch_size / world walkers.  Kept from the reference: esigma = std over the per-device copies
of the (already pmean'd) e_est, which is 0, so the branch cut passed to the weight update is 0
(:118, :137); weights are per device.  Deviations (documented in DESIGN.md): the Philox key
offset advances every step (the reference passes the same ``subkeys`` to every step, :162);
the re-indexing pads each device block to its own walker count (the reference compares the
unique count with the GLOBAL batch_size, which only reshapes back on one device, :219-229).
"""
from __future__ import annotations

import logging
import time
from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .. import checkpoint
from ..Energy import pphamiltonian
from ..VMC.VMCmcstep import PhiloxKey
from ..spin_indices import jastrow_indices_ee, spin_indices_h
from ..utils import writers
from ..wavefunction_Ynlm import nn
from .dmc import dmc_propagate
from .estimate_energy import estimate_energy
from .total_energy import calculate_total_energy


def reindex_walkers(x1: torch.Tensor, newindices: torch.Tensor, extra_uniform: torch.Tensor) -> torch.Tensor:
    """main_dmc.py:215-233 for one device block: the walkers at the sorted unique comb indices,
    then, if the comb killed walkers, n copies of the LAST unique walker plus U[0,1) noise
    (``extra_uniform`` [>= n, 3N], the reference's jax.random.uniform(key, (n, 3N)))."""
    B = x1.shape[0]
    unique = torch.unique(newindices.long().to(x1.device))          # sorted, as jnp.unique
    temp = x1[unique]
    n = B - unique.numel()
    if n > 0:
        extra = temp[-1] + extra_uniform[:n].to(x1.device, x1.dtype)
        temp = torch.cat([temp, extra], dim=0)
    return temp.contiguous()


def main(atoms, charges, spins, tstep: float, nelectrons: int, nsteps: int, natoms: int, ndim: int,
         batch_size: int, iterations: int, nblocks: int, feedback: float, nspins: Tuple[int, int],
         save_path: Optional[str], restore_path: Optional[str], Rn_local, Local_coes, Local_exps, Rn_non_local,
         Non_local_coes, Non_local_exps, save_frequency: float, structure=None, seed: Optional[int] = None):
    del structure
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank() if world > 1 else 0
    if batch_size % world:
        raise ValueError('Batch size must be divisible by number of devices!')
    device_batch_size = batch_size // world
    seed = int(1e6 * time.time()) % (1 << 62) if seed is None else int(seed)
    ckpt_save_path = checkpoint.create_save_path(save_path=save_path)
    ckpt_restore_path = checkpoint.get_restore_path(restore_path=restore_path)
    fname = checkpoint.find_last_checkpoint(ckpt_save_path) or checkpoint.find_last_checkpoint(ckpt_restore_path)
    if not fname:
        raise ValueError('DMC must use the wave function from VMC!')
    t_init, data, params, opt_state = checkpoint.restore(fname, batch_size)

    par, anti, npar, nanti = jastrow_indices_ee(spins=spins, nelectrons=nelectrons)
    up, dn = spin_indices_h(spins)
    network = nn.make_ai_net(ndim=ndim, nelectrons=nelectrons, natoms=natoms, nspins=nspins, determinants=1,
                             charges=charges, parallel_indices=par, antiparallel_indices=anti, n_parallel=npar,
                             n_antiparallel=nanti, spin_up_indices=up, spin_down_indices=dn)
    signed_network = network.apply
    log_network = nn.make_log_network(signed_network)
    localenergy = pphamiltonian.local_energy(f=signed_network, lognetwork=log_network, charges=charges,
                                             nspins=spins, rn_local=Rn_local, local_coes=Local_coes,
                                             local_exps=Local_exps, rn_non_local=Rn_non_local,
                                             non_local_coes=Non_local_coes, non_local_exps=Non_local_exps,
                                             natoms=natoms, nelectrons=nelectrons, ndim=ndim, list_l=2)
    total_e = calculate_total_energy(localenergy)
    dev = torch.device("cuda", torch.cuda.current_device())
    pos = torch.as_tensor(np.asarray(data.positions)).reshape(-1, nelectrons * ndim)
    if pos.shape[0] == batch_size and world > 1:
        pos = pos[rank * device_batch_size:(rank + 1) * device_batch_size]
    if pos.shape[0] != device_batch_size:
        raise ValueError(f"checkpoint holds {pos.shape[0]} walkers, expected {device_batch_size} per device")
    dtype = pos.dtype if pos.dtype in (torch.float32, torch.float64) else torch.float32
    data = nn.AINetData(positions=pos.to(dev, dtype).contiguous(), spins=data.spins, atoms=data.atoms,
                        charges=data.charges)
    key0 = PhiloxKey(seed + 7919 * rank, 0)
    e_l, _ = total_e(params, key0, data)
    from .. import constants
    e_trial = complex(constants.pmean(e_l.mean()))                 # :115 (pmean'd inside total_e)
    e_est = e_trial
    esigma = float(np.std(np.full(world, e_est.real)))            # :118 -- 0 by construction
    weights = torch.ones(device_batch_size, dtype=dtype, device=dev)
    branchcut_start = torch.full((device_batch_size,), 10.0, dtype=torch.float64)
    run = dmc_propagate(signed_network, log_network, signed_network, 2, nelectrons, natoms, ndim,
                        device_batch_size, tstep, nsteps, charges, spins, Rn_local, Local_coes, Local_exps,
                        Rn_non_local, Non_local_coes, Non_local_exps)
    ctx = network.apply._aiqmc_network.bind(params, data.atoms, dtype)
    rng = np.random.default_rng(seed + rank)
    energy_data = torch.zeros(nblocks, iterations, device_batch_size, dtype=torch.float64, device=dev)
    weights_data = torch.zeros_like(energy_data)
    time_of_last_ckpt = time.time()
    estimates = []
    step = 0
    with writers.Writer(name='DMC_states', schema=['block', 'energy', 'positions'],
                        directory=ckpt_restore_path or ckpt_save_path, iteration_key=None, log=False) as writer:
        for block in range(nblocks):
            for t in range(t_init, t_init + iterations):
                energy, weights, data = run(params, PhiloxKey(key0.seed, step), data, weights,
                                            branchcut_start * esigma, e_trial.real, e_est.real)
                step += 1
                energy_data[block, t - t_init] = energy.real.to(torch.float64)
                weights_data[block, t - t_init] = weights.to(torch.float64)
            e_est = complex(estimate_energy(energy_data, weights_data).item())
            if world > 1:   # the reference's estimate is over the global arrays
                v = torch.tensor([(energy_data * weights_data).sum().item(), weights_data.sum().item()],
                                 dtype=torch.float64, device=dev)
                dist.all_reduce(v)
                e_est = complex((v[0] / v[1]).item())
            logging.info('Block %05d: %03.4f E_h', block, e_est.real)
            if time.time() - time_of_last_ckpt > save_frequency * 60:
                checkpoint.save(ckpt_restore_path or ckpt_save_path, block, data, params, opt_state)
                time_of_last_ckpt = time.time()
            wn, newinds = ctx.dmc_branch(weights, float(rng.uniform()))
            weights = wn.expand(device_batch_size).contiguous()
            x2 = reindex_walkers(data.positions, newinds,
                                 torch.tensor(rng.uniform(size=(device_batch_size, nelectrons * ndim))))
            data = nn.AINetData(positions=x2, spins=data.spins, atoms=data.atoms, charges=data.charges)
            e_trial = complex(e_est.real - feedback * float(torch.log(weights.mean()).real), 0.0)
            estimates.append(e_est.real)
            if rank == 0:
                writer.write(block, block=block, energy=e_est.real, positions=np.asarray(x2.cpu()))
    return estimates, data, weights
