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
batch_size / world walkers.  Kept from the reference:
* ``total_e`` returns the PER-WALKER pp energies (DMC/total_energy.py:32), so the first
  block runs with per-walker e_trial = e_est = those energies (:115-116), and
  esigma = jnp.std(e_est) over every walker of every device (:118) = sqrt of total_e's
  pmean'd variance; the branch cut passed to the weight update is 10 esigma (:137, :162);
* the energy cut of comput_S is one minimum over all devices (aiqmc.DMC.dmc: MIN all-reduce);
* the block estimate is the weighted average over all blocks so far and all devices (:190);
* e_trial feedback uses jnp.mean over the per-device comb weights (:237): all-reduced here.
Multi-rank housekeeping: rank 0 alone writes the checkpoint and the CSV, with the positions
of all ranks gathered (the reference's arrays are global).  Whether a block checkpoints is
decided by rank 0's clock and broadcast (``make_checkpoint_hook``): every rank enters the
gather together, so the collectives never pair up across different call sites.  Deviations (documented in
DESIGN.md): the Philox key offset advances every step (the reference passes the same
``subkeys`` to every step, :162); the re-indexing pads each device block to its own walker
count (the reference compares the unique count with the GLOBAL batch_size, which only
reshapes back on one device, :219-229).
"""
from __future__ import annotations

import contextlib
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


def _gather_walkers(x: torch.Tensor, world: int) -> torch.Tensor:
    """The global walker array (rank-major, the reference's [ndev, B] reshape) on every rank."""
    if world == 1:
        return x
    parts = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(parts, x.contiguous())
    return torch.cat(parts, dim=0)


def _rank0_decides(flag: bool, world: int, device) -> bool:
    """Rank 0's flag on every rank (one MAX all-reduce of rank 0's value; other ranks add 0)."""
    if world == 1:
        return flag
    rank = dist.get_rank()
    if dist.get_backend() == "nccl" and device.type != "cuda":
        device = torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor([1 if (flag and rank == 0) else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return bool(t.item())


def make_checkpoint_hook(out_dir: str, params, opt_state, save_frequency: float, clock=time.time):
    """on_block hook of main_dmc.py:195-200: a checkpoint when more than ``save_frequency``
    minutes passed since the last one.  Rank 0's clock decides for all ranks (the reference
    runs one process, so it has one clock); then every rank joins the gather of the walkers and
    rank 0 writes.  ``clock`` is injectable for the multi-rank test."""
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank() if world > 1 else 0
    last = [clock()]
    saved = []

    def on_block(block, e_est, data):
        del e_est
        due = _rank0_decides(clock() - last[0] > save_frequency * 60, world, data.positions.device)
        if not due:
            return
        all_pos = _gather_walkers(data.positions, world)
        if rank == 0:
            saved.append(checkpoint.save(out_dir, block, nn.AINetData(positions=all_pos, spins=data.spins,
                                                                      atoms=data.atoms, charges=data.charges),
                                         params, opt_state))
        if world > 1:
            dist.barrier()
        last[0] = clock()

    on_block.saved = saved
    return on_block


def dmc_blocks(run, ctx, params, data, e_l0, variance0, nblocks: int, iterations: int, feedback: float,
               step_key, block_draws, t_init: int = 0, on_block=None, writer=None, trace: bool = False):
    """The block loop of main_dmc.py:113-244 over this rank's walkers.

    run: dmc_propagate_run; ctx: the bound HIP context (comb); e_l0 [B] / variance0: total_e of
    the starting walkers (per-walker e_trial = e_est = e_l0 in the first block, esigma =
    sqrt(variance0) = jnp.std(e_est), :113-118); step_key(step) -> the key of one
    dmc_propagate_run call (PhiloxKey or HostDmcDraws); block_draws(block) -> (u, extra) with
    u the comb's uniform (branch.py:17) and extra [B,3N] the re-indexing noise (:222).
    Returns (block estimates, data, weights, trace).  With ``trace=True`` (the parity tests)
    trace holds device copies of every step's energies / weights / positions and every block's
    comb indices; otherwise it is None and nothing per step is kept beyond the reference's own
    [nblocks, iterations, B] energy and weight arrays."""
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    B = data.positions.shape[0]
    dev = data.positions.device
    dtype = data.positions.dtype
    e_trial = e_l0
    e_est = e_l0
    esigma = float(torch.sqrt(torch.as_tensor(variance0).real.clamp(min=0)).item())   # :118 jnp.std(e_est)
    weights = torch.ones(B, dtype=dtype, device=dev)
    branchcut_start = torch.full((B,), 10.0, dtype=torch.float64)
    energy_data = torch.zeros(nblocks, iterations, B, dtype=torch.float64, device=dev)
    weights_data = torch.zeros_like(energy_data)
    estimates = []
    tr = {"energy": [], "weights": [], "positions": [], "newinds": [], "comb_weight": [], "e_trial": []} \
        if trace else None
    step = 0
    for block in range(nblocks):
        for t in range(t_init, t_init + iterations):
            energy, weights, data = run(params, step_key(step), data, weights, branchcut_start * esigma, e_trial,
                                        e_est)
            step += 1
            energy_data[block, t - t_init] = energy.real.to(torch.float64)
            weights_data[block, t - t_init] = weights.to(torch.float64)
            if tr is not None:
                tr["energy"].append(energy.detach().clone())
                tr["weights"].append(weights.detach().clone())
                tr["positions"].append(data.positions.detach().clone())
        # :190 jnp.average over the global [nblocks, iterations, batch] arrays
        v = torch.stack([(energy_data * weights_data).sum(), weights_data.sum()])
        if world > 1:
            dist.all_reduce(v)
        e_est = complex((v[0] / v[1]).item())
        logging.info('Block %05d: %03.4f E_h', block, e_est.real)
        if on_block is not None:
            on_block(block, e_est, data)
        u, extra = block_draws(block)
        wn, newinds = ctx.dmc_branch(weights, float(u))                 # :202
        weights = wn.expand(B).contiguous()
        x2 = reindex_walkers(data.positions, newinds, extra)           # :204-233
        data = nn.AINetData(positions=x2, spins=data.spins, atoms=data.atoms, charges=data.charges)
        wmean = wn.to(torch.float64).reshape(1).clone()               # :237 jnp.mean over the devices' weights
        if world > 1:
            dist.all_reduce(wmean)
            wmean /= world
        e_trial = complex(e_est.real - feedback * float(torch.log(wmean).item()), 0.0)
        estimates.append(e_est.real)
        if tr is not None:
            tr["newinds"].append(newinds.detach().clone())
            tr["comb_weight"].append(float(wn.item()))
            tr["e_trial"].append(e_trial.real)
        all_x2 = _gather_walkers(x2, world)
        if writer is not None:
            writer.write(block, block=block, energy=e_est.real, positions=np.asarray(all_x2.cpu()))
    return estimates, data, weights, tr


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
    e_l0, variance0 = total_e(params, key0, data)                  # :113-116 (e_trial, e_est per walker)
    run = dmc_propagate(signed_network, log_network, signed_network, 2, nelectrons, natoms, ndim,
                        device_batch_size, tstep, nsteps, charges, spins, Rn_local, Local_coes, Local_exps,
                        Rn_non_local, Non_local_coes, Non_local_exps)
    ctx = network.apply._aiqmc_network.bind(params, data.atoms, dtype)
    rng = np.random.default_rng(seed + rank)
    out_dir = ckpt_restore_path or ckpt_save_path
    on_block = make_checkpoint_hook(out_dir, params, opt_state, save_frequency)

    writer = writers.Writer(name='DMC_states', schema=['block', 'energy', 'positions'], directory=out_dir,
                            iteration_key=None, log=False) if rank == 0 else contextlib.nullcontext()
    with writer:
        estimates, data, weights, _ = dmc_blocks(
            run, ctx, params, data, e_l0, variance0, nblocks, iterations, feedback, t_init=t_init,
            step_key=lambda step: PhiloxKey(key0.seed, step),
            block_draws=lambda block: (float(rng.uniform()),
                                       torch.tensor(rng.uniform(size=(device_batch_size, nelectrons * ndim)))),
            on_block=on_block, writer=writer if rank == 0 else None)
    return estimates, data, weights
