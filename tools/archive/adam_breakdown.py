"""Host-side breakdown of one C-atom ccECP (AIQMC_SYSTEM=Be: Be all-electron) Adam iteration (bench.pp_adam_side_bench's loop):
wall time of mc_step and of the training step, with and without a device synchronisation after
each, and the GPU-side duration of each from CUDA events.  AIQMC_HOST_PARAMS=1: the parameters
round-trip through the host (the round-4 behaviour)."""
import os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
sys.path.insert(0, bench.PKG)
from aiqmc import systems
from aiqmc.Energy import pphamiltonian
from aiqmc.Loss import loss as L
from aiqmc.Optimizer import adam, optax_like as optax
from aiqmc.VMC import VMCmcstep
from aiqmc.wavefunction_Ynlm import nn
from aiqmc.initial_electrons_positions.init import init_electrons
if os.environ.get("AIQMC_HOST_PARAMS"):
    _orig = L._unflatten_like
    L._unflatten_like = lambda t, f: _orig(t, f.detach().cpu().numpy() if isinstance(f, torch.Tensor) else f)
walkers, device, dtype = 4096, torch.device("cuda", 0), torch.float32
system = os.environ.get("AIQMC_SYSTEM", "C_ecp")
s = systems.make_system(system)
network = s.make_network()
params = network.init(4)
if system == "C_ecp":
    e = systems.ccecp_tables("C_ecp")
    log_network = nn.make_log_network(network.apply)
    le = pphamiltonian.local_energy(f=network.apply, lognetwork=log_network, charges=s.charges, nspins=s.spins,
                                    rn_local=e.rn_local, local_coes=e.local_coes, local_exps=e.local_exps,
                                    rn_non_local=e.rn_non_local, non_local_coes=e.non_local_coes,
                                    non_local_exps=e.non_local_exps, natoms=1, nelectrons=4, ndim=3, list_l=2)
    ev = L.make_loss(network=log_network, local_energy=le, clip_local_energy=5.0, clip_from_median=False,
                     center_at_clipped_energy=True, complex_output=True)
else:   # Be, all-electron (bench.adam_side_bench)
    from aiqmc.Energy import hamiltonian as H
    le = H.local_energy(f=network.apply, charges=s.charges, nspins=s.spins)
    ev = L.make_loss(network=network.apply, local_energy=le, clip_local_energy=5.0, clip_from_median=False,
                     center_at_clipped_energy=True, complex_output=True)
opt = optax.chain(optax.scale_by_adam(b1=0.9, b2=0.999, eps=1e-8, eps_root=0.0),
                  optax.scale_by_schedule(lambda t: 0.05 * (1.0 / (1.0 + t)) ** 10000), optax.scale(-1.))
step = adam.make_training_step(adam.make_opt_update_step(ev, opt))
mc_step = VMCmcstep.main_monte_carlo(f=network.apply, tstep=0.05, ndim=3, nelectrons=s.nelectrons, nsteps=10,
                                     batch_size=walkers)
pos, sp = init_electrons(17, None, s.atoms, s.charges, s.spins, walkers, 1.0)
data = nn.AINetData(positions=pos.to(device, dtype).contiguous(), spins=sp, atoms=s.atoms, charges=s.charges)
state = None
for sync in (False, True):
    rows = []
    for t in range(8):
        torch.cuda.synchronize()
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        t0 = time.perf_counter()
        e0.record()
        data = mc_step(params, data, VMCmcstep.PhiloxKey(19, 100 + 10 * t))
        e1.record()
        if sync:
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        data, params, state, loss_v, aux = step(data, params, state, VMCmcstep.PhiloxKey(23, 100 + t))
        e2.record()
        if sync:
            torch.cuda.synchronize()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        rows.append((1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t0), e0.elapsed_time(e1), e1.elapsed_time(e2)))
    r = torch.tensor(rows[2:]).median(0).values.tolist()
    print(f"sync={sync}: host mc_step {r[0]:.3f} ms, host step {r[1]:.3f} ms, wall {r[2]:.3f} ms; "
          f"GPU mc_step {r[3]:.3f} ms, GPU step {r[4]:.3f} ms", flush=True)
