"""Generate the golden parity fixtures in tests/golden/ from the float64 oracle.

Run from the repo root:  python tests/golden/make_golden.py [names...]  (default: all)
Each <system>.npz holds (all float64):
  params_flat   canonical tree_flatten parameter vector (aiqmc_set_params input)
  pos           [B,3N] walker positions (init_electrons semantics, width 1.0)
  logabs, phase [B]    oracle.network apply (nn.py:545-551)
  grad          [B,3N] jax.grad(logabs) restated with torch.func.grad
  e_l           [B]    hamiltonian.local_energy via jvp-of-grad (hamiltonian.py:100-131)
  mc_*          one nsteps=2 Metropolis run with injected draws (VMCmcstep.py:28-140):
                mc_gauss1 [2,B,3N], mc_gauss2 [2,B,N,3N], mc_u [2,B,N], mc_tstep, mc_pos_out
These are oracle outputs (the reference itself cannot run here: JAX is absent);
see DESIGN.md "Oracle" for what pins the oracle.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import hamiltonian, mcstep, network, system  # noqa: E402

torch.set_default_dtype(torch.float64)

SYSTEMS = {"H2": 8, "Be": 8, "N2": 8, "Ne": 8, "C2": 4, "O2": 4, "C": 8}
SEEDS = {"H2": 11, "Be": 12, "N2": 13, "Ne": 14, "C2": 16, "O2": 15, "C": 17}


def make(name: str, B: int, out_dir: str):
    s = system.make_system(name)
    rng = np.random.default_rng(SEEDS[name])
    params = system.init_params(rng, s, randomize_aux=True)
    flat = system.flatten_params(params)
    pos = system.init_electrons(rng, s.atoms, s.charges, B, 1.0)
    net = network.Network(s)
    pt = network.to_torch(params)
    x = torch.tensor(pos)
    e_l, logabs, grad = hamiltonian.batch_local_energy(net, pt, x)
    phase = torch.stack([net.apply(pt, x[b])[0] for b in range(B)])
    nsteps, tstep = 2, 0.05
    N = s.nelectrons
    g1 = torch.tensor(rng.standard_normal((nsteps, B, 3 * N)))
    g2 = torch.tensor(rng.standard_normal((nsteps, B, N, 3 * N)))
    u = torch.tensor(rng.uniform(size=(nsteps, B, N)))
    pos_out = mcstep.mc_step(net, pt, x.clone(), g1, g2, u, tstep, nsteps)
    np.savez_compressed(
        os.path.join(out_dir, f"{name}.npz"),
        params_flat=flat, pos=pos, logabs=logabs.numpy(), phase=phase.detach().numpy(),
        grad=grad.numpy(), e_l=e_l.numpy(),
        mc_gauss1=g1.numpy(), mc_gauss2=g2.numpy(), mc_u=u.numpy(), mc_tstep=np.float64(tstep),
        mc_pos_out=pos_out.numpy())
    print(name, "E_L", e_l.numpy())


if __name__ == "__main__":
    out = os.path.dirname(os.path.abspath(__file__))
    for n in sys.argv[1:] or list(SYSTEMS):
        make(n, SYSTEMS[n], out)
