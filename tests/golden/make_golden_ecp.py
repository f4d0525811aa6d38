"""Generate tests/golden/C_ecp.npz from the float64 ECP oracle (oracle/pphamiltonian.py).

Run from the repo root:  python tests/golden/make_golden_ecp.py [C_ecp] [C2_ecp]
Configs: the reference's single-atom carbon ccECP example
(AIQMCrelease3/example/single_atom_C/single_atom_C.py: Z_eff = 4, 4 electrons,
spins +-+-, list_l = 2, tables :13-23) -> C_ecp.npz, and its C2 example
(example/C2/C2.py:8-27: atoms at z = -+1, both ccECP carbons, block spins ++++----)
-> C2_ecp.npz, where the rotated electron NOT being offset by its atom (quirk E2)
matters, and the CO2 example (AIQMCrelease2/example/CO2/co2_test.py: C, O, O ccECP, 16
electrons, the three-atom shape) -> CO2_ecp.npz (2 walkers).  Arrays (float64):
  params_flat  canonical parameter vector; pos [B,12]; rot [B,3,3] the injected
  grid rotations (jax.random.orthogonal's role, pseudopotential.py:233-241);
  e_re, e_im [B]  complex E_L (pphamiltonian.py:177-188);
  e_nl_re, e_nl_im [B] nonlocal part; e_loc [B] local pp part;
  logq_re, logq_im [B,N,A,50] complex log psi at the quadrature configurations.
Oracle outputs, not reference outputs (JAX is absent here).
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import network, pphamiltonian, system  # noqa: E402

torch.set_default_dtype(torch.float64)


CONFIGS = {"C_ecp": (31, pphamiltonian.c_atom_ccecp), "C2_ecp": (32, pphamiltonian.c2_ccecp),
           "CO2_ecp": (33, pphamiltonian.co2_ccecp)}
BATCH = {"CO2_ecp": 2}   # 16 electrons x 3 atoms x 50 points per walker through the oracle network


def make(out_dir: str, name: str = "C_ecp", B: int = 4):
    s = system.make_system(name)
    seed, tables = CONFIGS[name]
    rng = np.random.default_rng(seed)
    params = system.init_params(rng, s, randomize_aux=True)
    pos = system.init_electrons(rng, s.atoms, s.charges, B, 1.0)
    rots = pphamiltonian.haar_rotations(rng, B)
    ecp = tables()
    net = network.Network(s)
    pt = network.to_torch(params)
    e, nl, loc, logs = pphamiltonian.batch_local_energy_pp(net, pt, ecp, torch.tensor(pos), rots)
    e, nl, logs = e.detach(), nl.detach(), logs.detach()
    np.savez_compressed(
        os.path.join(out_dir, f"{name}.npz"), params_flat=system.flatten_params(params), pos=pos, rot=rots,
        e_re=e.real.numpy(), e_im=e.imag.numpy(), e_nl_re=nl.real.numpy(), e_nl_im=nl.imag.numpy(),
        e_loc=loc.detach().numpy(), logq_re=logs.real.numpy(), logq_im=logs.imag.numpy())
    print(name, "E_L", e.numpy())


if __name__ == "__main__":
    for n in sys.argv[1:] or list(CONFIGS):
        make(os.path.dirname(os.path.abspath(__file__)), n, BATCH.get(n, 4))
