"""Generate tests/golden/C_tmoves.npz from the float64 T-move oracle (oracle/dmc.py tmoves).

Run from the repo root:  python tests/golden/make_golden_tmoves.py [C_ecp] [C2_ecp]  (C2_tmoves.npz: C2 example)
Config: the single-atom carbon system of the ccECP example (4 electrons, Z_eff = 4) with
two nonlocal tables: "ccecp" (single_atom_C.py:13-23, list_l = 2) and "attractive", a
synthetic list_l = 1 table with negative coefficients, so that forward amplitudes are
non-zero and the selection / back-amplitude / acceptance path is exercised.  Arrays (float64),
per table name T in (ccecp, attractive):
  params_flat; pos [B,12]; rot [B,3,3]; u_sel [B]; u_acc [B,4]; tstep_T;
  new_T [B,12] positions after the T-moves; acc_T [B,4] acceptance Re(norm / back_norm).
Oracle outputs, not reference outputs (JAX is absent here).
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import dmc, network, pphamiltonian, system  # noqa: E402

torch.set_default_dtype(torch.float64)

# C2 (example/C2/C2.py, atoms at z = -+1): the example's tables on both atoms, and the
# attractive list_l = 1 table on both atoms (moves happen, quirk E2 -- moved electrons at
# r_ia p_q R without the atom offset -- is exercised off the origin)
C2_TABLES = {
    "ccecp": (pphamiltonian.c2_ccecp(), 0.1),
    "attractive": (pphamiltonian.ECP([[1.0], [1.0]], [[0.0], [0.0]], [[1.0], [1.0]], [[[2.0], [1.0]]] * 2,
                                     [[[-3.0], [-5.0]]] * 2, [[[0.7], [0.4]]] * 2, 1), 0.3),
}

TABLES = {
    "ccecp": (pphamiltonian.c_atom_ccecp(), 0.1),
    "attractive": (pphamiltonian.ECP([[1.0]], [[0.0]], [[1.0]], [[[2.0], [1.0]]], [[[-3.0], [-5.0]]],
                                     [[[0.7], [0.4]]], 1), 0.3),
}


def make(out_dir: str, sysname: str = "C_ecp", B: int = 8):
    s = system.make_system(sysname)
    rng = np.random.default_rng(41 if sysname == "C_ecp" else 42)
    tables = TABLES if sysname == "C_ecp" else C2_TABLES
    params = system.init_params(rng, s, randomize_aux=True)
    pos = system.init_electrons(rng, s.atoms, s.charges, B, 1.0)
    rots = pphamiltonian.haar_rotations(rng, B)
    u_sel = np.array([0.0, 1e-4, 1e-3, 3e-3, 0.0, 0.5, 2e-4, 0.9])[:B]
    u_acc = rng.uniform(size=(B, s.nelectrons))
    net = network.Network(s)
    pt = network.to_torch(params)
    out = dict(params_flat=system.flatten_params(params), pos=pos, rot=rots, u_sel=u_sel, u_acc=u_acc)
    for name, (ecp, tau) in tables.items():
        new, acc = zip(*[dmc.tmoves(net, pt, ecp, torch.tensor(pos[b]), rots[b], u_sel[b], u_acc[b], tau)
                         for b in range(B)])
        out[f"new_{name}"] = torch.stack(new).numpy()
        out[f"acc_{name}"] = np.stack(acc)
        out[f"tstep_{name}"] = np.array(tau)
        moved = np.abs(out[f"new_{name}"] - pos).reshape(B, -1, 3).sum(-1) > 0
        print(name, "moved electrons per walker", moved.sum(1))
    fname = "C_tmoves.npz" if sysname == "C_ecp" else "C2_tmoves.npz"
    np.savez_compressed(os.path.join(out_dir, fname), **out)


if __name__ == "__main__":
    for n in sys.argv[1:] or ["C_ecp", "C2_ecp"]:
        make(os.path.dirname(os.path.abspath(__file__)), n)
