"""fp32 accuracy of the ECP quadrature log|psi| in the walker's pivot order vs partial pivoting,
both against the fp64 partial-pivoting values of the same configurations (C / C2 ccECP, 512
walkers, host Haar rotations): max / 99.99th-percentile absolute error and counts above 1e-4."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd"))
from oracle import system  # noqa: E402
from oracle import pphamiltonian as pp  # noqa: E402
from aiqmc import _lib  # noqa: E402

for name in ("C_ecp", "C2_ecp"):
    s = system.make_system(name)
    t = s.tables()
    e = {"C_ecp": pp.c_atom_ccecp, "C2_ecp": pp.c2_ccecp}[name]()
    rng = np.random.default_rng(11)
    params = system.flatten_params(system.init_params(rng, s, randomize_aux=True))
    pos = system.init_electrons(rng, s.atoms, s.charges, 512, 1.0)
    rot = pp.haar_rotations(rng, 512)
    out = {}
    for dt in (torch.float64, torch.float32):
        ctx = _lib.Context(s.nelectrons, s.natoms, s.nspins, s.atoms, s.charges, t["spin_up_indices"],
                           t["spin_down_indices"], t["parallel_indices"], t["antiparallel_indices"], dtype=dt, device=0)
        ctx.set_ecp(e.rn_local, e.local_coes, e.local_exps, e.rn_non_local, e.non_local_coes, e.non_local_exps, e.list_l)
        ctx.set_params(params)
        p = torch.tensor(pos, device="cuda", dtype=dt)
        r = torch.tensor(rot, device="cuda", dtype=dt)
        for piv in (False, True):
            ctx.set_quad_pivoted(piv)
            el, l, ph = ctx.local_energy_ecp(p, rot=r, want_quadrature=True)
            torch.cuda.synchronize()
            out[(dt, piv)] = (l.double().cpu().numpy().ravel(), el.cpu().numpy())
    ref = out[(torch.float64, True)][0]
    print(name, "fp64 fixed vs pivoted max", float(np.max(np.abs(out[(torch.float64, False)][0] - ref))))
    for piv in (False, True):
        d = np.abs(out[(torch.float32, piv)][0] - ref)
        de = np.abs(out[(torch.float32, piv)][1] - out[(torch.float64, True)][1])
        print(name, "fp32", "pivoted" if piv else "walker-order", "max", float(d.max()), "p99.99", float(np.quantile(d, 0.9999)),
              ">1e-4:", int((d > 1e-4).sum()), "of", d.size, "| E_L max abs err", float(de.max()), "mean", float(de.mean()))
