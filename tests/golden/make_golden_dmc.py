"""DMC trajectory fixtures from the float64 oracle (oracle/dmc.py dmc_blocks): the reference
driver's loop (DMC/main_dmc.py:113-244 over dmc.py:72-93) with every draw injected.

Run from the repo root:  python tests/golden/make_golden_dmc.py [ccecp attractive ne_allelectron]
C_dmc_<T>.npz for T in (ccecp, attractive): the single-atom carbon system, B = 8 walkers,
2 blocks x 3 iterations, tstep 0.05, feedback 1.0.  "ccecp" is the example's table (its
T-move amplitudes are all negative: no electron moves); "attractive" (list_l = 1, negative
coefficients) makes the T-moves select and accept moves.
Ne_dmc_ne_allelectron.npz: all-electron Ne (10 e-) through the same pp-only DMC step with zero
ECP coefficients (what "Ne + DMC" maps to), B = 4, 1 block x 2 iterations.
C_dmc_attractive_2dev.npz: the "attractive" table with the 8 walkers split over 2 devices
(oracle.dmc.dmc_blocks_devices: per-device T-moves / drift-diffusion / comb, global cut, estimate
and feedback), 2 blocks x 2 iterations; u_comb [2, 2], extra [2, 2, 4, 12] per (block, device).
Ne_dmc_ne_allelectron_2dev.npz: all-electron Ne (BASELINE config 5, the multi-GPU DMC one) the
same way, 4 walkers over 2 devices, 2 blocks x 2 iterations.
Arrays: params_flat, x0 [B,12], e_l0_re/_im [B] (pp energies of x0 with rot0), rot0;
per step k (6): rot_tm, u_sel, u_acc, gauss1 [B,12], gauss2 [B,4,12], u [B,4], rot_old, rot_new;
per block (2): u_comb, extra [B,12]; outputs: energy_re/_im [6,B], weights [6,B],
positions [6,B,12], newinds [2,B], comb_weight [2], e_est [2], e_trial [2], x_final [B,12].
Oracle outputs, not reference outputs (JAX is absent here).
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import dmc, network, pphamiltonian as pp, system  # noqa: E402

torch.set_default_dtype(torch.float64)

TABLES = {
    # all-electron Ne through the pp path (dmc_propagate is pp-only, DMC/dmc.py:13-94): zero local
    # coefficients leave the -Z/r part of local_pp_energy (pseudopotential.py:86-117) = V_en, zero
    # nonlocal coefficients make E_nl = 0 and every T-move amplitude 0 (no move)
    "ne_allelectron": pp.ECP([[1.0]], [[0.0]], [[1.0]], [[[2.0], [2.0], [2.0]]], [[[0.0], [0.0], [0.0]]],
                             [[[1.0], [1.0], [1.0]]], 2),
    "ccecp": pp.c_atom_ccecp(),
    "attractive": pp.ECP([[1.0]], [[0.0]], [[1.0]], [[[2.0], [1.0]]], [[[-3.0], [-5.0]]], [[[0.7], [0.4]]], 1),
}
TSTEP, FEEDBACK = 0.05, 1.0


def make_2dev(out_dir: str, name: str = "attractive"):
    """The multi-device driver (main_dmc.py pmapped over 2 devices) on one table."""
    sysname = "Ne" if name == "ne_allelectron" else "C_ecp"
    s = system.make_system(sysname)
    N = s.nelectrons
    B, NDEV, NBLOCKS, ITERS = (4 if sysname == "Ne" else 8), 2, 2, 2
    rng = np.random.default_rng({"attractive": 54, "ne_allelectron": 55}[name])
    params = system.init_params(rng, s, randomize_aux=True)
    x0 = system.init_electrons(rng, s.atoms, s.charges, B, 1.0)
    rot0 = pp.haar_rotations(rng, B)
    steps = []
    for _ in range(NBLOCKS * ITERS):
        steps.append(dict(rot_tm=pp.haar_rotations(rng, B), u_sel=rng.uniform(size=B) * 2e-3,
                          u_acc=rng.uniform(size=(B, N)), gauss1=rng.standard_normal((B, 3 * N)),
                          gauss2=rng.standard_normal((B, N, 3 * N)), u=rng.uniform(size=(B, N)),
                          rot_old=pp.haar_rotations(rng, B), rot_new=pp.haar_rotations(rng, B)))
    u_comb = rng.uniform(size=(NBLOCKS, NDEV))
    extra = rng.uniform(size=(NBLOCKS, NDEV, B // NDEV, 3 * N))
    net = network.Network(s)
    pt = network.to_torch(params)
    ecp = TABLES[name]
    e_l0 = pp.batch_local_energy_pp(net, pt, ecp, torch.tensor(x0), rot0)[0].detach().numpy()
    trace, x, w = dmc.dmc_blocks_devices(net, pt, ecp, x0, e_l0, NBLOCKS, ITERS, TSTEP, FEEDBACK,
                                         lambda k: steps[k],
                                         lambda b: [(float(u_comb[b, d]), extra[b, d]) for d in range(NDEV)], NDEV)
    out = dict(params_flat=system.flatten_params(params), x0=x0, rot0=rot0, e_l0_re=e_l0.real, e_l0_im=e_l0.imag,
               u_comb=u_comb, extra=extra, ndev=np.int64(NDEV),
               energy_re=np.stack(trace["energy"]).real, energy_im=np.stack(trace["energy"]).imag,
               weights=np.stack(trace["weights"]), positions=np.stack(trace["positions"]),
               newinds=np.stack(trace["newinds"]), comb_weight=np.stack(trace["comb_weight"]),
               e_est=np.array(trace["e_est"]), e_trial=np.array(trace["e_trial"]), x_final=x,
               tstep=np.float64(TSTEP), feedback=np.float64(FEEDBACK))
    for key in steps[0]:
        out[key] = np.stack([st[key] for st in steps])
    np.savez_compressed(os.path.join(out_dir, f"{'Ne' if sysname == 'Ne' else 'C'}_dmc_{name}_2dev.npz"), **out)
    print(name, "2dev e_est", trace["e_est"], "comb weights", trace["comb_weight"], "newinds", trace["newinds"])


def make(out_dir: str, name: str):
    sysname = "Ne" if name == "ne_allelectron" else "C_ecp"
    s = system.make_system(sysname)
    N = s.nelectrons
    B, NBLOCKS, ITERS = (4, 1, 2) if sysname == "Ne" else (8, 2, 3)
    rng = np.random.default_rng({"ccecp": 51, "attractive": 52, "ne_allelectron": 53}[name])
    params = system.init_params(rng, s, randomize_aux=True)
    x0 = system.init_electrons(rng, s.atoms, s.charges, B, 1.0)
    rot0 = pp.haar_rotations(rng, B)
    nsteps = NBLOCKS * ITERS
    steps = []
    for _ in range(nsteps):
        steps.append(dict(rot_tm=pp.haar_rotations(rng, B), u_sel=rng.uniform(size=B) * 2e-3,
                          u_acc=rng.uniform(size=(B, N)), gauss1=rng.standard_normal((B, 3 * N)),
                          gauss2=rng.standard_normal((B, N, 3 * N)), u=rng.uniform(size=(B, N)),
                          rot_old=pp.haar_rotations(rng, B), rot_new=pp.haar_rotations(rng, B)))
    blocks = [(float(rng.uniform()), rng.uniform(size=(B, 3 * N))) for _ in range(NBLOCKS)]
    net = network.Network(s)
    pt = network.to_torch(params)
    ecp = TABLES[name]
    e_l0 = pp.batch_local_energy_pp(net, pt, ecp, torch.tensor(x0), rot0)[0].detach().numpy()
    trace, x, w = dmc.dmc_blocks(net, pt, ecp, x0, e_l0, NBLOCKS, ITERS, TSTEP, FEEDBACK, lambda k: steps[k],
                                 lambda b: blocks[b])
    out = dict(params_flat=system.flatten_params(params), x0=x0, rot0=rot0, e_l0_re=e_l0.real, e_l0_im=e_l0.imag,
               u_comb=np.array([b[0] for b in blocks]), extra=np.stack([b[1] for b in blocks]),
               energy_re=np.stack(trace["energy"]).real, energy_im=np.stack(trace["energy"]).imag,
               weights=np.stack(trace["weights"]), positions=np.stack(trace["positions"]),
               newinds=np.stack(trace["newinds"]), comb_weight=np.array(trace["comb_weight"]),
               e_est=np.array(trace["e_est"]), e_trial=np.array(trace["e_trial"]), x_final=x,
               tstep=np.float64(TSTEP), feedback=np.float64(FEEDBACK))
    for key in steps[0]:
        out[key] = np.stack([st[key] for st in steps])
    np.savez_compressed(os.path.join(out_dir, f"{'Ne' if sysname == 'Ne' else 'C'}_dmc_{name}.npz"), **out)
    moved = [int((np.abs(dmc.tmoves(net, pt, ecp, torch.tensor(x0[b]), steps[0]["rot_tm"][b],
                                    steps[0]["u_sel"][b], steps[0]["u_acc"][b], TSTEP)[0].numpy() - x0[b]) > 0).any())
             for b in range(2)]
    print(name, "e_est", trace["e_est"], "comb weights", trace["comb_weight"], "newinds", trace["newinds"],
          "T-moved (first 2 walkers, step 0)", moved)


if __name__ == "__main__":
    for n in sys.argv[1:] or list(TABLES) + ["attractive_2dev", "ne_allelectron_2dev"]:
        if n.endswith("_2dev"):
            make_2dev(os.path.dirname(os.path.abspath(__file__)), n[:-len("_2dev")])
        else:
            make(os.path.dirname(os.path.abspath(__file__)), n)
