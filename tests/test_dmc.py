"""DMC pieces (AIQMCrelease3/DMC): drift-diffusion step, S / weight update, stochastic comb.
T-moves.  CPU: the oracle against closed forms and its golden fixture; GPU: the HIP path
against the oracle (fp64; E_L, weights and positions to 1e-9, indices and T-move selections
exact)."""
import math

import numpy as np
import pytest
import torch

from oracle import dmc as odmc


def test_comb_closed_form():
    w = np.array([0.5, 1.5, 1.0, 1.0])
    wn, idx = odmc.branch(w, 0.1)
    # cumsum [0.5, 2, 3, 4]; targets (0.4 + [0, 1, 2, 3]) % 4 = [0.4, 1.4, 2.4, 3.4]
    np.testing.assert_array_equal(idx, [0, 1, 2, 3])
    assert wn == 1.0
    wn, idx = odmc.branch(np.array([3.0, 0.0, 0.5, 0.5]), 0.0)
    np.testing.assert_array_equal(idx, [0, 0, 0, 0])   # cumsum [3, 3, 3.5, 4], targets [0, 1, 2, 3]


def test_comput_S_single_global_cut():
    eloc = np.array([-1.0, -3.0, -2.5])
    v2 = np.zeros((3, 6))
    S = odmc.comput_S(e_trial=-2.0, e_est=-2.0, branchcut=10.0, v2=v2, tau=0.01, eloc=eloc, nelec=2)
    # e_est - eloc = [-1, 1, 0.5]; ONE cut = min(|.|, 10) = 0.5 for every walker (D1)
    np.testing.assert_allclose(S, [-0.5, 0.5, 0.5])


def _ctx(name, dtype=torch.float64):
    from oracle import system
    from aiqmc import _lib
    s = system.make_system(name)
    t = s.tables()
    ctx = _lib.Context(s.nelectrons, s.natoms, s.nspins, s.atoms, s.charges, t["spin_up_indices"],
                       t["spin_down_indices"], t["parallel_indices"], t["antiparallel_indices"], dtype=dtype, device=0)
    return s, ctx


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["Be", "N2", "Ne", "Z7", "Z3-2-2"])   # + odd N, three atoms (round 5)
def test_drift_diffusion_matches_oracle(name):
    from oracle import network, system
    s, ctx = _ctx(name)
    rng = np.random.default_rng(17)
    params = system.init_params(rng, s, randomize_aux=True)
    ctx.set_params(system.flatten_params(params))
    B, N = 6, s.nelectrons
    x = torch.tensor(system.init_electrons(rng, s.atoms, s.charges, B, 1.0))
    g1 = torch.tensor(rng.standard_normal((B, 3 * N)))
    g2 = torch.tensor(rng.standard_normal((B, N, 3 * N)))
    u = torch.tensor(rng.uniform(size=(B, N)))
    xr, td_r, go_r, gn_r = odmc.drift_diffusion(network.Network(s), network.to_torch(params), x.clone(), g1, g2, u, 0.05)
    pos = x.cuda().contiguous()
    idx = torch.arange(N)
    g2d = g2.reshape(B, N, N, 3)[:, idx, idx, :].contiguous()
    go, gn, td = ctx.dmc_drift_diffusion(pos, 0.05, gauss1=g1[None], gauss2=g2d[None], u=u[None])
    torch.cuda.synchronize()
    np.testing.assert_allclose(pos.cpu().numpy(), xr.numpy(), rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(go.cpu().numpy(), go_r.numpy(), rtol=1e-8, atol=1e-9)
    np.testing.assert_allclose(gn.cpu().numpy(), gn_r.numpy(), rtol=1e-8, atol=1e-9)
    assert abs(td[2].item() - td_r.item()) < 1e-10


@pytest.mark.gpu
def test_weights_and_branch_match_oracle():
    s, ctx = _ctx("Be")
    rng = np.random.default_rng(4)
    B, N = 300, s.nelectrons
    eo, en = rng.normal(-14.6, 0.4, B), rng.normal(-14.6, 0.4, B)
    go, gn = rng.standard_normal((B, 3 * N)), rng.standard_normal((B, 3 * N))
    w0 = rng.uniform(0.5, 1.5, B)
    tdamp = torch.tensor([0.0, 0.0, 0.97], dtype=torch.float64, device="cuda")
    w = torch.tensor(w0, device="cuda")
    ctx.dmc_weights(w, torch.tensor(eo), torch.tensor(en), torch.tensor(go, device="cuda"),
                    torch.tensor(gn, device="cuda"), tdamp, 0.01, -14.5, -14.62, 0.3)
    S_old = odmc.comput_S(-14.5, -14.62, 0.3, go ** 2, 0.01, eo, N)
    S_new = odmc.comput_S(-14.5, -14.62, 0.3, gn ** 2, 0.01, en, N)
    w_ref = odmc.update_weights(w0, 0.01, 0.97, S_new, S_old)
    np.testing.assert_allclose(w.cpu().numpy(), w_ref, rtol=1e-12)
    wn, idx = ctx.dmc_branch(w, 0.37)
    wn_r, idx_r = odmc.branch(w_ref, 0.37)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(idx.cpu().numpy(), idx_r)
    assert abs(wn.item() - wn_r) < 1e-12


def test_comput_S_dropin_matches_oracle():
    from aiqmc.DMC.S_matrix import comput_S
    rng = np.random.default_rng(2)
    eloc = rng.normal(-5, 1, 40)
    v2 = rng.standard_normal((40, 12)) ** 2
    got = comput_S(-5.1, -5.0, 0.7, torch.tensor(v2), 0.02, torch.tensor(eloc), 4).numpy()
    np.testing.assert_allclose(got, odmc.comput_S(-5.1, -5.0, 0.7, v2, 0.02, eloc, 4), rtol=1e-14)
    # first DMC block (main_dmc.py:115-124): per-walker e_trial = e_est = total_e energies (complex,
    # as total_e returns them) and a per-walker branch cut 10 * esigma
    e0 = eloc + rng.normal(0, 0.3, 40) + 1j * rng.normal(0, 0.1, 40)
    bc = np.full(40, 10.0) * 0.05
    got = comput_S(torch.tensor(e0), torch.tensor(e0), torch.tensor(bc), torch.tensor(v2), 0.02,
                   torch.tensor(eloc + 0j), 4).numpy()
    want = odmc.comput_S(e0, e0, bc, v2, 0.02, eloc, 4)
    assert want.shape == (40,)
    np.testing.assert_allclose(got, want, rtol=1e-14)
    got = comput_S(e0, e0, bc, torch.tensor(v2), 0.02, torch.tensor(eloc), 4).numpy()   # numpy arrays
    np.testing.assert_allclose(got, want, rtol=1e-14)


@pytest.mark.gpu
def test_dmc_propagate_step_c_atom():
    """One dmc_propagate_run step (drift-diffusion + pp energies + weights) on the C-atom ccECP
    config driven like main_dmc.py:123-177: finite energies, positive weights, and the same
    positions as the stand-alone drift-diffusion step with the same Philox key."""
    from oracle import pphamiltonian as opp, system
    from aiqmc import spin_indices
    from aiqmc.DMC import dmc
    from aiqmc.DMC.drift_diffusion import propose_drift_diffusion
    from aiqmc.VMC.VMCmcstep import PhiloxKey
    from aiqmc.wavefunction_Ynlm import nn
    s = system.make_system("C_ecp")
    par, anti, npar, nanti = spin_indices.jastrow_indices_ee(spins=s.spins, nelectrons=4)
    up, dn = spin_indices.spin_indices_h(s.spins)
    network = nn.make_ai_net(ndim=3, nelectrons=4, natoms=1, nspins=(2, 2), charges=s.charges,
                             parallel_indices=par, antiparallel_indices=anti, n_parallel=npar,
                             n_antiparallel=nanti, spin_up_indices=up, spin_down_indices=dn)
    params = system.init_params(np.random.default_rng(8), s, randomize_aux=True)
    e = opp.c_atom_ccecp()
    B = 256
    pos = torch.tensor(system.init_electrons(np.random.default_rng(9), s.atoms, s.charges, B, 1.0), device="cuda")
    data = nn.AINetData(positions=pos, spins=s.spins, atoms=s.atoms, charges=s.charges)
    run = dmc.dmc_propagate(network.apply, None, network.apply, 2, 4, 1, 3, B, 0.01, 1, s.charges, s.spins,
                            e.rn_local, e.local_coes, e.local_exps, e.rn_non_local, e.non_local_coes,
                            e.non_local_exps)
    w0 = torch.ones(B, dtype=torch.float64, device="cuda")
    eloc, w, new = run(params, PhiloxKey(3, 0), data, w0, torch.full((B,), 10.0), -3.0, -3.1)
    torch.cuda.synchronize()
    assert torch.isfinite(eloc.real).all() and torch.isfinite(w).all() and bool((w > 0).all())
    # same T-moves + drift-diffusion outside: identical positions (deterministic Philox draws)
    from aiqmc.DMC.Tmoves import compute_tmoves
    tm = compute_tmoves(2, 0.01, 4, 1, 3, nn.make_log_network(network.apply), e.rn_non_local, e.non_local_coes,
                        e.non_local_exps)
    pos_t, _ = tm(data, params, PhiloxKey(3 + 3, 0))
    data_t = nn.AINetData(positions=pos_t, spins=s.spins, atoms=s.atoms, charges=s.charges)
    dd = propose_drift_diffusion(network.apply, 0.01, 3, 4, B)
    new2, _, td, go, gn = dd(params, PhiloxKey(3, 0), data_t)
    torch.cuda.synchronize()
    assert torch.equal(new.positions, new2.positions)


# ----------------------------------------------------------------------------- T-moves

def test_searchsorted_scan_matches_numpy_on_sorted():
    rng = np.random.default_rng(0)
    for n in range(1, 40):
        a = np.sort(rng.uniform(size=n))
        for q in np.concatenate([rng.uniform(size=8), a[:3], [-1.0, 2.0]]):
            assert odmc.searchsorted_scan(a, q) == np.searchsorted(a, q)
    # complex lexicographic order: equal real parts compare the imaginary parts
    assert odmc.searchsorted_scan(np.array([1 - 1j, 1 + 0j, 1 + 1j]), 1.0) == 1


def _c_atom():
    from oracle import network, system
    s = system.make_system("C_ecp")
    return s, network


def test_tmoves_zero_nonlocal_never_moves():
    """v_l = 0: every t_amp is 0, norm = back_norm = 1, acceptance 1, no electron moves."""
    from oracle import pphamiltonian as opp, system
    s, network = _c_atom()
    rng = np.random.default_rng(5)
    params = system.init_params(rng, s, randomize_aux=True)
    ecp = opp.ECP([[1.0]], [[0.0]], [[1.0]], [[[2.0], [2.0]]], [[[0.0], [0.0]]], [[[1.0], [1.0]]], 1)
    pos = torch.tensor(system.init_electrons(rng, s.atoms, s.charges, 1, 1.0)[0])
    new, acc = odmc.tmoves(network.Network(s), network.to_torch(params), ecp, pos, opp.haar_rotations(rng, 1)[0],
                           0.0, np.full(4, 0.999), 0.5)
    np.testing.assert_array_equal(new.numpy(), pos.numpy())
    np.testing.assert_allclose(acc, 1.0, rtol=0, atol=1e-15)


def test_tmoves_golden_fixture(golden_dir):
    """The committed fixture is what the oracle computes (first two walkers recomputed), and
    every moved electron sits on its own shell |x| = r_i (atom at the origin, E2; to the
    1e-8 of the reference's 8-digit grid literals)."""
    import os
    from oracle import pphamiltonian as opp
    s, network = _c_atom()
    g = dict(np.load(os.path.join(golden_dir, "C_tmoves.npz")))
    net = network.Network(s)
    from oracle import system
    pt = network.to_torch(system.unflatten_params(system.init_params(np.random.default_rng(0), s), g["params_flat"]))
    ecp = {"ccecp": opp.c_atom_ccecp(),
           "attractive": opp.ECP([[1.0]], [[0.0]], [[1.0]], [[[2.0], [1.0]]], [[[-3.0], [-5.0]]], [[[0.7], [0.4]]], 1)}
    for name in ("ccecp", "attractive"):
        new, pos = g[f"new_{name}"].reshape(-1, 4, 3), g["pos"].reshape(-1, 4, 3)
        np.testing.assert_allclose(np.linalg.norm(new, axis=-1), np.linalg.norm(pos, axis=-1), rtol=1e-7)  # 8-digit grid literals
        for b in range(2):
            nb, ab = odmc.tmoves(net, pt, ecp[name], torch.tensor(g["pos"][b]), g["rot"][b], g["u_sel"][b],
                                 g["u_acc"][b], float(g[f"tstep_{name}"]))
            np.testing.assert_allclose(nb.numpy(), g[f"new_{name}"][b], rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(ab, g[f"acc_{name}"][b], rtol=1e-10)
    assert (np.abs(g["new_attractive"] - g["pos"]).sum() > 0)


def _tm_ctx(dtype, ecp, sysname="C_ecp"):
    from oracle import system
    from aiqmc import _lib
    s = system.make_system(sysname)
    t = s.tables()
    ctx = _lib.Context(s.nelectrons, s.natoms, s.nspins, s.atoms, s.charges, t["spin_up_indices"],
                       t["spin_down_indices"], t["parallel_indices"], t["antiparallel_indices"], dtype=dtype, device=0)
    ctx.set_ecp(ecp.rn_local, ecp.local_coes, ecp.local_exps, ecp.rn_non_local, ecp.non_local_coes,
                ecp.non_local_exps, ecp.list_l)
    return s, ctx


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ccecp", "attractive"])
def test_tmoves_match_golden(golden_dir, name):
    """HIP T-moves (fp64, injected draws) reproduce the oracle fixture: selections exact,
    positions to 1e-9, acceptance to 1e-8."""
    import os
    from oracle import pphamiltonian as opp
    g = dict(np.load(os.path.join(golden_dir, "C_tmoves.npz")))
    ecp = opp.c_atom_ccecp() if name == "ccecp" else opp.ECP([[1.0]], [[0.0]], [[1.0]], [[[2.0], [1.0]]],
                                                            [[[-3.0], [-5.0]]], [[[0.7], [0.4]]], 1)
    s, ctx = _tm_ctx(torch.float64, ecp)
    ctx.set_params(g["params_flat"])
    pos = torch.tensor(g["pos"], device="cuda").contiguous()
    acc = ctx.dmc_tmoves(pos, float(g[f"tstep_{name}"]), rot=torch.tensor(g["rot"]), u_sel=torch.tensor(g["u_sel"]),
                         u_acc=torch.tensor(g["u_acc"]))
    torch.cuda.synchronize()
    np.testing.assert_allclose(pos.cpu().numpy(), g[f"new_{name}"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(acc.cpu().numpy(), g[f"acc_{name}"], rtol=1e-8, atol=1e-10)


def _c2_tables(name):
    from oracle import pphamiltonian as opp
    if name == "ccecp":
        return opp.c2_ccecp()
    return opp.ECP([[1.0], [1.0]], [[0.0], [0.0]], [[1.0], [1.0]], [[[2.0], [1.0]]] * 2, [[[-3.0], [-5.0]]] * 2,
                   [[[0.7], [0.4]]] * 2, 1)


def test_c2_tmoves_golden_fixture(golden_dir):
    """C2 example (atoms at z = -+1): the fixture is what the oracle computes (one walker
    recomputed), moved electrons sit at |x_i| = r_ia about the ORIGIN (E2) and some move."""
    import os
    from oracle import network, system
    g = dict(np.load(os.path.join(golden_dir, "C2_tmoves.npz")))
    s = system.make_system("C2_ecp")
    net = network.Network(s)
    pt = network.to_torch(system.unflatten_params(system.init_params(np.random.default_rng(0), s), g["params_flat"]))
    nb, ab = odmc.tmoves(net, pt, _c2_tables("attractive"), torch.tensor(g["pos"][0]), g["rot"][0], g["u_sel"][0],
                         g["u_acc"][0], float(g["tstep_attractive"]))
    np.testing.assert_allclose(nb.numpy(), g["new_attractive"][0], rtol=1e-12, atol=1e-12)
    new, pos = g["new_attractive"].reshape(-1, 8, 3), g["pos"].reshape(-1, 8, 3)
    moved = np.abs(new - pos).sum(-1) > 0
    assert moved.any()
    r_new = np.linalg.norm(new, axis=-1)
    r_ia = np.linalg.norm(pos[:, :, None, :] - s.atoms[None, None], axis=-1)      # [B, N, A]
    ok = np.min(np.abs(r_new[..., None] - r_ia), axis=-1) < 1e-6
    assert ok[moved].all()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ccecp", "attractive"])
def test_c2_tmoves_match_golden(golden_dir, name):
    """HIP T-moves on the C2 example (fp64, injected draws) reproduce the oracle fixture."""
    import os
    g = dict(np.load(os.path.join(golden_dir, "C2_tmoves.npz")))
    s, ctx = _tm_ctx(torch.float64, _c2_tables(name), "C2_ecp")
    ctx.set_params(g["params_flat"])
    pos = torch.tensor(g["pos"], device="cuda").contiguous()
    acc = ctx.dmc_tmoves(pos, float(g[f"tstep_{name}"]), rot=torch.tensor(g["rot"]), u_sel=torch.tensor(g["u_sel"]),
                         u_acc=torch.tensor(g["u_acc"]))
    torch.cuda.synchronize()
    np.testing.assert_allclose(pos.cpu().numpy(), g[f"new_{name}"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(acc.cpu().numpy(), g[f"acc_{name}"], rtol=1e-8, atol=1e-10)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_tmoves_full_batch_properties(dtype):
    """4096 walkers, Philox draws: finite acceptance, every electron stays on its shell
    |x_i| (moves go to r_i p_q R, atom at the origin), the attractive table moves electrons,
    and a walker's result does not depend on the batch it runs in (host draws)."""
    from oracle import pphamiltonian as opp, system
    ecp = opp.ECP([[1.0]], [[0.0]], [[1.0]], [[[2.0], [1.0]]], [[[-3.0], [-5.0]]], [[[0.7], [0.4]]], 1)
    s, ctx = _tm_ctx(dtype, ecp)
    rng = np.random.default_rng(12)
    ctx.set_params(system.flatten_params(system.init_params(rng, s, randomize_aux=True)))
    B = 4096
    x0 = torch.tensor(system.init_electrons(rng, s.atoms, s.charges, B, 1.0), dtype=dtype, device="cuda")
    pos = x0.clone()
    acc = ctx.dmc_tmoves(pos, 0.3, seed=7, offset=1)
    torch.cuda.synchronize()
    assert torch.isfinite(acc).all()
    tol = 1e-5 if dtype == torch.float32 else 1e-7   # the grid's 8-digit literals are not unit vectors
    r0, r1 = x0.reshape(B, 4, 3).norm(dim=-1), pos.reshape(B, 4, 3).norm(dim=-1)
    assert torch.allclose(r1, r0, rtol=tol, atol=tol)
    assert bool(((pos - x0).abs().reshape(B, 4, 3).sum(-1) > 0).any())
    # host draws: a sub-batch gives the same walkers' results
    rot = torch.tensor(opp.haar_rotations(rng, B), dtype=dtype)
    us = torch.tensor(np.where(rng.uniform(size=B) < 0.5, 0.0, rng.uniform(size=B) * 1e-3), dtype=dtype)
    ua = torch.tensor(rng.uniform(size=(B, 4)), dtype=dtype)
    pa = x0.clone()
    ctx.dmc_tmoves(pa, 0.3, rot=rot, u_sel=us, u_acc=ua)
    sub = torch.arange(100, 164)
    pb = x0[sub].clone().contiguous()
    ctx.dmc_tmoves(pb, 0.3, rot=rot[sub], u_sel=us[sub], u_acc=ua[sub])
    torch.cuda.synchronize()
    assert torch.equal(pa[sub], pb)


@pytest.mark.gpu
def test_compute_tmoves_dropin(golden_dir):
    """aiqmc.DMC.Tmoves.compute_tmoves (reference signature) with injected draws equals the
    fixture; the walker data are not modified in place."""
    import os
    from oracle import pphamiltonian as opp
    from aiqmc import spin_indices
    from aiqmc.DMC.Tmoves import HostTmoveDraws, compute_tmoves
    from aiqmc.wavefunction_Ynlm import nn
    s, _ = _c_atom()
    g = dict(np.load(os.path.join(golden_dir, "C_tmoves.npz")))
    par, anti, npar, nanti = spin_indices.jastrow_indices_ee(spins=s.spins, nelectrons=4)
    up, dn = spin_indices.spin_indices_h(s.spins)
    network = nn.make_ai_net(ndim=3, nelectrons=4, natoms=1, nspins=(2, 2), charges=s.charges,
                             parallel_indices=par, antiparallel_indices=anti, n_parallel=npar,
                             n_antiparallel=nanti, spin_up_indices=up, spin_down_indices=dn)
    e = opp.c_atom_ccecp()
    tm = compute_tmoves(2, float(g["tstep_ccecp"]), 4, 1, 3, nn.make_log_network(network.apply), e.rn_non_local,
                        e.non_local_coes, e.non_local_exps)
    pos = torch.tensor(g["pos"], device="cuda")
    keep = pos.clone()
    data = nn.AINetData(positions=pos, spins=s.spins, atoms=s.atoms, charges=s.charges)
    from oracle import system
    params = system.unflatten_params(system.init_params(np.random.default_rng(0), s), g["params_flat"])
    new, acc = tm(data, params, HostTmoveDraws(torch.tensor(g["rot"]), torch.tensor(g["u_sel"]),
                                                         torch.tensor(g["u_acc"])))
    torch.cuda.synchronize()
    assert torch.equal(pos, keep)
    np.testing.assert_allclose(new.cpu().numpy(), g["new_ccecp"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(acc.cpu().numpy(), g["acc_ccecp"], rtol=1e-8, atol=1e-10)
    with pytest.raises(TypeError):
        compute_tmoves(2, 0.1, 4, 1, 3, lambda *a: None, e.rn_non_local, e.non_local_coes, e.non_local_exps)


# ----------------------------------------------------------------------------- DMC driver pieces

def test_reindex_walkers_follows_driver():
    """main_dmc.py:215-233: sorted unique comb indices, killed walkers replaced by the last
    unique walker plus U[0,1) noise."""
    from aiqmc.DMC.main_dmc import reindex_walkers
    rng = np.random.default_rng(6)
    x1 = torch.tensor(rng.standard_normal((6, 12)))
    idx = torch.tensor([4, 1, 1, 4, 4, 0], dtype=torch.int32)
    noise = torch.tensor(rng.uniform(size=(6, 12)))
    got = reindex_walkers(x1, idx, noise)
    unique = np.unique(idx.numpy())
    temp = x1.numpy()[unique]
    want = np.concatenate([temp, temp[-1] + noise.numpy()[:6 - len(unique)]])
    np.testing.assert_array_equal(got.numpy(), want)
    full = reindex_walkers(x1, torch.arange(6), noise)
    assert torch.equal(full, x1)


def test_estimate_and_total_energy_dropins():
    from aiqmc.DMC.estimate_energy import estimate_energy
    from aiqmc.DMC.total_energy import calculate_total_energy
    e = torch.tensor([[1.0, 2.0], [3.0, 0.0]])
    w = torch.tensor([[1.0, 1.0], [2.0, 0.0]])
    assert abs(estimate_energy(e, w).item() - np.average(e.numpy(), weights=w.numpy())) < 1e-12
    el = torch.tensor([1.0 + 1j, 3.0 - 1j, 2.0 + 0j], dtype=torch.complex128)
    te = calculate_total_energy(lambda params, key, data: (el, None))
    e_l, var = te(None, 0, None)
    d = el.numpy() - el.numpy().mean()
    assert torch.equal(e_l, el) and abs(var.item() - np.mean(d * np.conj(d))) < 1e-12


@pytest.mark.gpu
def test_main_dmc_driver_runs_from_vmc_checkpoint(tmp_path):
    """aiqmc.DMC.main_dmc.main with the reference driver's arguments (single_atom_C tables),
    restarted from a VMC checkpoint written by aiqmc.checkpoint: finite block estimates, a
    DMC_states.csv row per block, walkers kept per device."""
    from oracle import pphamiltonian as opp, system
    from aiqmc import checkpoint
    from aiqmc.DMC import main_dmc
    from aiqmc.wavefunction_Ynlm import nn
    s = system.make_system("C_ecp")
    B = 128
    params = system.init_params(np.random.default_rng(8), s, randomize_aux=True)
    pos = torch.tensor(system.init_electrons(np.random.default_rng(9), s.atoms, s.charges, B, 1.0))
    checkpoint.save(str(tmp_path), 5, nn.AINetData(positions=pos, spins=s.spins, atoms=s.atoms, charges=s.charges),
                    params, np.zeros(1))
    e = opp.c_atom_ccecp()
    est, data, w = main_dmc.main(atoms=s.atoms, charges=s.charges, spins=s.spins, tstep=0.01, nelectrons=4,
                                 nsteps=1, natoms=1, ndim=3, batch_size=B, iterations=2, nblocks=2, feedback=1.0,
                                 nspins=(2, 2), save_path=str(tmp_path), restore_path=None, Rn_local=e.rn_local,
                                 Local_coes=e.local_coes, Local_exps=e.local_exps, Rn_non_local=e.rn_non_local,
                                 Non_local_coes=e.non_local_coes, Non_local_exps=e.non_local_exps,
                                 save_frequency=1e9, structure=None, seed=3)
    torch.cuda.synchronize()
    assert len(est) == 2 and all(np.isfinite(est))
    assert data.positions.shape == (B, 12) and torch.isfinite(data.positions).all()
    rows = open(tmp_path / "DMC_states.csv").read().strip().split("\n")
    assert rows[0] == "block,energy,positions" and len(rows) >= 3


# ----------------------------------------------------------------------------- multi-step DMC trajectories

_TRAJ_TABLES = {
    "ccecp": lambda opp: opp.c_atom_ccecp(),
    "attractive": lambda opp: opp.ECP([[1.0]], [[0.0]], [[1.0]], [[[2.0], [1.0]]], [[[-3.0], [-5.0]]],
                                      [[[0.7], [0.4]]], 1),
    # the product's zero tables (aiqmc.systems.all_electron_tables); the fixture was made with the
    # oracle's identical ECP([[1]], [[0]], [[1]], [[[2]]*3], [[[0]]*3], [[[1]]*3], 2)
    "ne_allelectron": lambda opp: __import__("aiqmc.systems", fromlist=["x"]).all_electron_tables("Ne"),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ccecp", "attractive", "ne_allelectron"])
def test_dmc_trajectory_matches_oracle(golden_dir, name):
    """The driver's block loop (aiqmc.DMC.main_dmc.dmc_blocks: dmc_propagate_run steps = T-moves,
    drift-diffusion, pp energies, weights; then comb, re-indexing, e_est / e_trial feedback) with
    every draw injected reproduces the oracle's chain (oracle.dmc.dmc_blocks, main_dmc.py:113-244):
    first block with per-walker e_trial = e_est, branch cut 10 std(E_L); positions to 1e-9,
    weights to 1e-12 relative, comb indices exact.  ne_allelectron: all-electron Ne (10 e-)
    through the pp-only DMC step with zero ECP coefficients (BASELINE's "Ne + DMC")."""
    import os
    from oracle import pphamiltonian as opp, system
    from aiqmc import systems
    from aiqmc.DMC import dmc, main_dmc
    from aiqmc.DMC.Tmoves import HostTmoveDraws
    from aiqmc.VMC.VMCmcstep import HostDraws
    from aiqmc.wavefunction_Ynlm import nn
    sysname = "Ne" if name == "ne_allelectron" else "C_ecp"
    g = dict(np.load(os.path.join(golden_dir, f"{'Ne' if sysname == 'Ne' else 'C'}_dmc_{name}.npz")))
    s = systems.make_system(sysname)
    N, A = s.nelectrons, s.natoms
    network = s.make_network()
    params = system.unflatten_params(system.init_params(np.random.default_rng(0), system.make_system(sysname)),
                                     g["params_flat"])
    e = _TRAJ_TABLES[name](opp)
    B = g["x0"].shape[0]
    nblocks, iters = g["newinds"].shape[0], g["weights"].shape[0] // g["newinds"].shape[0]
    tstep = float(g["tstep"])
    run = dmc.dmc_propagate(network.apply, nn.make_log_network(network.apply), network.apply, e.list_l, N, A, 3, B,
                            tstep, 1, s.charges, s.spins, e.rn_local, e.local_coes, e.local_exps, e.rn_non_local,
                            e.non_local_coes, e.non_local_exps)
    ctx = network.apply._aiqmc_network.bind(params, s.atoms, torch.float64)
    data = nn.AINetData(positions=torch.tensor(g["x0"], device="cuda").contiguous(), spins=s.spins, atoms=s.atoms,
                        charges=s.charges)
    e_l0 = torch.complex(torch.tensor(g["e_l0_re"]), torch.tensor(g["e_l0_im"])).cuda()
    d0 = e_l0 - e_l0.mean()
    var0 = (d0 * d0.conj()).mean()
    T = lambda a: torch.tensor(a)
    step_key = lambda k: dmc.HostDmcDraws(HostTmoveDraws(T(g["rot_tm"][k]), T(g["u_sel"][k]), T(g["u_acc"][k])),
                                          HostDraws(T(g["gauss1"][k]), T(g["gauss2"][k]), T(g["u"][k])),
                                          T(g["rot_old"][k]), T(g["rot_new"][k]))
    block_draws = lambda b: (float(g["u_comb"][b]), T(g["extra"][b]))
    est, data, w, trace = main_dmc.dmc_blocks(run, ctx, params, data, e_l0, var0, nblocks, iters, float(g["feedback"]),
                                              step_key, block_draws, trace=True)
    torch.cuda.synchronize()
    for k in range(nblocks * iters):
        np.testing.assert_allclose(trace["positions"][k].cpu().numpy(), g["positions"][k], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(trace["energy"][k].real.cpu().numpy(), g["energy_re"][k], rtol=0, atol=1e-6)
        np.testing.assert_allclose(trace["weights"][k].cpu().numpy(), g["weights"][k], rtol=1e-12)
    for b in range(nblocks):
        np.testing.assert_array_equal(trace["newinds"][b].cpu().numpy(), g["newinds"][b])
        assert abs(trace["comb_weight"][b] - g["comb_weight"][b]) <= 1e-12 * abs(g["comb_weight"][b])
        assert abs(est[b] - g["e_est"][b]) < 1e-9 and abs(trace["e_trial"][b] - g["e_trial"][b]) < 1e-9
    np.testing.assert_allclose(data.positions.cpu().numpy(), g["x_final"], rtol=1e-9, atol=1e-9)
