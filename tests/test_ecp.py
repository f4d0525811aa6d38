"""Pseudopotential (ccECP) local energy: oracle known answers (CPU) and HIP parity (GPU).

Reference: AIQMCrelease3/Energy/pphamiltonian.py:130-190,
pseudopotential/pseudopotential.py:86-318, pseudopotential/pp_energy_test.py:45-105;
config example/single_atom_C/single_atom_C.py (C atom, Z_eff = 4, list_l = 2).
The reference has no ECP tests and cannot run here (JAX absent): the oracle is
pinned by quadrature identities and closed forms below, and the kernels by the
oracle's golden fixture tests/golden/C_ecp.npz (make_golden_ecp.py).

Tolerances: float64 kernels |dE| <= 1e-6 Ha (the north_star bound; observed
~1e-12), quadrature log psi to 1e-9; float32 kernels 2e-4 relative on Re E_L.
"""
import math
import os

import numpy as np
import pytest
import torch

from oracle import pphamiltonian as pp


# ----------------------------------------------------------------------------- CPU: oracle

def test_grid_weights_and_norms():
    groups, w = pp.quadrature_grids()
    assert [g.shape[0] for g in groups] == [6, 12, 8, 24]
    assert abs(sum(len(g) * wi for g, wi in zip(groups, w)) - 1.0) < 1e-15
    for g in groups:
        np.testing.assert_allclose(np.linalg.norm(g, axis=1), 1.0, atol=2e-8)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_grid_integrates_legendre(seed):
    """The 50-point octahedral rule (Mitas-Shirley-Ceperley) integrates P_l(u.p) exactly
    for l <= 11 (weights already normalised to the sphere average)."""
    rng = np.random.default_rng(seed)
    u = rng.standard_normal(3)
    u /= np.linalg.norm(u)
    groups, w = pp.quadrature_grids()
    rot = pp.haar_rotations(rng, 1)[0]
    for l in range(1, 8):
        s = 0.0
        for g, wi in zip(groups, w):
            x = pp.rotate_points(rot, g) @ u
            s += wi * np.polynomial.legendre.legval(x, [0] * l + [1]).sum()
        assert abs(s) < 1e-7, (l, s)


def test_local_pp_closed_form():
    ecp = pp.c_atom_ccecp()
    pos = torch.tensor([0.3, -0.2, 0.9, 1.1, 0.4, -0.5], dtype=torch.float64)
    atoms = torch.zeros(1, 3, dtype=torch.float64)
    charges = torch.tensor([4.0], dtype=torch.float64)
    got = pp.local_pp_energy(ecp, pos, atoms, charges).item()
    want = 0.0
    for i in range(2):
        r = float(np.linalg.norm(pos.numpy()[3 * i:3 * i + 3]))
        want += -4.0 / r
        for n, c, a in zip([1.0, 3.0, 2.0], [4.0, 57.74008, -25.81955], [14.43502, 8.39889, 7.38188]):
            want += c * r ** (n - 2) * math.exp(-a * r * r)      # pseudopotential.py:95,101-102
    assert abs(got - want) < 1e-13


class _ConstNet:
    """log psi = const: every ratio is the group weight."""

    def __init__(self, N):
        self.N, self.A = N, 1
        self.atoms = torch.zeros(1, 3, dtype=torch.float64)
        self.charges = torch.tensor([4.0], dtype=torch.float64)

    def apply(self, params, x):
        return torch.tensor(0.3, dtype=torch.float64), torch.tensor(-1.7, dtype=torch.float64)


@pytest.mark.parametrize("seed", [3, 4])
def test_nonlocal_constant_wavefunction(seed):
    """ratio == w: sum_q w P_0 = 1/(4 pi) (E5); the l = 1 term vanishes by inversion
    symmetry of every grid group; so E_nl = sum_i v_0(r_i) / (4 pi), any rotation."""
    rng = np.random.default_rng(seed)
    ecp = pp.ECP([[1.0]], [[0.0]], [[1.0]], [[[2.0], [1.0]]], [[[3.0], [5.0]]], [[[0.7], [0.4]]], 1)
    net = _ConstNet(2)
    pos = torch.tensor(rng.standard_normal(6))
    rot = pp.haar_rotations(rng, 1)[0]
    nl, _ = pp.nonlocal_pp_energy(net, None, ecp, pos, rot)
    want = 0.0
    for i in range(2):
        r = float(np.linalg.norm(pos.numpy()[3 * i:3 * i + 3]))
        want += 3.0 * r ** 2 * math.exp(-0.7 * r * r) / (4 * math.pi)
    assert abs(nl.real.item() - want) < 1e-12 and abs(nl.imag.item()) < 1e-12


def test_cos_theta_quirk():
    """E3: cos(theta) is the true cosine divided by sqrt(points in the group)."""
    pos = torch.tensor([0.3, -0.2, 0.9], dtype=torch.float64)
    atoms = torch.zeros(1, 3, dtype=torch.float64)
    groups, _ = pp.quadrature_grids()
    for g in groups:
        cos, cfg = pp.rotated_configurations(pos, atoms, g)
        u = pos.numpy() / np.linalg.norm(pos.numpy())
        true = g @ u / np.linalg.norm(g, axis=1)
        np.testing.assert_allclose(cos[0, 0].numpy(), true / math.sqrt(len(g)), rtol=1e-7, atol=1e-9)
        # E2: the moved electron sits at r p_q (atom at the origin here)
        np.testing.assert_allclose(cfg[0, 0].numpy(), np.linalg.norm(pos.numpy()) * g, rtol=1e-15)


@pytest.mark.parametrize("name,n3,B", [("C_ecp", 12, 4), ("C2_ecp", 24, 4), ("CO2_ecp", 48, 2)])
def test_golden_fixture_consistent(golden_dir, name, n3, B):
    g = dict(np.load(os.path.join(golden_dir, f"{name}.npz")))
    assert g["pos"].shape == (B, n3) and g["rot"].shape == (B, 3, 3)
    np.testing.assert_allclose(np.einsum("bij,bkj->bik", g["rot"], g["rot"]), np.broadcast_to(np.eye(3), (B, 3, 3)),
                               atol=1e-12)
    assert np.all(np.isfinite(g["e_re"])) and np.all(np.isfinite(g["logq_re"]))


# ----------------------------------------------------------------------------- GPU: HIP vs oracle

def _ecp_ctx(dtype, name="C_ecp"):
    from oracle import system
    from aiqmc import _lib
    s = system.make_system(name)
    t = s.tables()
    ctx = _lib.Context(s.nelectrons, s.natoms, s.nspins, s.atoms, s.charges, t["spin_up_indices"],
                       t["spin_down_indices"], t["parallel_indices"], t["antiparallel_indices"], dtype=dtype, device=0)
    e = {"C_ecp": pp.c_atom_ccecp, "C2_ecp": pp.c2_ccecp, "CO2_ecp": pp.co2_ccecp}[name]()
    ctx.set_ecp(e.rn_local, e.local_coes, e.local_exps, e.rn_non_local, e.non_local_coes, e.non_local_exps, e.list_l)
    return s, ctx


def test_product_ccecp_tables_equal_the_oracle_tables():
    """aiqmc.systems.ccecp_tables (what drivers and bench.py upload) == the oracle's tables."""
    from aiqmc import systems
    for name, o in [("C_ecp", pp.c_atom_ccecp()), ("C2_ecp", pp.c2_ccecp()), ("CO2_ecp", pp.co2_ccecp())]:
        t = systems.ccecp_tables(name)
        for k in ("rn_local", "local_coes", "local_exps", "rn_non_local", "non_local_coes", "non_local_exps"):
            np.testing.assert_array_equal(getattr(t, k), getattr(o, k), err_msg=f"{name}.{k}")
        assert t.list_l == o.list_l


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["C_ecp", "C2_ecp", "CO2_ecp"])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_ecp_local_energy_golden(golden_dir, dtype, name):
    """C atom, the C2 example (two ccECP centres off the origin: quirk E2, the rotated
    electron NOT offset by its atom, changes the answer there) and the CO2 example (three
    atoms, carbon and oxygen ccECP blocks, 16 electrons)."""
    g = dict(np.load(os.path.join(golden_dir, f"{name}.npz")))
    s, ctx = _ecp_ctx(dtype, name)
    ctx.set_params(g["params_flat"])
    pos = torch.tensor(g["pos"], dtype=dtype, device="cuda")
    rot = torch.tensor(g["rot"], dtype=dtype, device="cuda")
    e, lq, pq = ctx.local_energy_ecp(pos, rot=rot, want_quadrature=True)
    torch.cuda.synchronize()
    er, ei = e.real.double().cpu().numpy(), e.imag.double().cpu().numpy()
    if dtype == torch.float64:
        assert np.max(np.abs(er - g["e_re"])) <= 1e-6, (er, g["e_re"])
        assert np.max(np.abs(ei - g["e_im"])) <= 1e-6, (ei, g["e_im"])
        np.testing.assert_allclose(lq.cpu().numpy(), g["logq_re"], rtol=1e-9, atol=1e-9)
        ph = pq.cpu().numpy()
        np.testing.assert_allclose(np.cos(ph), np.cos(g["logq_im"]), atol=1e-9)
        np.testing.assert_allclose(np.sin(ph), np.sin(g["logq_im"]), atol=1e-9)
    else:
        np.testing.assert_allclose(er, g["e_re"], rtol=2e-4, atol=2e-3)
        assert np.max(np.abs(ei - g["e_im"])) <= 2e-3


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["Z4-2-2", "Z3-2-2"])
def test_ecp_packed_three_atoms_match_oracle(name):
    """pp E_L of N <= 8 systems with 3 atoms (the packed quadrature launch k_quad_value with
    A >= 3 -- wider layer-0 lane records than any reference example) against the fp64 oracle,
    live: the carbon ccECP block on every atom (the tables are independent of the charges),
    2 walkers, injected rotations."""
    from oracle import network, system
    from aiqmc import _lib
    s = system.make_system(name)
    assert (s.nelectrons, s.natoms) in _lib.supported_shapes() or pytest.skip("shape not built")
    c = pp.c_atom_ccecp()
    A = s.natoms
    rep = lambda a: np.concatenate([a] * A, axis=0)
    ecp = pp.ECP(rep(c.rn_local), rep(c.local_coes), rep(c.local_exps), rep(c.rn_non_local), rep(c.non_local_coes),
                 rep(c.non_local_exps), 2)
    rng = np.random.default_rng(71)
    params = system.init_params(rng, s, randomize_aux=True)
    pos = system.init_electrons(rng, s.atoms, s.charges, 2, 1.0)
    rots = pp.haar_rotations(rng, 2)
    ref, _, _, _ = pp.batch_local_energy_pp(network.Network(s), network.to_torch(params), ecp, torch.tensor(pos), rots)
    t = s.tables()
    ctx = _lib.Context(s.nelectrons, s.natoms, s.nspins, s.atoms, s.charges, t["spin_up_indices"],
                       t["spin_down_indices"], t["parallel_indices"], t["antiparallel_indices"], dtype=torch.float64,
                       device=0)
    ctx.set_ecp(ecp.rn_local, ecp.local_coes, ecp.local_exps, ecp.rn_non_local, ecp.non_local_coes,
                ecp.non_local_exps, ecp.list_l)
    ctx.set_params(system.flatten_params(params))
    e = ctx.local_energy_ecp(torch.tensor(pos, device="cuda"), rot=torch.tensor(rots, device="cuda"))
    torch.cuda.synchronize()
    ref = ref.detach().numpy()
    assert np.max(np.abs(e.real.cpu().numpy() - ref.real)) <= 1e-6, (e, ref)
    assert np.max(np.abs(e.imag.cpu().numpy() - ref.imag)) <= 1e-6, (e, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["C_ecp", "C2_ecp", "CO2_ecp"])
def test_ecp_reuse_matches_scratch(golden_dir, name):
    """Quadrature configurations from the walker cache == evaluated from scratch (fp64)."""
    g = dict(np.load(os.path.join(golden_dir, f"{name}.npz")))
    s, ctx = _ecp_ctx(torch.float64, name)
    ctx.set_params(g["params_flat"])
    pos = torch.tensor(g["pos"], device="cuda")
    rot = torch.tensor(g["rot"], device="cuda")
    e1, l1, p1 = ctx.local_energy_ecp(pos, rot=rot, want_quadrature=True)
    ctx.set_proposal_reuse(False)
    e2, l2, p2 = ctx.local_energy_ecp(pos, rot=rot, want_quadrature=True)
    torch.cuda.synchronize()
    np.testing.assert_allclose(l1.cpu().numpy(), l2.cpu().numpy(), rtol=1e-11, atol=1e-11)
    assert torch.max(torch.abs(e1 - e2)).item() < 1e-10


@pytest.mark.gpu
def test_ecp_full_batch_walker_independent():
    """4096 fp32 walkers with Philox rotations: finite, and a walker's energy does not depend
    on the rest of the batch (no batch coupling in the pp Hamiltonian) given its rotation."""
    from oracle import system
    s, ctx = _ecp_ctx(torch.float64)
    rng = np.random.default_rng(7)
    ctx.set_params(system.flatten_params(system.init_params(rng, s, randomize_aux=True)))
    B = 4096
    pos = torch.tensor(system.init_electrons(rng, s.atoms, s.charges, B, 1.0), device="cuda")
    e = ctx.local_energy_ecp(pos, seed=5, offset=0)
    rot = torch.tensor(pp.haar_rotations(rng, B), device="cuda")
    eh = ctx.local_energy_ecp(pos, rot=rot)
    sub = torch.arange(0, B, 97, device="cuda")
    es = ctx.local_energy_ecp(pos[sub].contiguous(), rot=rot[sub].contiguous())
    torch.cuda.synchronize()
    assert torch.isfinite(e.real).all() and torch.isfinite(e.imag).all()
    assert torch.max(torch.abs(eh[sub] - es)).item() < 1e-9


@pytest.mark.gpu
def test_ecp_errors():
    from oracle import system
    from aiqmc import _lib
    s = system.make_system("C_ecp")
    t = s.tables()
    ctx = _lib.Context(s.nelectrons, s.natoms, s.nspins, s.atoms, s.charges, t["spin_up_indices"],
                       t["spin_down_indices"], t["parallel_indices"], t["antiparallel_indices"],
                       dtype=torch.float64, device=0)
    ctx.set_params(system.flatten_params(system.init_params(np.random.default_rng(0), s)))
    pos = torch.zeros(2, 12, dtype=torch.float64, device="cuda")
    with pytest.raises(RuntimeError, match="aiqmc_set_ecp has not been called"):
        ctx.local_energy_ecp(pos)
    e = pp.c_atom_ccecp()
    with pytest.raises(RuntimeError, match="list_l"):
        ctx.set_ecp(e.rn_local, e.local_coes, e.local_exps, np.zeros((1, 5, 2)), np.zeros((1, 5, 2)),
                    np.zeros((1, 5, 2)), 4)


def test_c2_quadrature_not_offset_by_atom():
    """E2 on the C2 example: the quadrature configuration of electron i about atom a puts it at
    r_ia p_q -- on a sphere about the ORIGIN, not about the atom at z = -+1."""
    from oracle import system
    s = system.make_system("C2_ecp")
    rng = np.random.default_rng(3)
    pos = torch.tensor(system.init_electrons(rng, s.atoms, s.charges, 1, 1.0)[0])
    atoms = torch.tensor(s.atoms)
    groups, _ = pp.quadrature_grids()
    cos, cfg = pp.rotated_configurations(pos, atoms, groups[0])
    x = pos.numpy().reshape(8, 3)
    r = np.linalg.norm(x[:, None, :] - s.atoms[None], axis=-1)               # [N, A]
    moved = cfg.numpy().reshape(8, 2, groups[0].shape[0], 8, 3)
    for i in range(8):
        for a in range(2):
            np.testing.assert_allclose(np.linalg.norm(moved[i, a, :, i], axis=-1), r[i, a], rtol=1e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["C_ecp", "C2_ecp"])
def test_quad_walker_order_lu_matches_partial_pivoting(name):
    """k_quad_value (N <= 8) factors each displaced configuration in its walker's recorded pivot
    order and re-runs partial pivoting for a configuration whose pivot falls below 0.1 of the
    walker's; aiqmc_debug_set_quad_pivoted(1) sends every configuration down that fallback.
    512 walkers, host Haar rotations (C2: the fallback is taken for a few % of the configurations
    in the default mode, so both branches run).  fp64: both orders agree to 1e-11 (log|psi|,
    phase, E_L).  fp32: measured against the fp64 values, the walker order is no less accurate
    than partial pivoting (max and 99.99th-percentile |error| of log|psi|, within 1.5x; measured
    on MI355X: equal maxima, 3.2e-4 C and 1.2e-3 C2, tools/quad_lu_accuracy.py) and E_L agrees
    to 1e-5 relative."""
    from oracle import system
    rng = np.random.default_rng(11)
    s0, _ = _ecp_ctx(torch.float64, name)
    params = system.flatten_params(system.init_params(rng, s0, randomize_aux=True))
    pos = system.init_electrons(rng, s0.atoms, s0.charges, 512, 1.0)
    rot = pp.haar_rotations(rng, 512)
    res = {}
    for dtype in (torch.float64, torch.float32):
        s, ctx = _ecp_ctx(dtype, name)
        ctx.set_params(params)
        p = torch.tensor(pos, device="cuda", dtype=dtype)
        r = torch.tensor(rot, device="cuda", dtype=dtype)
        for piv in (False, True):
            ctx.set_quad_pivoted(piv)
            e, l, ph = ctx.local_energy_ecp(p, rot=r, want_quadrature=True)
            torch.cuda.synchronize()
            res[(dtype, piv)] = (e.cpu().numpy().astype(np.complex128), l.double().cpu().numpy().ravel(),
                                 ph.double().cpu().numpy().ravel())
        ctx.set_quad_pivoted(False)
        e3 = ctx.local_energy_ecp(p, rot=r)
        torch.cuda.synchronize()
        assert np.array_equal(e3.cpu().numpy().astype(np.complex128), res[(dtype, False)][0])   # switch restored
    (ef, lf, pf), (ep, lp, pq) = res[(torch.float64, False)], res[(torch.float64, True)]
    assert np.isfinite(lf).all()
    np.testing.assert_allclose(lf, lp, rtol=1e-11, atol=1e-11)
    assert np.max(np.abs(np.angle(np.exp(1j * (pf - pq))))) <= 1e-10
    assert np.max(np.abs(ef - ep)) <= 1e-10
    ref = lp
    errs = {}
    for piv in (False, True):
        e32, l32, _ = res[(torch.float32, piv)]
        assert np.isfinite(l32).all()
        d = np.abs(l32 - ref)
        errs[piv] = (d.max(), np.quantile(d, 0.9999))
    assert errs[False][0] <= 1.5 * errs[True][0] + 1e-5, errs
    assert errs[False][1] <= 1.5 * errs[True][1] + 1e-6, errs
    e_a, e_b = res[(torch.float32, False)][0], res[(torch.float32, True)][0]
    assert np.max(np.abs(e_a - e_b) / np.maximum(np.abs(e_b), 1.0)) <= 1e-5
