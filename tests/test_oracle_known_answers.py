"""Pin the CPU oracle against the reference's own known-answer tests (CPU).

The reference AIQMC packages hold no tests; the vendored ferminet suite pins
the same local-energy algorithm that AIQMCrelease3 copied
(ferminet/hamiltonian.py:105-140 == AIQMCrelease3/Energy/hamiltonian.py:100-131).
Each test below re-expresses one of those tests against the oracle:
  ferminet/tests/hamiltonian_test.py:65-83    hydrogen KE = -(1 - 2/r)/2
  ferminet/tests/hamiltonian_test.py:85-120   potential energy cases
  ferminet/tests/hamiltonian_test.py:122-154  E_L == -0.5 for exact hydrogen
  ferminet/tests/hamiltonian_test.py:157-185  Laplacian == Hessian trace
  ferminet/tests/hamiltonian_test.py:187-250  network Laplacian vs Hessian (1e-10 in f64)
  ferminet/tests/network_blocks_test.py:38-45 slogdet vs numpy
plus AIQMC-specific checks: the 2,381-parameter N2 tree, the two
independent forward restatements agree, finite differences agree with AD.
"""
import numpy as np
import pytest
import torch

from oracle import hamiltonian, network, network_np, system

torch.set_default_dtype(torch.float64)


def h_atom_logabs(x):
    return -torch.abs(torch.linalg.norm(x))


def test_hydrogen_kinetic_energy():
    rng = np.random.default_rng(0)
    for _ in range(10):
        xs = torch.tensor(rng.standard_normal(3))
        ke = hamiltonian.kinetic_jvp_of_grad(h_atom_logabs)(xs)
        r = float(torch.linalg.norm(xs))
        np.testing.assert_allclose(float(ke), -(1 - 2 / r) / 2, rtol=1e-10)


def test_hydrogen_local_energy_is_minus_half():
    rng = np.random.default_rng(4)
    atoms = torch.zeros(1, 3)
    charges = torch.ones(1)
    el = hamiltonian.local_energy(h_atom_logabs, atoms, charges)
    xs = torch.tensor(rng.standard_normal((100, 3)))
    e = torch.stack([el(x) for x in xs])
    np.testing.assert_allclose(e.numpy(), -0.5, rtol=1e-10)


def test_potential_null():
    xs = torch.tensor(np.random.default_rng(1).standard_normal((1, 3)))
    r_ae = torch.linalg.norm(xs, dim=-1)[..., None, None]
    r_ee = torch.zeros(1, 1, 1)
    v = hamiltonian.potential_energy(r_ae, r_ee, torch.zeros(1, 3), torch.zeros(1))
    assert abs(float(v)) < 1e-12


def test_potential_ee():
    xs = np.random.default_rng(2).standard_normal((5, 3))
    r_ee = np.linalg.norm(xs[None] - xs[:, None], axis=-1)
    mask = ~np.eye(5, dtype=bool)
    expected = 0.5 * np.sum(1.0 / r_ee[mask])
    v = hamiltonian.potential_energy(torch.ones(5, 1, 1), torch.tensor(r_ee)[..., None], torch.zeros(1, 3),
                                     torch.zeros(1))
    np.testing.assert_allclose(float(v), expected, rtol=1e-12)


def test_potential_he2_ion():
    xs = np.random.default_rng(3).standard_normal((1, 3))
    atoms = np.array([[0, 0, -1], [0, 0, 1]], dtype=np.float64)
    r_ae = np.linalg.norm(xs - atoms, axis=-1)
    charges = np.array([2.0, 2.0])
    expected = -np.sum(charges / r_ae) + 4.0 / 2.0
    v = hamiltonian.potential_energy(torch.tensor(r_ae)[None, :, None], torch.zeros(1, 1, 1),
                                     torch.tensor(atoms), torch.tensor(charges))
    np.testing.assert_allclose(float(v), expected, rtol=1e-12)


def test_laplacian_equals_hessian_trace_hydrogen():
    rng = np.random.default_rng(5)
    for x in rng.uniform(size=(20, 3)):
        x = torch.tensor(x)
        a = hamiltonian.kinetic_jvp_of_grad(h_atom_logabs)(x)
        b = hamiltonian.kinetic_hessian(h_atom_logabs)(x)
        np.testing.assert_allclose(float(a), float(b), rtol=1e-10)


@pytest.mark.parametrize("name", ["H2", "Be", "C2"])
def test_network_laplacian_vs_hessian(name):
    s = system.make_system(name)
    p = system.init_params(np.random.default_rng(7), s, randomize_aux=True)
    net = network.Network(s)
    pt = network.to_torch(p)
    pos = torch.tensor(system.init_electrons(np.random.default_rng(8), s.atoms, s.charges, 2, 1.0))
    a, _, _ = hamiltonian.batch_local_energy(net, pt, pos, method="jvp")
    b, _, _ = hamiltonian.batch_local_energy(net, pt, pos, method="hess")
    np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=1e-10, atol=1e-10)


def test_slogdet_vs_numpy():
    rng = np.random.default_rng(9)
    for shape in [(10, 2, 2), (10, 3, 3), (4, 14, 14)]:
        a = rng.standard_normal(shape) + 1j * rng.standard_normal(shape)
        s1, l1 = torch.linalg.slogdet(torch.tensor(a))
        s2, l2 = np.linalg.slogdet(a)
        np.testing.assert_allclose(s1.numpy(), s2, atol=1e-10)
        np.testing.assert_allclose(l1.numpy(), l2, atol=1e-10)


def test_param_tree_size_n2():
    s = system.make_system("N2")
    p = system.init_params(np.random.default_rng(0), s)
    assert system.param_count(p) == 2381


@pytest.mark.parametrize("name", ["H2", "Be", "C", "N2"])
def test_two_restatements_agree(name):
    s = system.make_system(name)
    p = system.init_params(np.random.default_rng(1), s, randomize_aux=True)
    net = network.Network(s)
    pt = network.to_torch(p)
    pos = system.init_electrons(np.random.default_rng(2), s.atoms, s.charges, 3, 1.0)
    for x in pos:
        ph, la = net.apply(pt, torch.tensor(x))
        ph2, la2 = network_np.log_psi(s, p, x)
        np.testing.assert_allclose(float(la), la2, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(np.cos(float(ph)), np.cos(ph2), atol=1e-10)


@pytest.mark.parametrize("name", ["H2", "Be"])
def test_finite_difference_local_energy(name):
    s = system.make_system(name)
    p = system.init_params(np.random.default_rng(3), s, randomize_aux=True)
    net = network.Network(s)
    pt = network.to_torch(p)
    x = system.init_electrons(np.random.default_rng(4), s.atoms, s.charges, 1, 1.0)[0]
    e_ad, _, g_ad = hamiltonian.batch_local_energy(net, pt, torch.tensor(x[None]))
    h = 1e-4
    l0 = network_np.log_psi(s, p, x)[1]
    lap, gr = 0.0, []
    for i in range(x.size):
        xp, xm = x.copy(), x.copy()
        xp[i] += h
        xm[i] -= h
        lp, lm = network_np.log_psi(s, p, xp)[1], network_np.log_psi(s, p, xm)[1]
        lap += (lp - 2 * l0 + lm) / h ** 2
        gr.append((lp - lm) / (2 * h))
    e_fd = network_np.potential(s, x) - 0.5 * (lap + np.sum(np.square(gr)))
    np.testing.assert_allclose(g_ad.numpy()[0], gr, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(float(e_ad[0]), e_fd, rtol=1e-5, atol=1e-5)


def test_spin_tables_match_reference_order():
    # spin_indices.py:5-19 on alternating spins (every reference example)
    par, anti, npar, nanti = system.jastrow_indices_ee(system.alternating_spins(4), 4)
    np.testing.assert_array_equal(par, [[0, 1], [2, 3]])
    np.testing.assert_array_equal(anti, [[0, 0, 1, 2], [1, 3, 2, 3]])
    assert (npar, nanti) == (2, 4)
    up, dn = system.spin_indices_h(system.alternating_spins(6))
    np.testing.assert_array_equal(up, [0, 2, 4])
    np.testing.assert_array_equal(dn, [1, 3, 5])


def test_golden_fixtures_reproduce(golden_dir):
    """The committed fixtures are exactly what the oracle computes (H2, Be)."""
    import os
    for name in ["H2", "Be"]:
        g = dict(np.load(os.path.join(golden_dir, f"{name}.npz")))
        s = system.make_system(name)
        tmpl = system.init_params(np.random.default_rng(0), s)
        params = system.unflatten_params(tmpl, g["params_flat"])
        np.testing.assert_array_equal(system.flatten_params(params), g["params_flat"])
        net = network.Network(s)
        e, la, gr = hamiltonian.batch_local_energy(net, network.to_torch(params), torch.tensor(g["pos"]))
        np.testing.assert_allclose(e.numpy(), g["e_l"], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(la.numpy(), g["logabs"], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(gr.numpy(), g["grad"], rtol=1e-12, atol=1e-12)
