"""The complex_output=True local energy (Energy/hamiltonian.py:100-131 with its phase branch
:110-130) in the CPU oracle: KE = -1/2 [lap log|psi| + i lap theta] - 1/2 |grad log|psi||^2
+ 1/2 |grad theta|^2 - i grad log|psi| . grad theta, theta = arg psi.  Pinned here against central
finite differences of the independent numpy restatement (oracle/network_np.py), and its real part
against the real local energy (CPU)."""
import math

import numpy as np
import pytest
import torch

from oracle import hamiltonian, network, network_np, system

torch.set_default_dtype(torch.float64)


@pytest.mark.parametrize("name", ["H2", "Be"])
def test_complex_local_energy_vs_finite_differences(name):
    s = system.make_system(name)
    p = system.init_params(np.random.default_rng(13), s, randomize_aux=True)
    net = network.Network(s)
    pt = network.to_torch(p)
    x = system.init_electrons(np.random.default_rng(14), s.atoms, s.charges, 1, 1.0)[0]
    ec = hamiltonian.batch_local_energy_complex(net, pt, torch.tensor(x[None]))[0]
    h = 1e-4
    th0, l0 = network_np.log_psi(s, p, x)
    wrap = lambda d: (d + math.pi) % (2 * math.pi) - math.pi      # phase differences mod 2 pi
    lap_l = lap_t = 0.0
    gl, gt = [], []
    for i in range(x.size):
        xp, xm = x.copy(), x.copy()
        xp[i] += h
        xm[i] -= h
        tp, lp = network_np.log_psi(s, p, xp)
        tm, lm = network_np.log_psi(s, p, xm)
        lap_l += (lp - 2 * l0 + lm) / h ** 2
        lap_t += (wrap(tp - th0) + wrap(tm - th0)) / h ** 2
        gl.append((lp - lm) / (2 * h))
        gt.append(wrap(tp - tm) / (2 * h))
    gl, gt = np.array(gl), np.array(gt)
    re = network_np.potential(s, x) - 0.5 * (lap_l + gl @ gl) + 0.5 * (gt @ gt)
    im = -0.5 * lap_t - gl @ gt
    assert abs(gt).max() > 1e-3          # a genuinely complex wavefunction (random complex orbitals)
    np.testing.assert_allclose(float(ec.real), re, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(float(ec.imag), im, rtol=1e-5, atol=1e-5)


def test_complex_local_energy_real_part():
    s = system.make_system("Be")
    p = system.init_params(np.random.default_rng(15), s, randomize_aux=True)
    net = network.Network(s)
    pt = network.to_torch(p)
    pos = torch.tensor(system.init_electrons(np.random.default_rng(16), s.atoms, s.charges, 3, 1.0))
    ec = hamiltonian.batch_local_energy_complex(net, pt, pos)
    e, _, _ = hamiltonian.batch_local_energy(net, pt, pos)
    gt = torch.stack([torch.func.grad(lambda x: net.apply(pt, x)[0])(pos[b]) for b in range(3)])
    np.testing.assert_allclose(ec.real.numpy(), (e + 0.5 * (gt ** 2).sum(1)).numpy(), rtol=1e-10, atol=1e-10)
