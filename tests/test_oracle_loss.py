"""Energy-gradient / Adam oracle (oracle/loss.py) pinned by finite differences and closed forms."""
import math

import numpy as np
import torch


def test_param_grad_finite_differences():
    from oracle import loss, network, system
    s = system.make_system("H2")
    rng = np.random.default_rng(3)
    params = system.init_params(rng, s, randomize_aux=True)
    pos = torch.tensor(system.init_electrons(rng, s.atoms, s.charges, 2, 1.0))
    net = network.Network(s)
    O = loss.logabs_param_grad(net, params, pos)
    flat = system.flatten_params(params)
    for k in rng.choice(flat.size, 25, replace=False):
        h = 1e-6
        fp, fm = flat.copy(), flat.copy()
        fp[k] += h
        fm[k] -= h
        lp = net.logabs(network.to_torch(system.unflatten_params(params, fp)), pos[0]).item()
        lm = net.logabs(network.to_torch(system.unflatten_params(params, fm)), pos[0]).item()
        assert abs((lp - lm) / (2 * h) - O[0, k]) < 1e-6 * (1 + abs(O[0, k])), k


def test_energy_gradient_closed_form():
    from oracle import loss
    rng = np.random.default_rng(0)
    e = rng.standard_normal(50)
    e[3] = 40.0                                          # an outlier the 5-TV window clips
    O = rng.standard_normal((50, 7))
    l, var, g = loss.energy_gradient(e, O, clip_scale=5.0)
    tv = np.mean(np.abs(e - e.mean()))
    c = np.clip(e, e.mean() - 5 * tv, e.mean() + 5 * tv)
    assert c[3] < 40.0
    np.testing.assert_allclose(g, 2.0 / 50 * ((c - c.mean()) @ O), rtol=1e-12)
    assert abs(l - e.mean()) < 1e-14 and abs(var - e.var()) < 1e-12


def test_adam_restatement():
    from oracle import loss
    opt = loss.Adam(3)
    p = np.array([1.0, -2.0, 0.5])
    g = np.array([0.3, -0.1, 0.0])
    p1 = opt.update(g, p)
    # first step: m_hat = g, v_hat = g^2 -> u = g / (|g| + eps) * 0.05
    np.testing.assert_allclose(p1, p - 0.05 * g / (np.abs(g) + 1e-8), rtol=1e-12)
    p2 = opt.update(g, p1)
    assert loss.lr_schedule(1) == 0.05 * 2.0 ** -10000   # the reference schedule collapses after step 0
    np.testing.assert_allclose(p2, p1, atol=1e-300)


def test_complex_energy_gradient_reduces_to_weights():
    """The literal custom-JVP tangent (term1 - 2 term2).real / B for complex E_L equals
    (2/B) sum_b [Re(diff_b) O_abs_b + Im(cl_b) O_phase_b], cl = diff + aux.clipped_energy
    (the clip centre when clipping, E_L itself when not) -- the form the GPU path uses."""
    from oracle import loss
    rng = np.random.default_rng(3)
    B, P = 40, 7
    e = rng.normal(-5, 1, B) + 1j * rng.normal(0, 0.3, B)
    e[3] += 9.0 + 4.0j                       # outlier: exercises both clip windows
    Oa, Op = rng.standard_normal((B, P)), rng.standard_normal((B, P))
    for clip in (5.0, 0.0):
        _, g = loss.energy_gradient_complex(e, Oa, Op, clip_scale=clip)
        if clip > 0:
            m = e.mean()
            tr, ti = np.mean(np.abs(e.real - m.real)), np.mean(np.abs(e.imag - m.imag))
            c = np.clip(e.real, m.real - clip * tr, m.real + clip * tr) + 1j * np.clip(
                e.imag, m.imag - clip * ti, m.imag + clip * ti)
            center = c.mean()
            diff, cl = c - center, c
        else:
            diff = e - e.mean()
            cl = diff + e
        want = (2.0 / B) * (diff.real @ Oa + cl.imag @ Op)
        np.testing.assert_allclose(g, want, rtol=1e-12, atol=1e-12)


def test_clip_from_median_complex_matches_oracle():
    """loss.clip_local_values with clip_from_median=True on complex E_L (the pp drivers' path):
    the centre is the real median (jnp.median: even count -> mean of the middle pair) and the
    imaginary window is centred at 0 (JAX's .imag of a real array)."""
    from aiqmc.Loss.loss import clip_local_values
    rng = np.random.default_rng(5)
    e = rng.standard_normal(40) + 1j * rng.standard_normal(40)
    e[7] = 30.0 + 25.0j
    mean = e.mean()
    center, diff = clip_local_values(torch.tensor(e), torch.tensor(mean), 5.0, True, True)
    med = np.median(e.real)
    tv_re = np.mean(np.abs(e.real - med))
    tv_im = np.mean(np.abs(e.imag - 0.0))
    clipped = np.clip(e.real, med - 5 * tv_re, med + 5 * tv_re) + 1j * np.clip(e.imag, -5 * tv_im, 5 * tv_im)
    np.testing.assert_allclose(center.numpy(), clipped.mean(), rtol=1e-12)
    np.testing.assert_allclose(diff.numpy(), clipped - clipped.mean(), rtol=1e-12, atol=1e-12)
