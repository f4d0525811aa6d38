"""Parameter gradient of log|psi| (aiqmc_logpsi_param_grad) vs the float64 oracle
(torch.func.grad of the oracle network wrt the parameter tree), and the energy gradient
it feeds (Loss/loss.py:220-270).  Tolerances: fp64 1e-8 relative to the largest
component of each walker's gradient; fp32 2e-3."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(name, dtype, B=4, seed=41):
    from oracle import system
    from aiqmc import _lib
    s = system.make_system(name)
    t = s.tables()
    ctx = _lib.Context(s.nelectrons, s.natoms, s.nspins, s.atoms, s.charges, t["spin_up_indices"],
                       t["spin_down_indices"], t["parallel_indices"], t["antiparallel_indices"], dtype=dtype, device=0)
    rng = np.random.default_rng(seed)
    params = system.init_params(rng, s, randomize_aux=True)
    ctx.set_params(system.flatten_params(params))
    pos = system.init_electrons(rng, s.atoms, s.charges, B, 1.0)
    return s, ctx, params, pos


@pytest.mark.parametrize("name", ["H2", "Be", "N2"])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_param_grad_matches_oracle(name, dtype):
    from oracle import loss, network
    s, ctx, params, pos = _setup(name, dtype)
    g, la = ctx.logpsi_param_grad(torch.tensor(pos, dtype=dtype, device="cuda"), want_logabs=True)
    torch.cuda.synchronize()
    ref = loss.logabs_param_grad(network.Network(s), params, torch.tensor(pos))
    got = g.double().cpu().numpy()
    assert got.shape == ref.shape == (pos.shape[0], ctx.nparams)
    tol = 1e-8 if dtype == torch.float64 else 2e-3
    scale = np.abs(ref).max(axis=1, keepdims=True) + 1e-3
    err = np.abs(got - ref) / scale
    assert err.max() < tol, (err.max(), np.unravel_index(err.argmax(), err.shape))
    la_ref, _ = ctx.logpsi(torch.tensor(pos, dtype=dtype, device="cuda"))
    np.testing.assert_allclose(la.double().cpu().numpy(), la_ref.double().cpu().numpy(), rtol=1e-6, atol=1e-6)


def test_weighted_sum_and_energy_gradient():
    """sum_b w_b O_b on the device == the per-walker rows contracted on the host; the energy
    gradient of loss.py:220-270 built from it == the oracle formula."""
    from oracle import loss
    s, ctx, params, pos = _setup("Be", torch.float64, B=64, seed=5)
    x = torch.tensor(pos, device="cuda")
    O = ctx.logpsi_param_grad(x)
    e_l, _, _ = ctx.local_energy(x)
    el = e_l.cpu().numpy()
    l0, var0, g_ref = loss.energy_gradient(el, O.cpu().numpy(), clip_scale=5.0)
    center, diff = loss.clip_local_values(el, l0, 5.0)
    w = torch.tensor(2.0 * diff / len(el), device="cuda")
    g = ctx.logpsi_param_grad(x, weights=w)
    torch.cuda.synchronize()
    np.testing.assert_allclose(g.cpu().numpy(), (w.cpu().numpy() @ O.cpu().numpy()), rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(g.cpu().numpy(), g_ref, rtol=1e-9, atol=1e-11)


def test_param_grad_full_batch_finite():
    s, ctx, params, pos = _setup("N2", torch.float32, B=4096, seed=9)
    x = torch.tensor(pos, dtype=torch.float32, device="cuda")
    g = ctx.logpsi_param_grad(x, weights=torch.full((4096,), 1.0 / 4096, device="cuda"))
    O = ctx.logpsi_param_grad(x[:64])
    torch.cuda.synchronize()
    assert torch.isfinite(g).all() and torch.isfinite(O).all()


@pytest.mark.parametrize("name", ["H2", "Be", "N2"])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_phase_param_grad_matches_oracle(name, dtype):
    """d phase / d theta (aiqmc_phase_param_grad) vs torch.func.grad of the oracle's phase
    (itself pinned by finite differences in tests/test_oracle_loss.py)."""
    from oracle import loss, network
    s, ctx, params, pos = _setup(name, dtype, seed=43)
    g, ph = ctx.phase_param_grad(torch.tensor(pos, dtype=dtype, device="cuda"), want_phase=True)
    torch.cuda.synchronize()
    ref = loss.phase_param_grad(network.Network(s), params, torch.tensor(pos))
    got = g.double().cpu().numpy()
    tol = 1e-8 if dtype == torch.float64 else 2e-3
    scale = np.abs(ref).max(axis=1, keepdims=True) + 1e-3
    err = np.abs(got - ref) / scale
    assert err.max() < tol, (err.max(), np.unravel_index(err.argmax(), err.shape))
    _, ph_ref = ctx.logpsi(torch.tensor(pos, dtype=dtype, device="cuda"))
    ptol = 1e-9 if dtype == torch.float64 else 1e-3   # two different fp32 kernels (pgrad vs walker)
    np.testing.assert_allclose(ph.double().cpu().numpy(), ph_ref.double().cpu().numpy(), rtol=ptol, atol=ptol)
    # the Jastrow parameters carry no phase
    assert np.abs(got[:, np.abs(ref).max(axis=0) == 0]).max(initial=0.0) < 1e-12


def test_complex_energy_gradient_pp_loss():
    """make_loss(complex_output=True) on complex pp local energies (C-atom ccECP, the
    main_pp_adam_muti_GPU.py:150-156 configuration): the gradient equals the literal
    custom-JVP tangent of the oracle built from the per-walker d log|psi| and d phase rows."""
    from oracle import loss as oloss, pphamiltonian as opp, system
    from aiqmc import spin_indices
    from aiqmc.Energy import pphamiltonian
    from aiqmc.Loss import loss as L
    from aiqmc.VMC.VMCmcstep import PhiloxKey
    from aiqmc.wavefunction_Ynlm import nn
    s = system.make_system("C_ecp")
    par, anti, npar, nanti = spin_indices.jastrow_indices_ee(spins=s.spins, nelectrons=4)
    up, dn = spin_indices.spin_indices_h(s.spins)
    network = nn.make_ai_net(ndim=3, nelectrons=4, natoms=1, nspins=(2, 2), charges=s.charges,
                             parallel_indices=par, antiparallel_indices=anti, n_parallel=npar,
                             n_antiparallel=nanti, spin_up_indices=up, spin_down_indices=dn)
    params = system.init_params(np.random.default_rng(12), s, randomize_aux=True)
    e = opp.c_atom_ccecp()
    le = pphamiltonian.local_energy(f=network.apply, lognetwork=nn.make_log_network(network.apply),
                                    charges=s.charges, nspins=s.spins, rn_local=e.rn_local,
                                    local_coes=e.local_coes, local_exps=e.local_exps,
                                    rn_non_local=e.rn_non_local, non_local_coes=e.non_local_coes,
                                    non_local_exps=e.non_local_exps, natoms=1, nelectrons=4, ndim=3, list_l=2)
    B = 256
    pos = torch.tensor(system.init_electrons(np.random.default_rng(13), s.atoms, s.charges, B, 1.0), device="cuda")
    data = nn.AINetData(positions=pos, spins=s.spins, atoms=s.atoms, charges=s.charges)
    key = PhiloxKey(4, 0)
    e_l, _ = le(params, key, data)
    assert bool((e_l.imag != 0).any())
    ctx = network.apply._aiqmc_network.bind(params, s.atoms, torch.float64)
    Oa = ctx.logpsi_param_grad(pos).cpu().numpy()
    Op = ctx.phase_param_grad(pos).cpu().numpy()
    for clip in (5.0, 0.0):
        ev = L.make_loss(network=nn.make_log_network(network.apply), local_energy=le, clip_local_energy=clip,
                         clip_from_median=False, center_at_clipped_energy=True, complex_output=True)
        (lv, aux), g = ev.value_and_grad(params, key, data)
        torch.cuda.synchronize()
        l_ref, g_ref = oloss.energy_gradient_complex(e_l.cpu().numpy(), Oa, Op, clip_scale=clip)
        assert abs(lv.real.item() - l_ref) < 1e-10
        np.testing.assert_allclose(g.cpu().numpy(), g_ref, rtol=1e-9, atol=1e-11 * np.abs(g_ref).max())


def test_pp_adam_training_step():
    """One Adam step driven like main_pp_adam_muti_GPU.py:150-190 (complex pp E_L, clip 5.0,
    complex_output=True): parameters == the oracle Adam update of the literal custom-JVP
    gradient built from the same E_L and per-walker gradient rows."""
    from oracle import loss as oloss, pphamiltonian as opp, system
    from aiqmc import spin_indices
    from aiqmc.Energy import pphamiltonian
    from aiqmc.Loss import loss as L
    from aiqmc.Optimizer import adam, optax_like as optax
    from aiqmc.VMC.VMCmcstep import PhiloxKey
    from aiqmc.wavefunction_Ynlm import nn
    s = system.make_system("C_ecp")
    par, anti, npar, nanti = spin_indices.jastrow_indices_ee(spins=s.spins, nelectrons=4)
    up, dn = spin_indices.spin_indices_h(s.spins)
    network = nn.make_ai_net(ndim=3, nelectrons=4, natoms=1, nspins=(2, 2), charges=s.charges,
                             parallel_indices=par, antiparallel_indices=anti, n_parallel=npar,
                             n_antiparallel=nanti, spin_up_indices=up, spin_down_indices=dn)
    params = system.init_params(np.random.default_rng(14), s, randomize_aux=True)
    e = opp.c_atom_ccecp()
    log_network = nn.make_log_network(network.apply)
    le = pphamiltonian.local_energy(f=network.apply, lognetwork=log_network, charges=s.charges, nspins=s.spins,
                                    rn_local=e.rn_local, local_coes=e.local_coes, local_exps=e.local_exps,
                                    rn_non_local=e.rn_non_local, non_local_coes=e.non_local_coes,
                                    non_local_exps=e.non_local_exps, natoms=1, nelectrons=4, ndim=3, list_l=2)
    ev = L.make_loss(network=log_network, local_energy=le, clip_local_energy=5.0, clip_from_median=False,
                     center_at_clipped_energy=True, complex_output=True)
    opt = optax.chain(optax.scale_by_adam(b1=0.9, b2=0.999, eps=1e-8, eps_root=0.0),
                      optax.scale_by_schedule(lambda t: 0.05 * (1.0 / (1.0 + t)) ** 10000), optax.scale(-1.))
    step = adam.make_training_step(adam.make_opt_update_step(ev, opt))
    B = 128
    pos = torch.tensor(system.init_electrons(np.random.default_rng(15), s.atoms, s.charges, B, 1.0), device="cuda")
    data = nn.AINetData(positions=pos, spins=s.spins, atoms=s.atoms, charges=s.charges)
    key = PhiloxKey(6, 0)
    _, new_params, state, loss_v, aux = step(data, params, None, key)
    torch.cuda.synchronize()
    e_l, _ = le(params, key, data)
    ctx = network.apply._aiqmc_network.bind(params, s.atoms, torch.float64)
    Oa, Op = ctx.logpsi_param_grad(pos).cpu().numpy(), ctx.phase_param_grad(pos).cpu().numpy()
    l_ref, g_ref = oloss.energy_gradient_complex(e_l.cpu().numpy(), Oa, Op, clip_scale=5.0)
    flat = system.flatten_params(params)
    p_ref = oloss.Adam(flat.size).update(g_ref, flat)
    assert abs(float(loss_v.real) - l_ref) < 1e-9
    np.testing.assert_allclose(system.flatten_params(new_params), p_ref, rtol=1e-9, atol=1e-9)
