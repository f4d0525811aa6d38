"""The reference-shaped Python API (make_ai_net / local_energy / main_monte_carlo)
driven exactly like main_all_electrons_adam_muti_GPU.py:104-197, vs the oracle."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(name="Be", B=16, dtype=torch.float64):
    from oracle import system
    from aiqmc import spin_indices
    from aiqmc.wavefunction_Ynlm import nn
    from aiqmc.initial_electrons_positions.init import init_electrons
    s = system.make_system(name)
    par, anti, npar, nanti = spin_indices.jastrow_indices_ee(spins=s.spins, nelectrons=s.nelectrons)
    up, dn = spin_indices.spin_indices_h(s.spins)
    network = nn.make_ai_net(ndim=3, nelectrons=s.nelectrons, natoms=s.natoms, nspins=s.nspins, determinants=1,
                             charges=s.charges, parallel_indices=par, antiparallel_indices=anti,
                             n_parallel=npar, n_antiparallel=nanti, spin_up_indices=up, spin_down_indices=dn)
    params = system.init_params(np.random.default_rng(3), s, randomize_aux=True)
    pos, spins = init_electrons(7, None, s.atoms, s.charges, s.spins, B, 1.0)
    atoms = np.tile(s.atoms[None], (B, 1, 1))          # batch-tiled, as the driver does
    charges = np.tile(s.charges[None], (B, 1))
    data = nn.AINetData(positions=pos.to("cuda", dtype).contiguous(), spins=spins, atoms=atoms,
                        charges=charges)
    return s, network, params, data


def test_apply_and_local_energy_match_oracle():
    from oracle import hamiltonian, network as onet
    from aiqmc.Energy import hamiltonian as H
    s, network, params, data = _setup()
    phase, logabs = network.apply(params, data.positions, data.spins, data.atoms, data.charges)
    el_fn = H.local_energy(f=network.apply, charges=s.charges, nspins=s.spins)
    e_l, mat = el_fn(params, None, data)
    assert mat is None
    net = onet.Network(s)
    e_ref, l_ref, _ = hamiltonian.batch_local_energy(net, onet.to_torch(params), data.positions.cpu())
    np.testing.assert_allclose(logabs.cpu().numpy(), l_ref.numpy(), rtol=1e-10, atol=1e-10)
    assert np.max(np.abs(e_l.cpu().numpy() - e_ref.numpy())) < 1e-6
    ke = H.local_kinetic_energy(network.apply, complex_output=False)(params, data)
    assert torch.isfinite(ke).all()


def test_main_monte_carlo_host_draws_match_oracle():
    from oracle import mcstep, network as onet
    from aiqmc.VMC import VMCmcstep
    s, network, params, data = _setup(B=8)
    N, B, nsteps = s.nelectrons, 8, 2
    rng = np.random.default_rng(9)
    g1 = torch.tensor(rng.standard_normal((nsteps, B, 3 * N)))
    g2 = torch.tensor(rng.standard_normal((nsteps, B, N, 3 * N)))
    u = torch.tensor(rng.uniform(size=(nsteps, B, N)))
    x0 = data.positions.cpu().clone()
    mc_step = VMCmcstep.main_monte_carlo(f=network.apply, tstep=0.05, ndim=3, nelectrons=N, nsteps=nsteps,
                                         batch_size=B)
    out = mc_step(params, data, VMCmcstep.HostDraws(g1, g2, u))
    ref = mcstep.mc_step(onet.Network(s), onet.to_torch(params), x0, g1, g2, u, 0.05, nsteps)
    np.testing.assert_allclose(out.positions.cpu().numpy(), ref.numpy(), rtol=1e-9, atol=1e-9)
    assert out.positions.data_ptr() == data.positions.data_ptr()     # in place (donate_argnums analogue)


def test_param_update_is_picked_up():
    s, network, params, data = _setup(B=4)
    _, l1 = network.apply(params, data.positions, None, data.atoms, None)
    params["orbitals"][0]["b"] = params["orbitals"][0]["b"] + 0.5
    _, l2 = network.apply(params, data.positions, None, data.atoms, None)
    assert not torch.allclose(l1, l2)


def test_pphamiltonian_drop_in_matches_golden(golden_dir):
    """pphamiltonian.local_energy driven like main_pp_adam_muti_GPU.py:119-148 (C atom ccECP)."""
    import os
    from oracle import pphamiltonian as opp, system
    from aiqmc import spin_indices
    from aiqmc.Energy import pphamiltonian
    from aiqmc.wavefunction_Ynlm import nn
    g = dict(np.load(os.path.join(golden_dir, "C_ecp.npz")))
    s = system.make_system("C_ecp")
    par, anti, npar, nanti = spin_indices.jastrow_indices_ee(spins=s.spins, nelectrons=s.nelectrons)
    up, dn = spin_indices.spin_indices_h(s.spins)
    network = nn.make_ai_net(ndim=3, nelectrons=4, natoms=1, nspins=(2, 2), determinants=1, charges=s.charges,
                             parallel_indices=par, antiparallel_indices=anti, n_parallel=npar,
                             n_antiparallel=nanti, spin_up_indices=up, spin_down_indices=dn)
    params = system.unflatten_params(system.init_params(np.random.default_rng(0), s), g["params_flat"])
    e = opp.c_atom_ccecp()

    def log_network(*args, **kwargs):
        phase, mag = network.apply(*args, **kwargs)
        return mag + 1.j * phase

    el = pphamiltonian.local_energy(f=network.apply, lognetwork=log_network, charges=s.charges, nspins=s.spins,
                                    rn_local=e.rn_local, local_coes=e.local_coes, local_exps=e.local_exps,
                                    rn_non_local=e.rn_non_local, non_local_coes=e.non_local_coes,
                                    non_local_exps=e.non_local_exps, natoms=1, nelectrons=4, ndim=3, list_l=2)
    data = nn.AINetData(positions=torch.tensor(g["pos"], device="cuda"), spins=s.spins, atoms=s.atoms,
                        charges=s.charges)
    out, mat = el(params, pphamiltonian.HostRotations(torch.tensor(g["rot"])), data)
    assert mat is None and out.is_complex()
    assert np.max(np.abs(out.real.cpu().numpy() - g["e_re"])) < 1e-6
    assert np.max(np.abs(out.imag.cpu().numpy() - g["e_im"])) < 1e-6
    out2, _ = el(params, 11, data)                      # Philox rotations
    assert torch.isfinite(out2.real).all()


def test_adam_training_step_matches_oracle():
    """make_loss + Adam chain + make_training_step driven like
    main_all_electrons_adam_muti_GPU.py:143-190 (clip 5.0, complex_output=True, Adam 0.9/0.999,
    lr 0.05 (1+t)^-10000), one step, vs the oracle energy gradient and Adam restatement."""
    from oracle import hamiltonian, loss as oloss, network as onet, system
    from aiqmc.Energy import hamiltonian as H
    from aiqmc.Loss import loss as L
    from aiqmc.Optimizer import adam, optax_like as optax
    s, network, params, data = _setup(B=16)

    def log_network(*args, **kwargs):
        phase, mag = network.apply(*args, **kwargs)
        return mag + 1.j * phase

    local_energy = H.local_energy(f=network.apply, charges=s.charges, nspins=s.spins, use_scan=False)
    evaluate_loss = L.make_loss(network=log_network, local_energy=local_energy, clip_local_energy=5.0,
                                clip_from_median=False, center_at_clipped_energy=True, complex_output=True)
    sched = lambda t: 0.05 * (1.0 / (1.0 + t)) ** 10000
    optimizer = optax.chain(optax.scale_by_adam(b1=0.9, b2=0.999, eps=1e-8, eps_root=0.0),
                            optax.scale_by_schedule(sched), optax.scale(-1.))
    step = adam.make_training_step(adam.make_opt_update_step(evaluate_loss, optimizer))
    _, new_params, state, loss_v, aux = step(data, params, None, 0)
    # oracle
    net = onet.Network(s)
    x = data.positions.cpu()
    e_ref, _, _ = hamiltonian.batch_local_energy(net, onet.to_torch(params), x)
    O = oloss.logabs_param_grad(net, params, x)
    l_ref, var_ref, g_ref = oloss.energy_gradient(e_ref.numpy(), O, clip_scale=5.0)
    flat = system.flatten_params(params)
    p_ref = oloss.Adam(flat.size).update(g_ref, flat)
    assert abs(float(loss_v) - l_ref) < 1e-6
    assert abs(float(aux.variance) - var_ref) < 1e-5 * (1 + var_ref)
    np.testing.assert_allclose(system.flatten_params(new_params), p_ref, rtol=1e-9, atol=1e-9)
    # the reference schedule collapses after step 0: the second step leaves the parameters unchanged
    _, p2, state, _, _ = step(data, new_params, state, 1)
    np.testing.assert_allclose(system.flatten_params(p2), system.flatten_params(new_params), rtol=0, atol=1e-300)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["N2", "Be", "C2_ecp"])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_network_orbitals_match_oracle(name, dtype):
    """Network.orbitals (nn.py:409-506,553): the complex [N, N] matrix, rows up then down
    electrons, row r with electron r's envelope / y row (Q1), times exp(J_ee/N) exp(J_ae/N);
    its slogdet is apply()'s output."""
    from oracle import network, system
    from aiqmc import systems
    s = systems.make_system(name)
    net = s.make_network()
    os_ = system.make_system(name)
    rng = np.random.default_rng(3)
    params = system.init_params(rng, os_, randomize_aux=True)
    pos = system.init_electrons(rng, os_.atoms, os_.charges, 6, 1.0)
    x = torch.tensor(pos, dtype=dtype, device="cuda")
    (m,) = net.orbitals(params, x, s.spins, s.atoms, s.charges)
    phase, logabs = net.apply(params, x, s.spins, s.atoms, s.charges)
    torch.cuda.synchronize()
    assert m.shape == (6, s.nelectrons, s.nelectrons) and m.is_complex()
    onet = network.Network(os_)
    pt = network.to_torch(params)
    ref = torch.stack([onet.orbitals(pt, torch.tensor(pos[b])) for b in range(6)]).numpy()
    got = m.to(torch.complex128).cpu().numpy()
    tol = 1e-10 if dtype == torch.float64 else 2e-4
    scale = np.abs(ref).max(axis=(1, 2), keepdims=True)
    assert np.all(np.abs(got - ref) <= tol * scale), float(np.max(np.abs(got - ref) / scale))
    sign, ld = np.linalg.slogdet(got)
    np.testing.assert_allclose(ld, logabs.double().cpu().numpy(), rtol=tol, atol=tol * 10)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("n", [1, 7, 1000, 4096, 33000])
def test_pmean_stats_device_kernel_matches_two_pass(dtype, n):
    """constants.pmean_stats on a device tensor runs aiqmc_energy_stats; compare with the
    reference's two pmeans (loss.py:206-208) on one rank in float64: E = mean(e),
    var = mean(|e - E|^2), including heavy-tailed energies like the bench's random network."""
    from aiqmc import constants, _lib
    g = torch.Generator().manual_seed(n)
    e = torch.randn(n, generator=g, dtype=torch.float64) * 30.0 - 100.0
    e[:: 97] *= 1e3
    ed = e.to("cuda", dtype)
    mean, var = constants.pmean_stats(ed)
    e64 = ed.cpu().to(torch.float64)
    m_ref = e64.mean()
    v_ref = ((e64 - m_ref) ** 2).mean()
    assert mean.dtype == torch.float64 and mean.is_cuda
    np.testing.assert_allclose(float(mean), float(m_ref), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(float(var), float(v_ref), rtol=1e-12, atol=0)
    v = _lib.energy_stats(ed, finalize=False)
    _lib.energy_stats_final(v)
    # the multi-rank finalisation (Chan's combination of the summed 4-vector) on one rank
    np.testing.assert_allclose(v[4:].cpu().numpy(), torch.stack([mean, var]).cpu().numpy(), rtol=1e-12, atol=0)
    assert float(v[3]) == n


def test_energy_stats_rejects_empty_and_host():
    from aiqmc import _lib
    with pytest.raises(RuntimeError, match="empty"):
        _lib.energy_stats(torch.empty(0, device="cuda"))
    with pytest.raises(ValueError):
        _lib.energy_stats(torch.ones(4))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["N2", "Be", "C2_ecp", "H2"])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_set_params_device_equals_host_upload(name, dtype):
    """aiqmc_set_params_device (canonical parameters repacked on the device, stream-ordered) gives
    the same kernel layout as the host upload: log|psi|, its gradient, E_L and the parameter
    gradient (which also reads the W_y row norms) bitwise equal on the same walkers."""
    from aiqmc import systems
    from aiqmc.initial_electrons_positions.init import init_electrons
    from aiqmc.wavefunction_Ynlm.nn import flatten_params
    s = systems.make_system(name)
    flat = flatten_params(s.make_network().init(7))
    pos = init_electrons(3, None, s.atoms, s.charges, s.spins, 64, 1.0)[0].to("cuda", dtype).contiguous()
    outs = []
    for mode in ("host", "device"):
        ctx = s.context(dtype=dtype)
        if mode == "host":
            ctx.set_params(flat)
        else:
            ctx.set_params_device(torch.tensor(flat, dtype=torch.float64, device="cuda"))
        la, g = ctx.logpsi_grad(pos)
        e, _, _ = ctx.local_energy(pos)
        pg = ctx.logpsi_param_grad(pos)
        torch.cuda.synchronize()
        outs.append([t.cpu() for t in (la, g, e, pg)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_adam_steps_stay_on_the_device():
    """The drop-in Adam step returns device-tensor leaves (views of one float64 vector) and the
    next bind repacks them on the device: two steps through that path equal two steps with the
    parameters round-tripped through the host (numpy leaves) -- the same optimiser arithmetic."""
    from aiqmc.Energy import hamiltonian as H
    from aiqmc.Loss import loss as L
    from aiqmc.Optimizer import adam, optax_like as optax
    from aiqmc.VMC import VMCmcstep
    from aiqmc.wavefunction_Ynlm.nn import flatten_params
    s, network, params, data = _setup(B=64)
    local_energy = H.local_energy(f=network.apply, charges=s.charges, nspins=s.spins, use_scan=False)
    runs = []
    for host_roundtrip in (False, True):
        ev = L.make_loss(network=network.apply, local_energy=local_energy, clip_local_energy=5.0,
                         clip_from_median=False, center_at_clipped_energy=True, complex_output=True)
        opt = optax.chain(optax.scale_by_adam(b1=0.9, b2=0.999, eps=1e-8, eps_root=0.0),
                          optax.scale_by_schedule(lambda t: 0.05 / (1.0 + 0.01 * t)), optax.scale(-1.))
        step = adam.make_training_step(adam.make_opt_update_step(ev, opt))
        p, st, d = params, None, data
        for t in range(2):
            d, p, st, loss_v, aux = step(d, p, st, t)
            if host_roundtrip:
                p = L._unflatten_like(p, flatten_params(p))     # numpy leaves: the host upload path
            else:
                leaves = [l for l in _leaves(p)]
                assert all(isinstance(l, torch.Tensor) and l.is_cuda for l in leaves)
        runs.append(flatten_params(p))
    np.testing.assert_array_equal(runs[0], runs[1])


def _leaves(tree):
    if isinstance(tree, dict):
        return [x for k in sorted(tree) for x in _leaves(tree[k])]
    if isinstance(tree, (list, tuple)):
        return [x for v in tree for x in _leaves(v)]
    return [tree]


@pytest.mark.gpu
@pytest.mark.parametrize("complex_e", [False, True])
@pytest.mark.parametrize("clip,center", [(5.0, True), (5.0, False), (0.0, True)])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_fused_loss_weights_match_torch_path(complex_e, clip, center, dtype):
    """aiqmc_loss_weights (one launch: statistics, total-variation clipping, the two weight
    vectors; Loss/loss.py:73-135, 206-208, 256-265) against the same formulas in torch float64
    on heavy-tailed energies (outliers so the clipping window bites)."""
    from aiqmc import _lib
    g = torch.Generator().manual_seed(11)
    B = 3001
    re = torch.randn(B, generator=g, dtype=torch.float64) * 2 - 10
    re[::97] *= 40.0
    im = torch.randn(B, generator=g, dtype=torch.float64) * 0.3
    im[::53] *= 30.0
    e64 = torch.complex(re, im) if complex_e else re
    cdt = {torch.float32: torch.complex64, torch.float64: torch.complex128}[dtype]
    e = (e64.to(cdt) if complex_e else e64.to(dtype)).cuda()
    wscale = 2.0 / B
    w, wp, clipped, st = _lib.loss_weights(e, clip, center, wscale, complex_e)
    # reference (torch path of make_loss, in float64 on the float-rounded energies)
    x = e.cpu().to(torch.complex128 if complex_e else torch.float64)
    m = x.mean()
    var = ((x - m) * (x - m).conj()).mean().real
    if clip > 0:
        def cl(v, c):
            tv = (v - c).abs().mean()
            return torch.clamp(v, c - clip * tv, c + clip * tv)
        if complex_e:
            cx = torch.complex(cl(x.real, m.real), cl(x.imag, m.imag))
        else:
            cx = cl(x, m)
        dc = cx.mean() if center else m
        diff = cx - dc
        aux = dc
    else:
        dc, diff, aux = m, x - m, x
    tol = dict(rtol=1e-11, atol=1e-11) if dtype == torch.float64 else dict(rtol=2e-6, atol=2e-6)
    np.testing.assert_allclose(w.cpu().double().numpy(), (wscale * diff.real).numpy(), **tol)
    if complex_e:
        np.testing.assert_allclose(wp.cpu().double().numpy(), (wscale * (diff + aux).imag).numpy(), **tol)
        np.testing.assert_allclose(clipped.cpu().to(torch.complex128).numpy(), (dc + diff).numpy(), rtol=1e-6)
    np.testing.assert_allclose(st[0].item(), float(m.real), rtol=1e-12)
    np.testing.assert_allclose(st[2].item(), float(var), rtol=1e-12)
    np.testing.assert_allclose(st[3].item(), float(dc.real), rtol=1e-12)
