"""complex_output=True local energy (Energy/hamiltonian.py:100-131 with the phase branch :110-130)
on the GPU against the CPU oracle (oracle/hamiltonian.batch_local_energy_complex, itself pinned by
finite differences in test_oracle_complex_el.py): aiqmc_local_energy_complex = the log|psi| launch
pair + the theta = arg psi launch pair (PH instantiations of the adjoint and first-derivative
passes) + one combining launch."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ctx_and_oracle(name, dtype, B, seed):
    from oracle import network, system
    from aiqmc import _lib
    s = system.make_system(name)
    t = s.tables()
    rng = np.random.default_rng(seed)
    params = system.init_params(rng, s, randomize_aux=True)
    pos = system.init_electrons(rng, s.atoms, s.charges, B, 1.0)
    ctx = _lib.Context(s.nelectrons, s.natoms, s.nspins, s.atoms, s.charges, t["spin_up_indices"],
                       t["spin_down_indices"], t["parallel_indices"], t["antiparallel_indices"], dtype=dtype,
                       device=0)
    ctx.set_params(system.flatten_params(params))
    return s, ctx, network.Network(s), params, pos


@pytest.mark.parametrize("name", ["H2", "Be", "C", "Ne", "N2"])
def test_complex_local_energy_matches_oracle_fp64(name):
    from oracle import hamiltonian, network
    s, ctx, net, params, pos = _ctx_and_oracle(name, torch.float64, 16, 31)
    x = torch.tensor(pos, device="cuda")
    ec = ctx.local_energy_complex(x)
    e_re, _, _ = ctx.local_energy(x)
    torch.cuda.synchronize()
    ref = hamiltonian.batch_local_energy_complex(net, network.to_torch(params), torch.tensor(pos))
    got = ec.cpu().numpy()
    print(name, "max |d re|", np.abs(got.real - ref.real.numpy()).max(), "max |d im|",
          np.abs(got.imag - ref.imag.numpy()).max(), "max |im|", np.abs(ref.imag.numpy()).max())
    assert np.abs(ref.imag.numpy()).max() > 1e-3          # a genuinely complex wavefunction
    np.testing.assert_allclose(got.real, ref.real.numpy(), rtol=1e-8, atol=1e-6)
    np.testing.assert_allclose(got.imag, ref.imag.numpy(), rtol=1e-8, atol=1e-6)
    # Re = E_L + |grad theta|^2 / 2 >= E_L
    assert np.all(got.real >= e_re.cpu().numpy() - 1e-9)


def test_complex_local_energy_fp32_vs_oracle():
    """fp32 N2 (the reference's dtype): errors against the float64 oracle at fp32 level (the
    determinant terms cancel as in the real E_L; bounds as test_precision_fp32's quantiles)."""
    from oracle import hamiltonian, network
    s, ctx, net, params, pos = _ctx_and_oracle("N2", torch.float32, 64, 33)
    pos32 = pos.astype(np.float32)
    ec = ctx.local_energy_complex(torch.tensor(pos32, device="cuda"))
    torch.cuda.synchronize()
    ref = hamiltonian.batch_local_energy_complex(net, network.to_torch(params), torch.tensor(pos32.astype(np.float64)))
    got = ec.cpu().numpy().astype(np.complex128)
    r = ref.numpy()
    scale = np.maximum(1.0, np.abs(r))
    err = np.abs(got - r) / scale
    print("fp32 complex E_L: rel err median", np.median(err), "p90", np.quantile(err, 0.9), "max", err.max())
    assert np.median(err) < 1e-4
    assert np.quantile(err, 0.9) < 2e-3


def test_drop_in_complex_output():
    """hamiltonian.local_energy / local_kinetic_energy with complex_output=True through the drop-in
    API (make_ai_net apply), as the reference's drivers would call it."""
    from oracle import hamiltonian as oh, network as onet, system
    from aiqmc import spin_indices
    from aiqmc.Energy import hamiltonian as H
    from aiqmc.wavefunction_Ynlm import nn
    s = system.make_system("Be")
    par, anti, npar, nanti = spin_indices.jastrow_indices_ee(spins=s.spins, nelectrons=s.nelectrons)
    up, dn = spin_indices.spin_indices_h(s.spins)
    network = nn.make_ai_net(ndim=3, nelectrons=s.nelectrons, natoms=s.natoms, nspins=s.nspins, determinants=1,
                             charges=s.charges, parallel_indices=par, antiparallel_indices=anti,
                             n_parallel=npar, n_antiparallel=nanti, spin_up_indices=up, spin_down_indices=dn)
    params = system.init_params(np.random.default_rng(35), s, randomize_aux=True)
    pos = system.init_electrons(np.random.default_rng(36), s.atoms, s.charges, 8, 1.0)
    data = nn.AINetData(positions=torch.tensor(pos, device="cuda"), spins=s.spins, atoms=s.atoms, charges=s.charges)
    e, mat = H.local_energy(f=network.apply, charges=s.charges, nspins=s.spins, complex_output=True)(params, None, data)
    ke = H.local_kinetic_energy(network.apply, complex_output=True)(params, data)
    e_real, _ = H.local_energy(f=network.apply, charges=s.charges, nspins=s.spins)(params, None, data)
    torch.cuda.synchronize()
    assert mat is None and e.is_complex() and ke.is_complex()
    ref = oh.batch_local_energy_complex(onet.Network(s), onet.to_torch(params), torch.tensor(pos)).numpy()
    np.testing.assert_allclose(e.cpu().numpy(), ref, rtol=1e-8, atol=1e-6)
    # KE = E - V: same imaginary part, real parts differ by the (real) potential
    np.testing.assert_allclose(ke.imag.cpu().numpy(), e.imag.cpu().numpy(), rtol=0, atol=1e-12)
    v = (e_real - H.local_kinetic_energy(network.apply, complex_output=False)(params, data)).cpu().numpy()
    np.testing.assert_allclose(e.real.cpu().numpy() - ke.real.cpu().numpy(), v, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_complex_local_energy_waves_and_ragged_batches(dtype):
    """The theta pass in both first-derivative instantiations (one wave per walker, and the
    2 / 4-waves split of small batches) agrees to rounding; ragged and empty batches give the rows
    of the full batch."""
    s, ctx, net, params, pos = _ctx_and_oracle("N2", dtype, 65, 37)
    x = torch.tensor(pos, dtype=dtype, device="cuda").contiguous()
    out = {}
    for w in (1, 2, 4):
        ctx.set_lap_waves(w)
        out[w] = ctx.local_energy_complex(x)
    ctx.set_lap_waves(0)
    full = ctx.local_energy_complex(x)
    part = ctx.local_energy_complex(x[:7])
    empty = ctx.local_energy_complex(x[:0])
    torch.cuda.synchronize()
    tol = 1e-10 if dtype == torch.float64 else 2e-4
    for w in (2, 4):
        d = (out[w] - out[1]).abs() / out[1].abs().clamp(min=1.0)
        assert float(d.max()) < tol, (w, float(d.max()))
    assert torch.equal(part, full[:7])
    assert empty.shape == (0,)


def test_pp_local_energy_complex_output(golden_dir):
    """pphamiltonian.local_energy(..., complex_output=True) (C atom ccECP, the golden walkers and
    rotations): the real-kinetic pp E_L of the golden fixture plus the oracle's phase terms of the
    kinetic energy (complex minus real all-electron E_L; pphamiltonian.py:84-104)."""
    import os
    from oracle import hamiltonian as oh, network as onet, pphamiltonian as opp, system
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
    kw = dict(f=network.apply, lognetwork=None, charges=s.charges, nspins=s.spins, rn_local=e.rn_local,
              local_coes=e.local_coes, local_exps=e.local_exps, rn_non_local=e.rn_non_local,
              non_local_coes=e.non_local_coes, non_local_exps=e.non_local_exps, natoms=1, nelectrons=4, ndim=3,
              list_l=2)
    data = nn.AINetData(positions=torch.tensor(g["pos"], device="cuda"), spins=s.spins, atoms=s.atoms,
                        charges=s.charges)
    rot = pphamiltonian.HostRotations(torch.tensor(g["rot"]))
    out_c, _ = pphamiltonian.local_energy(complex_output=True, **kw)(params, rot, data)
    torch.cuda.synchronize()
    net, pt, x = onet.Network(s), onet.to_torch(params), torch.tensor(g["pos"])
    corr = oh.batch_local_energy_complex(net, pt, x).numpy() - oh.batch_local_energy(net, pt, x)[0].numpy()
    ref = g["e_re"] + 1j * g["e_im"] + corr
    assert np.abs(corr.imag).max() > 1e-3
    np.testing.assert_allclose(out_c.cpu().numpy(), ref, rtol=1e-8, atol=1e-6)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_pp_complex_output_one_call_matches_composition(dtype):
    """aiqmc_local_energy_ecp_complex (one call: the phase terms added to the pp energy directly,
    ADVICE r4) against the composition the drop-in used before -- pp E_L + (complex all-electron
    E_L - real all-electron E_L) -- on 512 C-atom ccECP walkers with the same Philox rotations."""
    from aiqmc import systems
    from aiqmc.initial_electrons_positions.init import init_electrons
    from aiqmc.wavefunction_Ynlm.nn import flatten_params
    s = systems.make_system("C_ecp")
    ctx = s.context(dtype=dtype)
    ctx.set_params(flatten_params(s.make_network().init(3)))
    e = systems.ccecp_tables("C_ecp")
    ctx.set_ecp(e.rn_local, e.local_coes, e.local_exps, e.rn_non_local, e.non_local_coes, e.non_local_exps, e.list_l)
    pos = init_electrons(5, None, s.atoms, s.charges, s.spins, 512, 1.0)[0].to("cuda", dtype).contiguous()
    one = ctx.local_energy_ecp(pos, seed=4, offset=2, complex_output=True)
    pp = ctx.local_energy_ecp(pos, seed=4, offset=2)
    el_c = ctx.local_energy_complex(pos)
    el_r, _, _ = ctx.local_energy(pos)
    comp = pp + (el_c - el_r.to(el_c.real.dtype))
    torch.cuda.synchronize()
    a, b = one.cpu().numpy(), comp.cpu().numpy()
    assert np.isfinite(a).all()
    assert np.abs(a.imag - pp.imag.cpu().numpy()).max() > 1e-3        # the phase terms are there
    if dtype == torch.float64:
        np.testing.assert_allclose(a, b, rtol=1e-10, atol=1e-9)
    else:
        # the composition carries fl(E + x) - E rounding at the scale of |E_L|; the one
        # call adds x itself: compare at fp32 precision relative to |E_L|
        tol = 2e-6 * np.maximum(1.0, np.abs(el_r.double().cpu().numpy()))
        assert (np.abs(a - b) <= 4 * tol + 1e-4 * np.abs(b)).all(), np.abs(a - b).max()
