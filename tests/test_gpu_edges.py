"""Edge cases of the C-ABI on the GPU: empty batches, calls before set_params, bad
arguments (negative codes + aiqmc_last_error, raised as RuntimeError/ValueError by the host
layer), and the largest single-GPU batch of BASELINE.json (the 8-GPU N2 config's 32768
walkers on one device)."""
import numpy as np
import pytest
import torch

from oracle import pphamiltonian as opp, system


def _ctx(name, dtype=torch.float64, params=True, ecp=False):
    from aiqmc import _lib
    s = system.make_system(name)
    t = s.tables()
    ctx = _lib.Context(s.nelectrons, s.natoms, s.nspins, s.atoms, s.charges, t["spin_up_indices"],
                       t["spin_down_indices"], t["parallel_indices"], t["antiparallel_indices"], dtype=dtype, device=0)
    if params:
        ctx.set_params(system.flatten_params(system.init_params(np.random.default_rng(3), s, randomize_aux=True)))
    if ecp:
        e = opp.c_atom_ccecp()
        ctx.set_ecp(e.rn_local, e.local_coes, e.local_exps, e.rn_non_local, e.non_local_coes, e.non_local_exps,
                    e.list_l)
    return s, ctx


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_empty_batches_are_no_ops(dtype):
    s, ctx = _ctx("C_ecp", dtype, ecp=True)
    empty = torch.empty(0, 3 * s.nelectrons, dtype=dtype, device="cuda")
    la, ph = ctx.logpsi(empty)
    assert la.numel() == 0 and ph.numel() == 0
    la, g = ctx.logpsi_grad(empty)
    assert g.shape == (0, 3 * s.nelectrons)
    el, _, _ = ctx.local_energy(empty)
    assert el.numel() == 0
    ctx.mc_step(empty, 3, 0.05, seed=1)
    assert ctx.local_energy_ecp(empty, seed=1).numel() == 0
    assert ctx.dmc_tmoves(empty, 0.1, seed=1).shape == (0, s.nelectrons)
    assert ctx.logpsi_param_grad(empty).shape == (0, ctx.nparams)
    go, gn, _ = ctx.dmc_drift_diffusion(empty, 0.05, seed=1)
    assert go.numel() == 0 and gn.numel() == 0
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_calls_before_set_params_raise():
    s, ctx = _ctx("Be", params=False)
    pos = torch.zeros(2, 3 * s.nelectrons, dtype=torch.float64, device="cuda")
    with pytest.raises(RuntimeError, match="aiqmc_set_params has not been called"):
        ctx.logpsi(pos)
    with pytest.raises(RuntimeError, match="aiqmc_set_params has not been called"):
        ctx.mc_step(pos, 1, 0.05)


@pytest.mark.gpu
def test_bad_arguments_raise():
    s, ctx = _ctx("C_ecp")
    N = s.nelectrons
    pos = torch.tensor(system.init_electrons(np.random.default_rng(1), s.atoms, s.charges, 4, 1.0), device="cuda")
    with pytest.raises(ValueError):
        ctx.logpsi(pos[:, :-1])                       # trailing dim != 3N
    with pytest.raises(ValueError):
        ctx.set_params(np.zeros(ctx.nparams + 1))
    with pytest.raises(RuntimeError, match="aiqmc_set_ecp has not been called"):
        ctx.dmc_tmoves(pos.contiguous(), 0.1, seed=1)
    e = opp.c_atom_ccecp()
    ctx.set_ecp(e.rn_local, e.local_coes, e.local_exps, e.rn_non_local, e.non_local_coes, e.non_local_exps, e.list_l)
    with pytest.raises(RuntimeError, match="tstep"):
        ctx.dmc_tmoves(pos.contiguous(), 0.0, seed=1)
    with pytest.raises(ValueError):
        ctx.dmc_tmoves(pos.contiguous(), 0.1, rot=torch.eye(3).expand(4, 3, 3))   # partial host draws
    with pytest.raises(ValueError):
        ctx.dmc_tmoves(pos.t(), 0.1, seed=1)          # not contiguous / not in place-able
    with pytest.raises(ValueError):
        ctx.mc_step(pos.float(), 1, 0.05)             # wrong dtype for an in-place update
    # the context stays usable after failed calls
    la, _ = ctx.logpsi(pos)
    torch.cuda.synchronize()
    assert torch.isfinite(la).all()


@pytest.mark.gpu
def test_largest_single_gpu_batch_n2():
    """32768 N2 walkers (BASELINE config 'N2, 32768 walkers', all on one GPU): Philox sweeps,
    local energy and the gradient stay finite and batch-independent (a slice evaluated alone
    gives the same values)."""
    s, ctx = _ctx("N2", torch.float32)
    B = 32768
    from aiqmc.initial_electrons_positions.init import init_electrons
    pos, _ = init_electrons(3, None, s.atoms, s.charges, s.spins, B, 1.0)
    pos = pos.to("cuda", torch.float32).contiguous()
    ctx.mc_step(pos, 2, 0.05, seed=5, offset=0)
    el, la, g = ctx.local_energy(pos, want_logabs=True, want_grad=True)
    torch.cuda.synchronize()
    assert torch.isfinite(pos).all() and torch.isfinite(el).all() and torch.isfinite(g).all()
    sub = pos[B - 100:].contiguous()
    el2, la2, _ = ctx.local_energy(sub, want_logabs=True)
    ctx.set_lap_waves(1)   # the 32768-walker launch's layout: one wave per walker
    el1, _, _ = ctx.local_energy(sub, want_logabs=True)
    ctx.set_lap_waves(0)
    torch.cuda.synchronize()
    assert torch.equal(la[B - 100:], la2)
    assert torch.allclose(el[B - 100:], el1, rtol=1e-5, atol=1e-4)
    # by default 100 walkers run the first-derivative pass 4 waves per walker (partial sums in
    # another order): equal to fp32 rounding of the near-nodal walkers' large E_L
    assert torch.allclose(el[B - 100:], el2, rtol=2e-4, atol=2e-3)
