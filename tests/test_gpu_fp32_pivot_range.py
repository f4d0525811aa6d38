"""fp32 Gauss-Jordan / LU pivots outside the float range of |pivot|^2.

A far-out electron scales its row of A = Phi * Yt by its envelope (envelope.py:26-30,
network_blocks.py:156 takes slogdet of it):
* the reference's default envelope has the signed term sigma xi exp(-pi ae) (pi = sigma = xi = 1 at
  init), ~2e20 for an N2 electron 50 bohr on the negative side of an atom: |pivot|^2 ~ 1e40
  overflows float32 (before the fix: 1 / pivot = 0, log|det| = +inf, a silently wrong inverse);
* a Gaussian-only envelope (sigma = 0) gives exp(-beta r^2), ~1e-27 at 7.6 bohr: |pivot|^2 ~ 1e-54
  underflows to 0 (before the fix: log|det| = -inf, proposal ratios exp(-inf + inf) = NaN).
jets.h pivot_recip / pivot_recip_me scale such pivots by the power of two of their larger
component and pivot_mag2 forms |pivot|^2 in double, so every quantity is formed in range; the
fixed-order eliminations (gj_fixed_regs, proposals and later-sweep walker launches) send a pivot
outside the range to the pivoted fallback.  Here the fp32 kernels must be finite and agree
with the fp64 kernels (whose |pivot|^2 stays in range) on the same float-rounded positions, through
every launch that eliminates: the walker launch (logpsi_grad), the Metropolis proposals (mc_step,
one host-draw sweep: decisions and positions), the local-energy pair, and an N <= 8 system (the C
atom: packed k_quad_grad walker / proposal launches).  Synthetic walkers: init_electrons (seeded)
with one electron moved out along -x.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TSTEP = 0.05


def _ctx(name, dtype, gaussian_only):
    from oracle import system
    from aiqmc import _lib
    s = system.make_system(name)
    t = s.tables()
    ctx = _lib.Context(s.nelectrons, s.natoms, s.nspins, s.atoms, s.charges, t["spin_up_indices"],
                       t["spin_down_indices"], t["parallel_indices"], t["antiparallel_indices"], dtype=dtype,
                       device=0)
    p = system.init_params(np.random.default_rng(1), s)
    if gaussian_only:
        for env in p["envelope"]:
            env["sigma"] = np.zeros_like(env["sigma"])
    ctx.set_params(system.flatten_params(p))
    return s, ctx


# (gaussian_only, distance of the moved electron along -x from the first atom); the far row's
# max |A[i][c]| (oracle, walker 0) in the comment, N2 / C
CASES = [
    (False, 45.0),    # 1e18 / 7e19: |pivot|^2 past 1e36, float max 3.4e38
    (False, 50.0),    # 2e20 / 1e22 ("about -50 bohr along an axis, so the row is ~1e21")
    (False, 70.0),    # 8e28 / 8e30
    (True, 7.6),      # 1e-27 / 3e-26 (row scale <= 1e-25, |pivot|^2 underflows)
    (True, 8.3),      # 2e-32 / 5e-31
]


def _walkers(s, B, gaussian_only, dist, seed=3):
    from oracle import system
    x = system.init_electrons(np.random.default_rng(seed), s.atoms, s.charges, B, 1.0).reshape(B, s.nelectrons, 3)
    a0 = np.asarray(s.atoms, dtype=np.float64)[0]
    # walker b moves electron b % N out (every electron index gets a far-out row over the batch)
    for b in range(B):
        e = b % s.nelectrons
        x[b, e] = a0 + np.array([-dist, 0.3, -0.2])
    return np.ascontiguousarray(x.reshape(B, -1)).astype(np.float32).astype(np.float64)


def _far_row_scale(name, gaussian_only, x0):
    """max |A[i][c]| of the far electron's row of walker x0, A = Phi * Yt * e^{J/N} (the oracle's
    make_orbitals restatement, nn.py:485-506 / envelope.py:26-30)."""
    from oracle import network, system
    s = system.make_system(name)
    p = system.init_params(np.random.default_rng(1), s)
    if gaussian_only:
        for env in p["envelope"]:
            env["sigma"] = np.zeros_like(env["sigma"])
    m = network.Network(s).orbitals(network.to_torch(p), torch.tensor(x0))
    return float(m.abs().amax(1)[0])


def _ids(c):
    return f"{'gauss' if c[0] else 'signed'}-{c[1]}"


@pytest.mark.parametrize("name", ["N2", "C"])
@pytest.mark.parametrize("case", CASES, ids=_ids)
def test_fp32_walker_and_local_energy_with_out_of_range_pivots(name, case):
    gaussian_only, dist = case
    s, c32 = _ctx(name, torch.float32, gaussian_only)
    _, c64 = _ctx(name, torch.float64, gaussian_only)
    N = s.nelectrons
    x = _walkers(s, 2 * N, gaussian_only, dist)
    x64 = torch.tensor(x, device="cuda").contiguous()
    x32 = x64.float().contiguous()
    l64, g64 = c64.logpsi_grad(x64)
    l32, g32 = c32.logpsi_grad(x32)
    assert torch.isfinite(l64).all() and torch.isfinite(g64).all()
    # the case really leaves the float range of |pivot|^2: the far row's scale (fp64 oracle matrix)
    rmax = _far_row_scale(name, gaussian_only, x[0])
    assert (rmax > 1e17) if not gaussian_only else (rmax < 1e-17), rmax
    assert torch.isfinite(l32).all(), l32
    assert torch.isfinite(g32).all(), (~torch.isfinite(g32)).any(1).nonzero().flatten().tolist()
    np.testing.assert_allclose(l32.double().cpu().numpy(), l64.cpu().numpy(), rtol=2e-6, atol=2e-4)
    np.testing.assert_allclose(g32.double().cpu().numpy(), g64.cpu().numpy(), rtol=1e-3, atol=1e-3)
    # the local-energy launch pair (adjoint pass + first-derivative pass)
    e64, m64, h64 = c64.local_energy(x64, want_logabs=True, want_grad=True)
    e32, m32, h32 = c32.local_energy(x32, want_logabs=True, want_grad=True)
    assert torch.isfinite(e64).all()
    assert torch.isfinite(e32).all() and torch.isfinite(h32).all(), e32
    np.testing.assert_allclose(m32.double().cpu().numpy(), m64.cpu().numpy(), rtol=2e-6, atol=2e-4)
    np.testing.assert_allclose(h32.double().cpu().numpy(), h64.cpu().numpy(), rtol=1e-3, atol=1e-3)
    np.testing.assert_allclose(e32.double().cpu().numpy(), e64.cpu().numpy(), rtol=1e-3, atol=5e-2)


@pytest.mark.parametrize("name", ["N2", "C"])
@pytest.mark.parametrize("case", CASES, ids=_ids)
def test_fp32_proposals_with_out_of_range_pivots(name, case):
    """One host-draw Metropolis sweep over a batch of ordinary walkers plus far-electron walkers:
    the far walkers' proposals must neither poison the batch's limdrift sum (a NaN gradient
    rejects every move, VMCmcstep.py:58-60) nor decide differently from fp64."""
    gaussian_only, dist = case
    s, c32 = _ctx(name, torch.float32, gaussian_only)
    _, c64 = _ctx(name, torch.float64, gaussian_only)
    from oracle import system
    N, B, NF = s.nelectrons, 256, 2 * s.nelectrons
    xo = system.init_electrons(np.random.default_rng(8), s.atoms, s.charges, B - NF, 1.0)
    x = np.concatenate([_walkers(s, NF, gaussian_only, dist), xo.astype(np.float32).astype(np.float64)])
    g = torch.Generator().manual_seed(4)
    kw = dict(gauss1=torch.randn(1, B, 3 * N, generator=g, dtype=torch.float64),
              gauss2=torch.randn(1, B, N, 3, generator=g, dtype=torch.float64),
              u=torch.rand(1, B, N, generator=g, dtype=torch.float64))
    a = torch.tensor(x, device="cuda").contiguous()
    b = a.float().contiguous()
    acc64 = c64.mc_step(a, 1, TSTEP, count_accepts=True, **kw)
    acc32 = c32.mc_step(b, 1, TSTEP, count_accepts=True, **kw)
    torch.cuda.synchronize()
    assert torch.isfinite(b).all()
    n64, n32 = int(acc64.sum()), int(acc32.sum())
    assert n64 > B // 4, n64                      # the sweep moves (limdrift finite in fp64)
    assert abs(n32 - n64) <= 2, (n32, n64)        # and in fp32 (a NaN limdrift would reject all)
    dw = (b.double() - a).abs().reshape(B, -1).amax(1)
    flipped = dw > 1e-3
    assert int(flipped.sum()) <= 2, dw.topk(4)
    assert float(dw[~flipped].max()) < 5e-5 * max(1.0, dist / 10), float(dw[~flipped].max())
