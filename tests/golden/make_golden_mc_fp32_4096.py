"""Fixture for the benched fp32 Metropolis path at the benched size (BASELINE config: N2, 4096
walkers): one N2 sweep with injected draws through the oracle (oracle/mcstep.py,
VMCmcstep.py:11-111) in float32/complex64, the reference's own dtype.

Run from the repo root (a few minutes on 8 cores):  python tests/golden/make_golden_mc_fp32_4096.py
The inputs are not stored: inputs_4096() regenerates them (numpy default_rng(SEED), float32-valued)
and tests/test_gpu_mc_fp32.py imports it.  N2_mc_fp32_4096.npz holds
  params_flat, tstep          the network (oracle/system.py init_params, randomize_aux) and tau
  x32 [B,3N] float32          positions after the sweep
  ratio32 [B,N] float32       |exp(log|psi(x')| - log|psi(x)|)|^2 t_pro  (:100)
  cond32 [B,N] bool           ratio > u  (walkers_accept, :18-25)
  te32 [2]                    limdrift factors of the walker and proposal gradients (:60, :80)
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import system  # noqa: E402

TSTEP = 0.05
B = 4096
SEED = 4096


def inputs_4096():
    """params, float32-valued pos0 [B,3N], gauss1 [B,3N], gauss2d [B,N,3], u [B,N] (float64 arrays)."""
    s = system.make_system("N2")
    N = s.nelectrons
    rng = np.random.default_rng(SEED)
    params = system.init_params(rng, s, randomize_aux=True)
    f32 = lambda a: a.astype(np.float32).astype(np.float64)
    pos0 = f32(system.init_electrons(rng, s.atoms, s.charges, B, 1.0))
    g1 = f32(rng.standard_normal((B, 3 * N)))
    g2d = f32(rng.standard_normal((B, N, 3)))
    u = f32(rng.uniform(size=(B, N)))
    return s, params, pos0, g1, g2d, u


def main(out_dir: str):
    import torch
    from oracle import mcstep, network
    torch.set_num_threads(os.cpu_count() or 8)
    s, params, pos0, g1, g2d, u = inputs_4096()
    N = s.nelectrons
    g2 = np.zeros((B, N, N, 3))
    g2[:, np.arange(N), np.arange(N), :] = g2d
    g2 = g2.reshape(B, N, 3 * N)
    net = network.Network(s)
    dt = torch.float32
    pt = network.to_torch(params, dt)
    t0 = time.time()
    info = {}
    x, ratio = mcstep.walkers_update(net, pt, torch.tensor(pos0, dtype=dt), torch.tensor(g1, dtype=dt),
                                     torch.tensor(g2, dtype=dt), torch.tensor(u, dtype=dt), TSTEP, info=info)
    assert x.dtype == dt
    print(f"{time.time() - t0:.0f}s accepted", int(info["cond"].sum()), flush=True)
    np.savez_compressed(os.path.join(out_dir, "N2_mc_fp32_4096.npz"), params_flat=system.flatten_params(params),
                        tstep=np.float64(TSTEP), x32=x.numpy(), ratio32=ratio.numpy().astype(np.float32),
                        cond32=info["cond"].numpy(),
                        te32=np.array([float(info["taueff_walkers"]), float(info["taueff_proposals"])]))


if __name__ == "__main__":
    main(os.path.dirname(os.path.abspath(__file__)))
