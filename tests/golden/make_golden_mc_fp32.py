"""Fixture for the benched fp32 Metropolis path (VERDICT r3 "Next" #6): N2 sweeps with injected
draws through the oracle (oracle/mcstep.py, VMCmcstep.py:11-111) in float32/complex64 -- the
reference's own dtype -- and in float64, from the same float32-representable walkers.

Run from the repo root (a few minutes on 8 cores):  python tests/golden/make_golden_mc_fp32.py
N2_mc_fp32.npz holds, for each batch size B in {64, 512} (keys suffixed _<B>):
  pos0 [B,3N]                          starting walkers (float32)
  gauss1 [2,B,3N], gauss2d [2,B,N,3], u [2,B,N]   the draws of two sweeps (float32; gauss2d
                                       = the electron-diagonal blocks of the reference's [B,N,3N]
                                       draw, the only part VMCmcstep.py:83-94 reads)
  and per dtype tag t in {32, 64} and sweep s in {0, 1} (sweep 1 starts from that dtype's own
  sweep-0 result):
  x{t}_{s} [B,3N]       positions after the sweep (in that dtype)
  ratio{t}_{s} [B,N]    |exp(log|psi(x')| - log|psi(x)|)|^2 t_pro  (:100)
  cond{t}_{s} [B,N]     ratio > u  (walkers_accept, :18-25)
  te{t}_{s} [2]         limdrift factors of the walker and the proposal gradients (:60, :80)
tests/test_gpu_mc_fp32.py runs the HIP fp32 mc_step on the same inputs.
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import mcstep, network, system  # noqa: E402

TSTEP = 0.05


def main(out_dir: str):
    torch.set_num_threads(os.cpu_count() or 8)
    s = system.make_system("N2")
    N = s.nelectrons
    rng = np.random.default_rng(47)
    params = system.init_params(rng, s, randomize_aux=True)
    out = dict(params_flat=system.flatten_params(params), tstep=np.float64(TSTEP))
    net = network.Network(s)
    f32 = lambda a: a.astype(np.float32).astype(np.float64)
    st32 = lambda a: a.astype(np.float32)   # float32-valued arrays are stored as float32
    for B in (64, 512):
        pos0 = f32(system.init_electrons(rng, s.atoms, s.charges, B, 1.0))
        g1 = f32(rng.standard_normal((2, B, 3 * N)))
        g2d = f32(rng.standard_normal((2, B, N, 3)))
        u = f32(rng.uniform(size=(2, B, N)))
        g2 = np.zeros((2, B, N, N, 3))
        g2[:, :, np.arange(N), np.arange(N), :] = g2d
        g2 = g2.reshape(2, B, N, 3 * N)
        out.update({f"pos0_{B}": st32(pos0), f"gauss1_{B}": st32(g1), f"gauss2d_{B}": st32(g2d), f"u_{B}": st32(u)})
        for dt, tag in ((torch.float32, "32"), (torch.float64, "64")):
            pt = network.to_torch(params, dt)
            x = torch.tensor(pos0, dtype=dt)
            for st in range(2):
                t0 = time.time()
                info = {}
                x, ratio = mcstep.walkers_update(net, pt, x, torch.tensor(g1[st], dtype=dt),
                                                 torch.tensor(g2[st], dtype=dt), torch.tensor(u[st], dtype=dt),
                                                 TSTEP, info=info)
                assert x.dtype == dt
                out[f"x{tag}_{st}_{B}"] = x.numpy()
                out[f"ratio{tag}_{st}_{B}"] = ratio.numpy()
                out[f"cond{tag}_{st}_{B}"] = info["cond"].numpy()
                out[f"te{tag}_{st}_{B}"] = np.array([float(info["taueff_walkers"]), float(info["taueff_proposals"])])
                print(B, tag, st, f"{time.time() - t0:.0f}s", "accepted", int(info["cond"].sum()), flush=True)
        for st in range(2):
            c32, c64 = out[f"cond32_{st}_{B}"], out[f"cond64_{st}_{B}"]
            print(B, st, "fp32 vs fp64 oracle decisions differ:", int((c32 != c64).sum()))
    np.savez_compressed(os.path.join(out_dir, "N2_mc_fp32.npz"), **out)


if __name__ == "__main__":
    main(os.path.dirname(os.path.abspath(__file__)))
