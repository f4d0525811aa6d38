"""Precision fixture for the benched fp32 path: the oracle in float64 AND in float32/complex64
(the reference's own dtype) on the same 1,024 N2 walkers.

Run from the repo root (about 30 min on 8 cores):  python tests/golden/make_golden_fp32.py
N2_fp32.npz holds:
  params_flat [P] float64, pos [B,3N] float64 (exactly representable in float32: the walkers
  are rounded to float32 first, so both dtypes see identical coordinates),
  {logabs,grad,e_l}_64 -- float64 oracle, {logabs,grad,e_l}_32 -- float32 oracle (stored as float64).
tests/test_precision_fp32.py compares the HIP fp32 kernels' error against the fp32 oracle's
error, both measured against the float64 oracle.
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import hamiltonian, network, system  # noqa: E402

B = int(os.environ.get("AIQMC_FP32_FIXTURE_B", "1024"))


def main(out_dir: str):
    torch.set_num_threads(os.cpu_count() or 8)
    s = system.make_system("N2")
    rng = np.random.default_rng(31)
    params = system.init_params(rng, s, randomize_aux=True)
    flat = system.flatten_params(params)
    pos = system.init_electrons(rng, s.atoms, s.charges, B, 1.0).astype(np.float32).astype(np.float64)
    net = network.Network(s)
    out = dict(params_flat=flat, pos=pos)
    for dt, tag in ((torch.float64, "64"), (torch.float32, "32")):
        t0 = time.time()
        e, l, g = hamiltonian.batch_local_energy(net, network.to_torch(params, dt), torch.tensor(pos, dtype=dt),
                                                 chunk=16)
        assert e.dtype == dt, e.dtype
        out[f"e_l_{tag}"] = e.double().numpy()
        out[f"logabs_{tag}"] = l.double().numpy()
        out[f"grad_{tag}"] = g.double().numpy()
        print(tag, f"{time.time() - t0:.0f}s", flush=True)
    np.savez_compressed(os.path.join(out_dir, "N2_fp32.npz"), **out)
    d = np.abs(out["e_l_32"] - out["e_l_64"])
    print("fp32 oracle |dE|: median", np.median(d), "p99", np.quantile(d, 0.99), "max", d.max())


if __name__ == "__main__":
    main(os.path.dirname(os.path.abspath(__file__)))
