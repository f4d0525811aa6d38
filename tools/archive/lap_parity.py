"""Local-energy parity of a (dev) library variant against the float64 oracle: the N2 golden
fixture (8 walkers, fp64 and fp32) and N2_fp32.npz (1,024 walkers: fp64 max error, fp32 error
quantiles against the fp32 oracle's).  usage: AIQMC_LIB_VARIANT=<tag> python tools/lap_parity.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd"))
import numpy as np
import torch
from oracle import system
from aiqmc import _lib


def ctx_for(name, dtype):
    s = system.make_system(name)
    t = s.tables()
    return _lib.Context(s.nelectrons, s.natoms, s.nspins, s.atoms, s.charges, t["spin_up_indices"],
                        t["spin_down_indices"], t["parallel_indices"], t["antiparallel_indices"], dtype=dtype, device=0)


def main():
    tag = os.environ.get("AIQMC_LIB_VARIANT", "")
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "N2.npz")))
    for dtype in (torch.float64, torch.float32):
        ctx = ctx_for("N2", dtype)
        ctx.set_params(g["params_flat"])
        el, _, _ = ctx.local_energy(torch.tensor(g["pos"], dtype=dtype, device="cuda"))
        torch.cuda.synchronize()
        d = np.abs(el.double().cpu().numpy() - g["e_l"])
        print(f"[{tag}] N2 golden {dtype}: max |dE_L| {d.max():.3e}  max rel {np.max(d / np.abs(g['e_l'])):.3e}")
    f = dict(np.load(os.path.join(ROOT, "tests", "golden", "N2_fp32.npz")))
    print("keys", sorted(f))
    pos = f["pos"]
    for dtype in (torch.float64, torch.float32):
        ctx = ctx_for("N2", dtype)
        ctx.set_params(f["params_flat"])
        el, _, _ = ctx.local_energy(torch.tensor(pos, dtype=dtype, device="cuda"))
        torch.cuda.synchronize()
        d = np.abs(el.double().cpu().numpy() - f["e_l_64"])
        qs = np.quantile(d, [0.5, 0.9, 0.95, 0.99, 0.995, 1.0])
        print(f"[{tag}] N2_fp32 {dtype}: |dE_L| p50/p90/p95/p99/p99.5/max " + " ".join(f"{x:.3e}" for x in qs))
    d32 = np.abs(f["e_l_32"] - f["e_l_64"])
    qs = np.quantile(d32, [0.5, 0.9, 0.95, 0.99, 0.995, 1.0])
    print("fp32 oracle: " + " ".join(f"{x:.3e}" for x in qs))


if __name__ == "__main__":
    main()
