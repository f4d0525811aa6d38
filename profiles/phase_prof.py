"""Per-phase cycle breakdown of the reverse-mode value+gradient kernel.

Needs the diagnostics library (`make -C <pkg>/csrc phaseprof`); run as
    AIQMC_LIB_VARIANT=phaseprof python profiles/phase_prof.py
Shader-clock cycles (s_memtime) between phase boundaries, summed over waves and
divided by the wave count: wall cycles per wave, including time the wave was
resident but not issuing (latency and co-resident waves), so the shares show
where waves spend their residency.
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd"))

from oracle import system  # noqa: E402  (test infrastructure: system tables + random init)
from aiqmc import _lib  # noqa: E402

PHASES = ["F0 positions/cache", "F1 electron stage", "F2 pair stream", "F4 h layers", "F5 Phi + GJ",
          "B1 H/Yt adjoints", "B2 layers back", "B3 pair back", "B4 gradient", "outputs"]


def main():
    name = os.environ.get("SYSTEM", "N2")
    B = int(os.environ.get("WALKERS", "4096"))
    s = system.make_system(name)
    t = s.tables()
    ctx = _lib.Context(s.nelectrons, s.natoms, s.nspins, s.atoms, s.charges, t["spin_up_indices"],
                       t["spin_down_indices"], t["parallel_indices"], t["antiparallel_indices"],
                       dtype=torch.float32, device=0)
    ctx.set_params(system.flatten_params(system.init_params(np.random.default_rng(0), s)))
    pos = torch.tensor(system.init_electrons(np.random.default_rng(1), s.atoms, s.charges, B, 1.0),
                       dtype=torch.float32, device="cuda").contiguous()
    out = {}
    for reuse in (True, False):
        ctx.set_proposal_reuse(reuse)
        ctx.mc_step(pos, 2, 0.05, seed=1)
        ctx.phase_cycles()
        sweeps = 5
        ctx.mc_step(pos, sweeps, 0.05, seed=2)
        cyc = ctx.phase_cycles().astype(np.float64)
        res = {}
        for kind, off, waves in (("walker", 0, B * sweeps), ("proposal", 16, B * s.nelectrons * sweeps)):
            per = cyc[off:off + 10] / waves
            res[kind] = {PHASES[k]: round(float(per[k]), 1) for k in range(10)}
            res[kind]["total"] = round(float(per.sum()), 1)
        res["gj_fallbacks_per_proposal"] = float(cyc[15]) / (B * s.nelectrons * sweeps)
        out["reuse" if reuse else "recompute"] = res
    ctx.set_proposal_reuse(True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
