"""Time the proposal launch with phases skipped (dev build with -DAQ_ABLATE): marginal phase costs.
usage: AIQMC_LIB_VARIANT=dev python tools/ablate.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd"))
import torch
from aiqmc import systems, _lib
from aiqmc.initial_electrons_positions.init import init_electrons
from aiqmc.wavefunction_Ynlm.nn import flatten_params
s = systems.make_system("N2")
ctx = s.context(dtype=torch.float32)
ctx.set_params(flatten_params(s.make_network().init(1)))
B = 4096
pos0 = init_electrons(1000, None, s.atoms, s.charges, s.spins, B, 1.0)[0].to("cuda", torch.float32).contiguous()
names = {0: "full", 1: "-F2patch", 2: "-F4", 4: "-GJ", 8: "-B1", 16: "-B2", 32: "-B3", 64: "-B4",
         2 | 16: "-F4-B2", 32 | 64: "-B3-B4", 8 | 16 | 32 | 64: "-backward", 127: "-all"}
res = {}
for rep in range(2):
    for m, nm in names.items():
        ctx.set_ablate(m)
        pos = pos0.clone()
        ctx.mc_step(pos, 2, 0.05, seed=1, offset=0)
        torch.cuda.synchronize()
        ctx.profile(True)
        for k in range(5):
            pos = pos0.clone()
            ctx.mc_step(pos, 4, 0.05, seed=1, offset=0)
        torch.cuda.synchronize()
        ctx.profile(False)
        pm, pn = ctx.profile_read(_lib.PROF_MC_PROPOSAL)
        ctx.profile_read(_lib.PROF_MC_WALKER)
        res.setdefault(nm, []).append(1e3 * pm / pn)
ctx.set_ablate(0)
base = min(res["full"])
for nm, v in res.items():
    print(f"{nm:12s} {min(v):7.1f} us   saves {base - min(v):6.1f} us")
