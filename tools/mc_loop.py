"""Short N2 VMC loop for profiling passes: warm-up, then `iters` iterations of mc_step (10 sweeps)
+ local_energy on 4096 walkers, fp32, Philox draws.  usage: python tools/mc_loop.py [iters] [system] [walkers]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd"))
import torch
from aiqmc import systems, _lib
from aiqmc.initial_electrons_positions.init import init_electrons
from aiqmc.wavefunction_Ynlm.nn import flatten_params
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
NS = int(os.environ.get("AIQMC_NSTEPS", "10"))   # sweeps per mc_step call
name = sys.argv[2] if len(sys.argv) > 2 else "N2"
B = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
s = systems.make_system(name)
ctx = s.context(dtype=torch.float32)
ctx.set_params(flatten_params(s.make_network().init(1)))
if os.environ.get("AIQMC_NOFUSE"):
    ctx.set_fuse_accept(False)
if os.environ.get("AIQMC_FUSE_REDUCE"):     # 0: integer reduction launches, 1: by batch size (default), 2: integer atomics, 3: fp64 k_taueff launches
    ctx.set_fuse_reduce(int(os.environ["AIQMC_FUSE_REDUCE"]))
if os.environ.get("AIQMC_LAPW"):      # waves per walker of the local energy's second launch
    ctx.set_lap_waves(int(os.environ["AIQMC_LAPW"]))
if os.environ.get("AIQMC_WPIV") == "0":   # walker launches: partial pivoting every sweep
    ctx.set_walker_pivots(False)
if os.environ.get("AIQMC_PACKW") == "0":   # N <= 8 walker launches one wave each
    ctx.set_packed_walkers(False)
if os.environ.get("AIQMC_NOREUSE"):   # every proposal from scratch (PMC comparison of the two paths)
    ctx.set_proposal_reuse(False)
pos = init_electrons(1000, None, s.atoms, s.charges, s.spins, B, 1.0)[0].to("cuda", torch.float32).contiguous()
draws = {}
if os.environ.get("AIQMC_HOST_DRAWS"):   # device-resident draws passed in (no Philox in the walker launch)
    N = s.nelectrons
    g = torch.Generator(device="cuda").manual_seed(3)
    draws = dict(gauss1=torch.randn(10, B, 3 * N, device="cuda", generator=g),
                 gauss2=torch.randn(10, B, N, 3, device="cuda", generator=g),
                 u=torch.rand(10, B, N, device="cuda", generator=g))
ctx.mc_step(pos, NS, 0.05, seed=1, offset=0, **draws)
ctx.local_energy(pos)
torch.cuda.synchronize()
noprof = bool(os.environ.get("AIQMC_NOPROF"))   # no HIP events around the launches
ctx.profile(not noprof)
t0 = time.perf_counter()
for k in range(iters):
    ctx.mc_step(pos, NS, 0.05, seed=1, offset=NS * (k + 1), **draws)
    el, _, _ = ctx.local_energy(pos)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / iters
ctx.profile(False)
pm, pn = ctx.profile_read(_lib.PROF_MC_PROPOSAL)
wm, wn = ctx.profile_read(_lib.PROF_MC_WALKER)
lm, ln = ctx.profile_read(_lib.PROF_LOCAL_ENERGY)
print(f"{name} B={B}: {1e3 * dt:.3f} ms/iter  proposal {1e3 * pm / max(pn, 1):.1f} us  walker {1e3 * wm / max(wn, 1):.1f} us"
      f"  local-energy pair {1e3 * lm / max(ln, 1):.1f} us  finite={bool(torch.isfinite(el).all())}", flush=True)
