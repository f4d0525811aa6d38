"""Does a hipGraph of the Metropolis sweep pay?  Times mc_step (10 sweeps, N2, 4096 walkers, fp32)
launched eagerly vs replayed from a captured graph (torch.cuda.CUDAGraph over the HIP stream the
C-ABI launches on).  The replay reuses the captured Philox offset, so it is a timing probe only."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd"))
import torch
from aiqmc import systems
from aiqmc.initial_electrons_positions.init import init_electrons
from aiqmc.wavefunction_Ynlm.nn import flatten_params
s = systems.make_system("N2")
ctx = s.context(dtype=torch.float32)
ctx.set_params(flatten_params(s.make_network().init(1)))
pos = init_electrons(1000, None, s.atoms, s.charges, s.spins, 4096, 1.0)[0].to("cuda", torch.float32).contiguous()
ITER = 30
stream = torch.cuda.Stream()
with torch.cuda.stream(stream):
    for _ in range(3):
        ctx.mc_step(pos, 10, 0.05, seed=1, offset=0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(ITER):
        ctx.mc_step(pos, 10, 0.05, seed=1, offset=k)
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / ITER
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        ctx.mc_step(pos, 10, 0.05, seed=1, offset=0)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(ITER):
        g.replay()
    torch.cuda.synchronize()
    graph = (time.perf_counter() - t0) / ITER
print(f"mc_step (10 sweeps, 51 launches): eager {1e3 * eager:.3f} ms  graph replay {1e3 * graph:.3f} ms  "
      f"finite={bool(torch.isfinite(pos).all())}", flush=True)
