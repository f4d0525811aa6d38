"""Host side of the benched N2 iteration: time to ENQUEUE K iterations (mc_step + local_energy +
pmean_stats, no synchronisation) against the time to complete them.  If the enqueue rate is close to
the completion rate the GPU waits for the host.  usage: python tools/host_probe.py [walkers] [K]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd"))
import torch
from aiqmc import systems, constants
from aiqmc.initial_electrons_positions.init import init_electrons
from aiqmc.wavefunction_Ynlm.nn import flatten_params
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
s = systems.make_system("N2")
ctx = s.context(dtype=torch.float32)
ctx.set_params(flatten_params(s.make_network().init(1)))
pos = init_electrons(1000, None, s.atoms, s.charges, s.spins, B, 1.0)[0].to("cuda", torch.float32).contiguous()
el = torch.empty(B, dtype=torch.float32, device="cuda")
off = 0
for _ in range(3):
    ctx.mc_step(pos, 10, 0.05, seed=1, offset=off); off += 10
    ctx.local_energy(pos, out=el); constants.pmean_stats(el)
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    parts = [0.0, 0.0, 0.0]
    for _ in range(K):
        a = time.perf_counter(); ctx.mc_step(pos, 10, 0.05, seed=1, offset=off); off += 10
        b = time.perf_counter(); ctx.local_energy(pos, out=el)
        c = time.perf_counter(); constants.pmean_stats(el)
        d = time.perf_counter()
        parts[0] += b - a; parts[1] += c - b; parts[2] += d - c
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"B={B} K={K}: enqueue {1e3 * (t1 - t0) / K:.3f} ms/iter (mc_step {1e3 * parts[0] / K:.3f}, local_energy "
          f"{1e3 * parts[1] / K:.3f}, pmean_stats {1e3 * parts[2] / K:.3f}), complete {1e3 * (t2 - t0) / K:.3f} ms/iter",
          flush=True)
