"""pp local energy of a ccECP system with the walker cache on (packed quadrature kernel for
N <= 8) and off (one configuration per wave, k_walker_rev's general path), same rotations.
usage: python tools/ecp_ab.py [system] [walkers]"""
import json, os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd"))
from aiqmc import systems  # noqa: E402
from aiqmc.initial_electrons_positions.init import init_electrons  # noqa: E402
from aiqmc.wavefunction_Ynlm.nn import flatten_params  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2_ecp"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
s = systems.make_system(name)
ctx = s.context(dtype=torch.float32)
ctx.set_params(flatten_params(s.make_network().init(1)))
e = systems.ccecp_tables(name)
ctx.set_ecp(e.rn_local, e.local_coes, e.local_exps, e.rn_non_local, e.non_local_coes, e.non_local_exps, e.list_l)
pos = init_electrons(7, None, s.atoms, s.charges, s.spins, B, 1.0)[0].to("cuda", torch.float32).contiguous()
res = {}
for reuse in (True, False):
    ctx.set_proposal_reuse(reuse)
    ctx.local_energy_ecp(pos, seed=3, offset=0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(3):
        out = ctx.local_energy_ecp(pos, seed=3, offset=1 + k)
    torch.cuda.synchronize()
    res["packed" if reuse else "one_per_wave"] = {"ms": 1e3 * (time.perf_counter() - t0) / 3,
                                                  "mean_re": float(out.real.mean())}
ctx.set_proposal_reuse(True)
print(json.dumps({"system": name, "walkers": B, **res}))
