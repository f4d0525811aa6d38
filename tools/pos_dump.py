"""Walker positions after a few Metropolis steps (N2, fp32, Philox draws), saved for a bitwise
comparison of two library variants (AIQMC_LIB_VARIANT).  usage: python tools/pos_dump.py OUT.npy [system] [walkers]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd"))
import numpy as np
import torch
from aiqmc import systems
from aiqmc.initial_electrons_positions.init import init_electrons
from aiqmc.wavefunction_Ynlm.nn import flatten_params
name = sys.argv[2] if len(sys.argv) > 2 else "N2"
s = systems.make_system(name)
ctx = s.context(dtype=torch.float32)
ctx.set_params(flatten_params(s.make_network().init(1)))
B = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
pos = init_electrons(1000, None, s.atoms, s.charges, s.spins, B, 1.0)[0].to("cuda", torch.float32).contiguous()
for k in range(3):
    ctx.mc_step(pos, 10, 0.05, seed=7, offset=10 * k)
el, _, _ = ctx.local_energy(pos)
np.save(sys.argv[1], np.concatenate([pos.cpu().numpy().ravel(), el.cpu().numpy().ravel()]))
print(name, "saved", sys.argv[1], flush=True)
