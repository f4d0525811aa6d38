"""Per-phase wall cycles per wave of the local energy's two launches (N2, 4096 walkers, fp32): the adjoint
pass k_walker_rev<PREP> (phases of walker_rev.h) and k_walker_lap (LPH marks of walker_lap.h).  Needs a
-DAQ_PHASE_PROF library: tools/build_variant.sh lphase "-DAQ_PHASE_PROF"; AIQMC_LIB_VARIANT=lphase python tools/lap_phase.py"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd"))
import torch
from aiqmc import systems
from aiqmc.initial_electrons_positions.init import init_electrons
from aiqmc.wavefunction_Ynlm.nn import flatten_params

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
R = 5
s = systems.make_system("N2")
ctx = s.context(dtype=torch.float32)
ctx.set_params(flatten_params(s.make_network().init(1)))
pos = init_electrons(1000, None, s.atoms, s.charges, s.spins, B, 1.0)[0].to("cuda", torch.float32).contiguous()
ctx.local_energy(pos)
torch.cuda.synchronize()
ctx.phase_cycles()   # read-and-reset
for _ in range(R):
    ctx.local_energy(pos)
torch.cuda.synchronize()
c = np.asarray(ctx.phase_cycles(), dtype=np.float64) / (R * B)
prep = ["F0 positions", "F1 electron stage", "F2 pair stream", "F4 h layers", "F5 Phi+GJ", "B1 H/Yt adj",
        "B2 layers back", "pair pass (LapCache)", "-", "-"]
lap = ["stage copy + electron stage", "Yt jets", "layer 0", "layer 1", "layer 2", "E1 + Q_f staging", "E2",
       "E3", "E4", "reduction"]
for title, names, off in (("adjoint pass (PREP)", prep, 0), ("k_walker_lap", lap, 16)):
    tot = c[off:off + 10].sum()
    print(f"{title}: {tot:.0f} cycles per wave")
    for k, n in enumerate(names):
        if c[off + k] > 0:
            print(f"  {k} {n:32s} {c[off + k]:9.0f}  {100 * c[off + k] / tot:5.1f} %")
