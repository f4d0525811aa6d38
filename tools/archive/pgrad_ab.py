"""Per-walker parameter gradient (k_param_grad) timing and outputs for an A/B of two library
variants (AIQMC_LIB_VARIANT): usage python tools/pgrad_ab.py OUT.npz -> prints ms per launch
per system, saves the gradients for a cross-variant comparison (tools/pgrad_ab.py --cmp A B)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd"))

if sys.argv[1] == "--cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    for k in a.files:
        d = np.abs(a[k] - b[k]).max() / max(1e-30, np.abs(b[k]).max())
        print(f"{k}: max |a - b| / max |b| = {d:.2e}")
    sys.exit(0)

import torch
from aiqmc import systems
from aiqmc.initial_electrons_positions.init import init_electrons
from aiqmc.wavefunction_Ynlm.nn import flatten_params
B = 4096
out = {}
for name in ("Be", "C", "C_ecp", "C2_ecp", "N2"):
    s = systems.make_system(name)
    ctx = s.context(dtype=torch.float32)
    ctx.set_params(flatten_params(s.make_network().init(1)))
    pos = init_electrons(7, None, s.atoms, s.charges, s.spins, B, 1.0)[0].to("cuda", torch.float32).contiguous()
    w = torch.full((B,), 1.0 / B, device="cuda", dtype=torch.float32)
    g = ctx.logpsi_param_grad(pos, w)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(20):
        g = ctx.logpsi_param_grad(pos, w)
    ev[1].record()
    torch.cuda.synchronize()
    # per-walker rows of the first 256 walkers (both seeds: log|psi| and phase) for the comparison
    out[name] = ctx.logpsi_param_grad(pos[:256].contiguous()).double().cpu().numpy()
    out[name + "_phase"] = ctx.phase_param_grad(pos[:256].contiguous()).double().cpu().numpy()
    print(f"{name} (N={s.nelectrons}, A={s.natoms}) B={B}: logpsi_param_grad {ev[0].elapsed_time(ev[1]) / 20:.3f} ms", flush=True)
np.savez(sys.argv[1], **out)
