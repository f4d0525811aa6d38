"""Local energies (fp32 and fp64, N2, fixed init_electrons walkers) of the library variant selected by
AIQMC_LIB_VARIANT, saved for a variant-vs-variant comparison.  usage: python tools/el_dump.py OUT.npz [walkers]
python tools/el_dump.py --compare A.npz B.npz  prints the largest differences."""
import os, sys
import numpy as np

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    for k in a.files:
        x, y = a[k], b[k]
        d = np.abs(x - y)
        rel = d / np.maximum(np.abs(x), 1.0)
        print(f"{k}: max |diff| {d.max():.3e}  max rel {rel.max():.3e}  median rel {np.median(rel):.3e}  "
              f"bitwise {bool((x == y).all())}  finite {bool(np.isfinite(y).all())}")
    sys.exit(0)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd"))
import torch
from aiqmc import systems
from aiqmc.initial_electrons_positions.init import init_electrons
from aiqmc.wavefunction_Ynlm.nn import flatten_params

B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
out = {}
for name in os.environ.get("EL_SYSTEMS", "N2").split(","):
    s = systems.make_system(name)
    params = flatten_params(s.make_network().init(1))
    pos0 = init_electrons(1000, None, s.atoms, s.charges, s.spins, B, 1.0)[0]
    for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        ctx = s.context(dtype=dt)
        ctx.set_params(params)
        pos = pos0.to("cuda", dt).contiguous()
        el, logabs, grad = ctx.local_energy(pos, want_logabs=True, want_grad=True)
        torch.cuda.synchronize()
        out[f"{name}_{tag}_el"] = el.double().cpu().numpy()
        out[f"{name}_{tag}_grad"] = grad.double().cpu().numpy()
np.savez(sys.argv[1], **out)
print("saved", sys.argv[1], {k: v.shape for k, v in out.items()})
