"""pp local energy and T-moves of the ccECP example systems on one library (AIQMC_LIB_VARIANT):
outputs saved for a bitwise comparison between libraries, and ms per call (4096 walkers, fp32).
usage: python tools/ecp_tm_ab.py out.npz   (ECP_SYSTEMS="C_ecp C2_ecp" restricts the systems)"""
import json, os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd"))
from aiqmc import systems  # noqa: E402
from aiqmc.initial_electrons_positions.init import init_electrons  # noqa: E402
from aiqmc.wavefunction_Ynlm.nn import flatten_params  # noqa: E402

out, res = {}, {}
for name in os.environ.get("ECP_SYSTEMS", "C_ecp C2_ecp CO2_ecp").split():
    for dt in (torch.float32, torch.float64):
        s = systems.make_system(name)
        ctx = s.context(dtype=dt)
        ctx.set_params(flatten_params(s.make_network().init(1)))
        e = systems.ccecp_tables(name)
        ctx.set_ecp(e.rn_local, e.local_coes, e.local_exps, e.rn_non_local, e.non_local_coes, e.non_local_exps, e.list_l)
        B = 4096 if dt == torch.float32 else 256
        pos = init_electrons(7, None, s.atoms, s.charges, s.spins, B, 1.0)[0].to("cuda", dt).contiguous()
        tag = f"{name}_{'f32' if dt == torch.float32 else 'f64'}"
        el = ctx.local_energy_ecp(pos, seed=3, offset=0)
        p2 = pos.clone()
        acc = ctx.dmc_tmoves(p2, 0.01, seed=5, offset=0)
        torch.cuda.synchronize()
        out[tag + "_el"] = torch.view_as_real(el).cpu().numpy() if torch.is_complex(el) else el.cpu().numpy()
        out[tag + "_tm_pos"] = p2.cpu().numpy()
        out[tag + "_tm_acc"] = acc.cpu().numpy()
        if dt == torch.float32:
            t0 = time.perf_counter()
            for k in range(5):
                ctx.local_energy_ecp(pos, seed=3, offset=1 + k)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for k in range(5):
                ctx.dmc_tmoves(p2, 0.01, seed=5, offset=1 + k)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            res[name] = {"pp_el_ms": round(1e3 * (t1 - t0) / 5, 4), "tmoves_ms": round(1e3 * (t2 - t1) / 5, 4)}
np.savez(sys.argv[1], **out)
print(json.dumps(res))
