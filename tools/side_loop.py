"""The bench's side measurements alone (BASELINE configs 2, 3 and 5, and the reference's C2 ccECP
example), for rocprofv3 kernel-trace and PMC passes: python tools/side_loop.py [which ...]
which: ecp_c (C atom ccECP E_L), ecp_c2 (C2 ccECP E_L), adam_be (Be Adam iteration),
dmc_ne (Ne all-electron DMC step), dmc_c (C atom ccECP DMC step).  Default: all five.
Each runs the same function bench.py runs, with the same walkers, steps and seeds."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

which = sys.argv[1:] or ["ecp_c", "ecp_c2", "adam_be", "dmc_ne", "dmc_c"]
dev = torch.device("cuda", 0)
dt = torch.float32
for w in which:
    if w == "ecp_c":
        r = bench.ecp_side_bench(dt, dev, 4096, 5, False)
    elif w == "ecp_c2":
        r = bench.ecp_side_bench(dt, dev, 4096, 3, False, name="C2_ecp")
    elif w == "adam_be":
        r = bench.adam_side_bench(dt, dev, 4096, 5)
    elif w == "dmc_ne":
        r = bench.dmc_side_bench(dt, dev, 4096, 5, system="Ne")
    elif w == "dmc_c":
        r = bench.dmc_side_bench(dt, dev, 4096, 5)
    else:
        raise SystemExit(f"unknown side measurement {w}")
    torch.cuda.synchronize()
    print(w, {k: v for k, v in r.items() if not isinstance(v, dict)}, flush=True)
