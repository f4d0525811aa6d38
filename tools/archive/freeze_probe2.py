"""Diagnostic follow-up of tools/freeze_probe.py: replay the frozen walker with host draws in fp32
under each mc_step switch, and evaluate its 14 proposal configurations with logpsi_grad."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
sys.path.insert(0, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd")
from test_gpu_fp32_statistics import _ctx, TSTEP

d = np.load("tests/golden/N2_fp32_far_electron.npz")
b = int(d["cul"][0])
x0 = d["frozen"][b:b + 1]
g1, g2, u = (torch.tensor(d[k]) for k in ("g1", "g2", "u"))
N = 14
for label, setup in [("default", lambda c: None), ("reuse0", lambda c: c.set_proposal_reuse(False)),
                     ("fuse_reduce3", lambda c: c.set_fuse_reduce(3)), ("pivots0", lambda c: c.set_walker_pivots(False)),
                     ("fuse_accept0", lambda c: c.set_fuse_accept(False))]:
    s, c = _ctx("N2", torch.float32)
    setup(c)
    p = torch.tensor(x0, device="cuda").contiguous()
    acc = c.mc_step(p, 1, TSTEP, gauss1=g1, gauss2=g2, u=u, count_accepts=True)
    print(label, "accepts", int(acc.sum()), flush=True)
s, c = _ctx("N2", torch.float32)
_, c64 = _ctx("N2", torch.float64)
x = torch.tensor(x0, device="cuda")
la, g = c.logpsi_grad(x)
la64, g64 = c64.logpsi_grad(x.double())
te = 0.05 * 0  # drift is applied inside mc_step; here only the moved-electron configurations matter
v2 = float((g.double() ** 2).sum())
f = (np.sqrt(1 + 2 * TSTEP * 0.25 * v2) - 1) / (0.25 * v2)
step = (g.double() * f * TSTEP + np.sqrt(TSTEP) * g1[0].double().cuda()).reshape(N, 3)
xs = x.double().reshape(1, N, 3).repeat(N, 1, 1)
xs[torch.arange(N), torch.arange(N)] += step
xs = xs.reshape(N, 3 * N)
l32, gg32 = c.logpsi_grad(xs.float().contiguous())
l64, gg64 = c64.logpsi_grad(xs.contiguous())
print("proposal logabs fp32", l32.cpu().numpy().round(3).tolist(), flush=True)
print("proposal logabs fp64", l64.cpu().numpy().round(3).tolist(), flush=True)
print("proposal |g|^2 fp32", (gg32.double() ** 2).sum(1).cpu().numpy().tolist(), flush=True)
print("proposal |g|^2 fp64", (gg64 ** 2).sum(1).cpu().numpy().tolist(), flush=True)
lf, gf = c.logpsi_grad_forward_mode(xs.float().contiguous())
print("forward-mode fp32 logabs", lf.cpu().numpy().round(3).tolist(), "|g|^2", (gf.double() ** 2).sum(1).cpu().numpy().tolist(), flush=True)
