"""Walker-sharded multi-process runs on the HIP path.

The reference shards walkers over devices in contiguous blocks (main_all_electrons_adam_muti_GPU
.py:86-97), runs mc_step per device with no collective (:140; limdrift's v2 is a per-device sum,
Q8) and pmeans the energy statistics (loss.py:206-208).  Here two processes share the one GPU
of the test box over gloo (RCCL cannot put two ranks on one device); each owns a contiguous
2048-walker block of the 4096-walker N2 batch and runs mc_step (Philox, the rank's own stream) +
local_energy + pmean_stats.  Each rank's positions and E_L must be BITWISE equal to a
single-process run of the same block with the same draws, and the pooled statistics must equal
the single-process statistics of the concatenation.  A second test runs bench.py itself under
torch.distributed.run with two ranks (the driver's multi-GPU launch line, gloo rehearsal).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B_TOTAL, NSTEPS, TSTEP = 4096, 3, 0.05


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _block(rank, world):
    from aiqmc import systems
    from aiqmc.initial_electrons_positions.init import init_electrons
    s = systems.make_system("N2")
    pos, _ = init_electrons(2024, None, s.atoms, s.charges, s.spins, B_TOTAL, 1.0)
    n = B_TOTAL // world
    return s, pos[rank * n:(rank + 1) * n]


def _run_block(rank, world):
    """mc_step + local_energy on this rank's block (fp32, Philox stream seed 77 + rank)."""
    from aiqmc import systems
    s, pos = _block(rank, world)
    ctx = s.context(dtype=torch.float32)
    net = s.make_network()
    ctx.set_params(__import__("aiqmc.wavefunction_Ynlm.nn", fromlist=["flatten_params"]).flatten_params(net.init(9)))
    x = pos.to("cuda", torch.float32).contiguous()
    ctx.mc_step(x, NSTEPS, TSTEP, seed=77 + rank, offset=5)
    el, _, _ = ctx.local_energy(x)
    torch.cuda.synchronize()
    return x, el


_WORKER = r'''
import os, sys
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, os.path.join(sys.argv[1], "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd"))
sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
import numpy as np, torch, torch.distributed as dist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
import test_gpu_sharded as T
from aiqmc import constants
x, el = T._run_block(rank, world)
mean, var = constants.pmean_stats(el.cpu())
np.savez(os.path.join(sys.argv[2], f"rank{rank}.npz"), x=x.cpu().numpy(), el=el.cpu().numpy(),
         mean=mean.numpy(), var=var.numpy())
dist.barrier()
dist.destroy_process_group()
'''


def test_two_rank_blocks_equal_single_process(tmp_path):
    world = 2
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, "-c", _WORKER, ROOT, str(tmp_path)], env=env))
    for p in procs:
        assert p.wait(timeout=240) == 0
    outs = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)]
    from aiqmc import constants
    els = []
    for r in range(world):
        x, el = _run_block(r, world)
        np.testing.assert_array_equal(outs[r]["x"], x.cpu().numpy())
        np.testing.assert_array_equal(outs[r]["el"], el.cpu().numpy())
        els.append(el.cpu())
    mean, var = constants.pmean_stats(torch.cat(els))        # single process: identity collective
    for r in range(world):
        assert abs(float(outs[r]["mean"]) - float(mean)) <= 1e-12 * abs(float(mean))
        assert abs(float(outs[r]["var"]) - float(var)) <= 1e-10 * abs(float(var))
    # the reference's two-pass statistics (loss.py:206-208) on the concatenation, float64
    e = torch.cat(els).double().numpy()
    assert abs(float(mean) - e.mean()) <= 1e-9 * abs(e.mean())
    assert abs(float(var) - np.mean(np.abs(e - e.mean()) ** 2)) <= 1e-9 * np.var(e)


def test_bench_two_ranks_under_torchrun(tmp_path):
    """The driver's multi-GPU launch line with two ranks on the one test GPU (gloo): one JSON
    line from rank 0 with n_gpus = 2 and the whole-job walker count."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
           "2", "--warmup", "1", "--walkers", "512", "--no-cpu-baseline", "--no-ecp", "--no-adam", "--no-dmc",
           "--dist-backend", "gloo"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path),
                         env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["global_walkers"] == 1024 and r["finite"]
    assert r["value"] > 0
