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


def _block(rank, world, b_total=B_TOTAL):
    from aiqmc import systems
    from aiqmc.initial_electrons_positions.init import init_electrons
    s = systems.make_system("N2")
    pos, _ = init_electrons(2024, None, s.atoms, s.charges, s.spins, b_total, 1.0)
    n = b_total // world
    return s, pos[rank * n:(rank + 1) * n]


def _run_block(rank, world, b_total=B_TOTAL):
    """mc_step + local_energy on this rank's block (fp32, Philox stream seed 77 + rank)."""
    from aiqmc import systems
    s, pos = _block(rank, world, b_total)
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
x, el = T._run_block(rank, world, int(sys.argv[3]))
mean, var = constants.pmean_stats(el.cpu())
# the device path INTEGRATION.md advertises: aiqmc_energy_stats(finalize=False) -> all_reduce of the
# rank's 4-vector -> aiqmc_energy_stats_final (gloo all-reduces the CUDA tensor here, RCCL on a node)
mean_d, var_d = constants.pmean_stats(el)
np.savez(os.path.join(sys.argv[2], f"rank{rank}.npz"), x=x.cpu().numpy(), el=el.cpu().numpy(),
         mean=mean.numpy(), var=var.numpy(), mean_d=mean_d.cpu().numpy(), var_d=var_d.cpu().numpy())
dist.barrier()
dist.destroy_process_group()
'''


@pytest.mark.parametrize("world,b_total", [(2, B_TOTAL), (8, 32768)])
def test_two_rank_blocks_equal_single_process(tmp_path, world, b_total):
    """(8, 32768): BASELINE config 4's walker count sharded 8 ways (4,096 per rank; the reference's
    KFAC leg is out of scope), eight gloo ranks on the one test GPU."""
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, "-c", _WORKER, ROOT, str(tmp_path), str(b_total)], env=env))
    for p in procs:
        assert p.wait(timeout=240) == 0
    outs = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)]
    from aiqmc import constants
    els = []
    for r in range(world):
        x, el = _run_block(r, world, b_total)
        np.testing.assert_array_equal(outs[r]["x"], x.cpu().numpy())
        np.testing.assert_array_equal(outs[r]["el"], el.cpu().numpy())
        els.append(el.cpu())
    mean, var = constants.pmean_stats(torch.cat(els))        # single process: identity collective
    for r in range(world):
        for mk, vk in (("mean", "var"), ("mean_d", "var_d")):   # host path, device-kernel path
            assert abs(float(outs[r][mk]) - float(mean)) <= 1e-12 * abs(float(mean)), mk
            assert abs(float(outs[r][vk]) - float(var)) <= 1e-10 * abs(float(var)), vk
    # the reference's two-pass statistics (loss.py:206-208) on the concatenation, float64
    e = torch.cat(els).double().numpy()
    assert abs(float(mean) - e.mean()) <= 1e-9 * abs(e.mean())
    assert abs(float(var) - np.mean(np.abs(e - e.mean()) ** 2)) <= 1e-9 * np.var(e)


def _bench_two_ranks(tmp_path, extra, n=2):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps",
           "2", "--warmup", "1", "--no-cpu-baseline", "--no-ecp", "--no-adam", "--no-dmc",
           "--dist-backend", "gloo"] + extra
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path),
                         env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_bench_two_ranks_under_torchrun(tmp_path):
    """The driver's multi-GPU launch line with two ranks on the one test GPU (gloo).  Default =
    SURVEY 8(d)'s strong scaling: --global-walkers in total split over the ranks (here 1024 ->
    512 per rank), with the weak-scaling run (--walkers per rank) beside it."""
    r = _bench_two_ranks(tmp_path, ["--global-walkers", "1024", "--walkers", "256"])
    assert r["n_gpus"] == 2 and r["scaling"] == "strong" and r["finite"]
    assert r["config"]["global_walkers"] == 1024 and r["config"]["walkers_per_gpu"] == 512
    assert r["value"] > 0 and r["roofline"]["avg_launch_ms"] > 0
    w = r["weak_scaling"]
    assert w["walkers_per_gpu"] == 256 and w["global_walkers"] == 512 and w["value"] > 0 and w["finite"]


def test_bench_eight_ranks_under_torchrun(tmp_path):
    """The driver's N = 8 launch line (gloo rehearsal, eight ranks on the one test GPU): the
    default strong scaling splits BASELINE's 4,096 walkers into 512 per rank."""
    r = _bench_two_ranks(tmp_path, [], n=8)
    assert r["n_gpus"] == 8 and r["scaling"] == "strong" and r["finite"]
    assert r["config"]["global_walkers"] == 4096 and r["config"]["walkers_per_gpu"] == 512
    assert r["value"] > 0 and r["weak_scaling"]["walkers_per_gpu"] == 4096


def test_bench_two_ranks_weak_headline(tmp_path):
    r = _bench_two_ranks(tmp_path, ["--weak", "--walkers", "512"])
    assert r["scaling"] == "weak" and r["config"]["global_walkers"] == 1024 and "weak_scaling" not in r
    assert r["value"] > 0 and r["finite"]


def test_bench_gpus_flag_spawns_ranks_without_launcher(tmp_path):
    """``python bench.py --gpus 2`` with NO launcher (the form the driver's BENCH line uses): bench.py
    must start the two ranks itself (torch.distributed.run as a child, before any GPU call) and relay
    rank 0's line -- not silently run one rank."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--steps", "2",
           "--warmup", "1", "--no-ecp", "--no-adam", "--no-dmc", "--no-cpu-baseline", "--global-walkers", "1024",
           "--walkers", "256"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path),
                         env=dict(env, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["scaling"] == "strong" and r["finite"]
    assert r["config"]["walkers_per_gpu"] == 512 and r["config"]["global_walkers"] == 1024
    assert r["weak_scaling"]["walkers_per_gpu"] == 256 and r["weak_scaling"]["global_walkers"] == 512


_DMC_WORKER = r'''
import os, sys
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, os.path.join(sys.argv[1], "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd"))
sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
import numpy as np, torch, torch.distributed as dist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
import test_gpu_sharded as T
out = T._dmc_rank(rank, world, sys.argv[3])
np.savez(os.path.join(sys.argv[2], f"dmc{rank}.npz"), **out)
dist.barrier()
dist.destroy_process_group()
'''


def _dmc_rank(rank, world, fixture):
    """This rank's block of the 2-device DMC fixture through aiqmc.DMC.main_dmc.dmc_blocks."""
    from oracle import system
    from aiqmc import systems
    from aiqmc.DMC import dmc, main_dmc
    from aiqmc.DMC.Tmoves import HostTmoveDraws
    from aiqmc.VMC.VMCmcstep import HostDraws
    from aiqmc.wavefunction_Ynlm import nn
    g = dict(np.load(fixture))
    sysname = "Ne" if os.path.basename(fixture).startswith("Ne_") else "C_ecp"
    s = systems.make_system(sysname)
    N, A = s.nelectrons, s.natoms
    network = s.make_network()
    params = system.unflatten_params(system.init_params(np.random.default_rng(0), system.make_system(sysname)),
                                     g["params_flat"])
    from oracle import pphamiltonian as opp
    if sysname == "Ne":      # all-electron Ne through the pp-only DMC step (make_golden_dmc.TABLES)
        e = opp.ECP([[1.0]], [[0.0]], [[1.0]], [[[2.0], [2.0], [2.0]]], [[[0.0], [0.0], [0.0]]],
                    [[[1.0], [1.0], [1.0]]], 2)
    else:
        e = opp.ECP([[1.0]], [[0.0]], [[1.0]], [[[2.0], [1.0]]], [[[-3.0], [-5.0]]], [[[0.7], [0.4]]], 1)
    B = g["x0"].shape[0]
    Bd = B // world
    sl = slice(rank * Bd, (rank + 1) * Bd)
    nblocks, iters = g["newinds"].shape[0], g["weights"].shape[0] // g["newinds"].shape[0]
    tstep = float(g["tstep"])
    run = dmc.dmc_propagate(network.apply, nn.make_log_network(network.apply), network.apply, e.list_l, N, A, 3, Bd,
                            tstep, 1, s.charges, s.spins, e.rn_local, e.local_coes, e.local_exps, e.rn_non_local,
                            e.non_local_coes, e.non_local_exps)
    ctx = network.apply._aiqmc_network.bind(params, s.atoms, torch.float64)
    data = nn.AINetData(positions=torch.tensor(g["x0"][sl], device="cuda").contiguous(), spins=s.spins,
                        atoms=s.atoms, charges=s.charges)
    e_all = torch.complex(torch.tensor(g["e_l0_re"]), torch.tensor(g["e_l0_im"]))
    d0 = e_all - e_all.mean()
    var0 = (d0 * d0.conj()).mean().cuda()                      # total_e's pmean'd variance (global)
    e_l0 = e_all[sl].cuda()
    step_key = lambda k: dmc.HostDmcDraws(
        HostTmoveDraws(torch.tensor(g["rot_tm"][k][sl]), torch.tensor(g["u_sel"][k][sl]), torch.tensor(g["u_acc"][k][sl])),
        HostDraws(torch.tensor(g["gauss1"][k][sl]), torch.tensor(g["gauss2"][k][sl]), torch.tensor(g["u"][k][sl])),
        torch.tensor(g["rot_old"][k][sl]), torch.tensor(g["rot_new"][k][sl]))
    block_draws = lambda b: (float(g["u_comb"][b, rank]), torch.tensor(g["extra"][b, rank]))
    est, data, w, trace = main_dmc.dmc_blocks(run, ctx, params, data, e_l0, var0, nblocks, iters, float(g["feedback"]),
                                              step_key, block_draws, trace=True)
    torch.cuda.synchronize()
    return dict(positions=np.stack([p.cpu().numpy() for p in trace["positions"]]),
                energy=np.stack([x.real.cpu().numpy() for x in trace["energy"]]),
                weights=np.stack([x.cpu().numpy() for x in trace["weights"]]),
                newinds=np.stack([x.cpu().numpy() for x in trace["newinds"]]),
                comb_weight=np.array(trace["comb_weight"]), e_est=np.array(est), e_trial=np.array(trace["e_trial"]),
                x_final=data.positions.cpu().numpy())


@pytest.mark.parametrize("fixture_name", ["C_dmc_attractive_2dev.npz", "Ne_dmc_ne_allelectron_2dev.npz"])
def test_two_rank_dmc_driver_matches_two_device_oracle(tmp_path, golden_dir, fixture_name):
    """main_dmc.dmc_blocks on two ranks (gloo, one GPU), 4 walkers each, every draw injected, vs
    the oracle's two-device driver (oracle.dmc.dmc_blocks_devices, C_dmc_attractive_2dev.npz):
    per-rank T-moves / drift-diffusion / comb, the comput_S cut as ONE minimum over both ranks
    (MIN all-reduce), the global block estimate and the e_trial feedback from the mean of the two
    ranks' comb weights.  Positions 1e-9, weights 1e-12 relative, comb indices exact.  Also
    all-electron Ne (BASELINE config 5, Ne_dmc_ne_allelectron_2dev.npz), 2 walkers per rank."""
    world = 2
    fixture = os.path.join(golden_dir, fixture_name)
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, "-c", _DMC_WORKER, ROOT, str(tmp_path), fixture], env=env))
    for p in procs:
        assert p.wait(timeout=240) == 0
    g = dict(np.load(fixture))
    B = g["x0"].shape[0]
    Bd = B // world
    for r in range(world):
        o = dict(np.load(tmp_path / f"dmc{r}.npz"))
        sl = slice(r * Bd, (r + 1) * Bd)
        np.testing.assert_allclose(o["positions"], g["positions"][:, sl], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(o["energy"], g["energy_re"][:, sl], rtol=0, atol=1e-6)
        np.testing.assert_allclose(o["weights"], g["weights"][:, sl], rtol=1e-12)
        np.testing.assert_array_equal(o["newinds"], g["newinds"][:, r])
        np.testing.assert_allclose(o["comb_weight"], g["comb_weight"][:, r], rtol=1e-12)
        np.testing.assert_allclose(o["e_est"], g["e_est"], rtol=0, atol=1e-9)
        np.testing.assert_allclose(o["e_trial"], g["e_trial"], rtol=0, atol=1e-9)
        np.testing.assert_allclose(o["x_final"], g["x_final"][sl], rtol=1e-9, atol=1e-9)
