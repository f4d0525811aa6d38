"""RCCL (torch.distributed backend "nccl") on the HIP path, and the fused multi-rank training step.

BASELINE config 4 pmeans the training statistics and the gradient over RCCL
(main_all_electrons_adam_muti_GPU.py:140-190; Loss/loss.py:107,206,208; Optimizer/adam.py:55).
The test box has one GPU, and RCCL puts one rank per device, so the RCCL tests run a ONE-rank
nccl group with the collective path forced (aiqmc.constants.force_collectives): every all-reduce
then executes in RCCL.  A one-rank sum is the identity, so the results must be BITWISE those of
the same kernels with no process group.  The two-rank Adam step runs over gloo on the one GPU
(two ranks cannot share a device in RCCL) against a single process on the concatenated batch.
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
PKG = os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _be_training(B, dtype=torch.float64, lo=0, hi=None, seed=7):
    """Be, the all-electron multi-GPU driver's loss (clip 5, centred at the clipped mean,
    complex_output) and Adam chain; walkers [lo, hi) of a B-walker init_electrons batch."""
    from oracle import system
    from aiqmc import spin_indices
    from aiqmc.Energy import hamiltonian as H
    from aiqmc.Loss import loss as L
    from aiqmc.Optimizer import adam, optax_like as optax
    from aiqmc.wavefunction_Ynlm import nn
    from aiqmc.initial_electrons_positions.init import init_electrons
    s = system.make_system("Be")
    par, anti, npar, nanti = spin_indices.jastrow_indices_ee(spins=s.spins, nelectrons=s.nelectrons)
    up, dn = spin_indices.spin_indices_h(s.spins)
    network = nn.make_ai_net(ndim=3, nelectrons=s.nelectrons, natoms=s.natoms, nspins=s.nspins, determinants=1,
                             charges=s.charges, parallel_indices=par, antiparallel_indices=anti,
                             n_parallel=npar, n_antiparallel=nanti, spin_up_indices=up, spin_down_indices=dn)
    params = system.init_params(np.random.default_rng(3), s, randomize_aux=True)
    pos, spins = init_electrons(seed, None, s.atoms, s.charges, s.spins, B, 1.0)
    pos = pos[lo:hi]
    data = nn.AINetData(positions=pos.to("cuda", dtype).contiguous(), spins=spins, atoms=s.atoms, charges=s.charges)

    def log_network(*args, **kwargs):
        phase, mag = network.apply(*args, **kwargs)
        return mag + 1.j * phase

    le = H.local_energy(f=network.apply, charges=s.charges, nspins=s.spins, use_scan=False)
    ev = L.make_loss(network=log_network, local_energy=le, clip_local_energy=5.0, clip_from_median=False,
                     center_at_clipped_energy=True, complex_output=True)
    opt = optax.chain(optax.scale_by_adam(b1=0.9, b2=0.999, eps=1e-8, eps_root=0.0),
                      optax.scale_by_schedule(lambda t: 0.05 * (1.0 / (1.0 + t)) ** 10000), optax.scale(-1.))
    step = adam.make_training_step(adam.make_opt_update_step(ev, opt))
    return s, network, params, data, ev, step, le


def _pp_training(B, dtype=torch.float64):
    """C atom ccECP with the pp drivers' loss (complex E_L, complex_output=True), B walkers."""
    from aiqmc import systems
    from aiqmc.Energy import pphamiltonian
    from aiqmc.Loss import loss as L
    from aiqmc.VMC.VMCmcstep import PhiloxKey
    from aiqmc.wavefunction_Ynlm import nn
    from aiqmc.initial_electrons_positions.init import init_electrons
    s = systems.make_system("C_ecp")
    network = s.make_network()
    params = network.init(4)
    e = systems.ccecp_tables("C_ecp")
    log_network = nn.make_log_network(network.apply)
    le = pphamiltonian.local_energy(f=network.apply, lognetwork=log_network, charges=s.charges, nspins=s.spins,
                                    rn_local=e.rn_local, local_coes=e.local_coes, local_exps=e.local_exps,
                                    rn_non_local=e.rn_non_local, non_local_coes=e.non_local_coes,
                                    non_local_exps=e.non_local_exps, natoms=1, nelectrons=4, ndim=3, list_l=2)
    ev = L.make_loss(network=log_network, local_energy=le, clip_local_energy=5.0, clip_from_median=False,
                     center_at_clipped_energy=True, complex_output=True)
    ev._aiqmc_local_energy = le
    pos, sp = init_electrons(17, None, s.atoms, s.charges, s.spins, B, 1.0)
    data = nn.AINetData(positions=pos.to("cuda", dtype).contiguous(), spins=sp, atoms=s.atoms, charges=s.charges)
    return ev, params, data, PhiloxKey(23, 5), network.apply._aiqmc_network


_RCCL_WORKER = r'''
import os, sys
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2]); sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
import numpy as np, torch, torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + sys.argv[4], rank=0, world_size=1)
assert dist.get_backend() == "nccl"
import test_gpu_rccl as T
from aiqmc import constants
from aiqmc.Loss import loss as L
from aiqmc.wavefunction_Ynlm import nn
out = {}
# 1. pmean_stats: aiqmc_energy_stats -> RCCL all-reduce -> aiqmc_energy_stats_final
e = torch.tensor(np.random.default_rng(4).normal(-109.0, 3.0, 4096), dtype=torch.float32, device="cuda")
constants.force_collectives(False)
m0, v0 = constants.pmean_stats(e)
constants.force_collectives(True)
c0 = constants.ALLREDUCE_CALLS
m1, v1 = constants.pmean_stats(e)
out["stats_calls"] = constants.ALLREDUCE_CALLS - c0
out["stats"] = np.array([float(m0), float(v0), float(m1), float(v1)])
# 2. the fused training-step levels with and without the (one-rank) RCCL group
for tag, dt in (("f64", torch.float64), ("f32", torch.float32)):
    s, network, params, data, ev, step, le = T._be_training(256, dt)
    e_l, _ = le(params, None, data)
    ctx = network.apply._aiqmc_network.bind(params, data.atoms, dt)
    x = data.positions.reshape(256, -1)
    gfn = lambda w, wp: (ctx.param_grad_weighted(x, w),
                         ctx.param_grad_weighted(x, wp[None], phase=True)[0] if wp is not None else None)
    constants.force_collectives(True)
    c0 = constants.ALLREDUCE_CALLS
    (loss1, aux1), g1 = ev.value_and_pmean_grad(params, None, data)
    out[tag + "_calls"] = constants.ALLREDUCE_CALLS - c0
    constants.force_collectives(False)
    loss2, var2, cl2, g2, _ = L.fused_levels(e_l, gfn, 5.0, True, True)
    (loss3, aux3), g3 = ev.value_and_pmean_grad(params, None, data)     # one rank: aiqmc_loss_weights
    out[tag + "_g"] = np.stack([g1.cpu().numpy(), g2.cpu().numpy(), g3.cpu().numpy()]).astype(np.float64)
    out[tag + "_loss"] = np.array([complex(loss1), complex(loss2), complex(loss3)])
    out[tag + "_var"] = np.array([float(aux1.variance), float(var2), float(aux3.variance)])
    out[tag + "_clipped"] = np.stack([aux1.clipped_energy.cpu().numpy(), cl2.cpu().numpy(),
                                      aux3.clipped_energy.cpu().numpy()]).astype(np.complex128)
    # one Adam step (make_training_step) forced over RCCL and without a group
    constants.force_collectives(True)
    c0 = constants.ALLREDUCE_CALLS
    _, p1, _, _, _ = step(data, params, None, 0)
    out[tag + "_step_calls"] = constants.ALLREDUCE_CALLS - c0
    constants.force_collectives(False)
    _, p2, _, _, _ = step(data, params, None, 0)
    out[tag + "_params"] = np.stack([nn.flatten_params(p1), nn.flatten_params(p2)])
# 3. complex local energies (C atom ccECP, complex_output=True): the phase-gradient weights too
ev, params, data, key, net = T._pp_training(128)
e_l, _ = ev._aiqmc_local_energy(params, key, data)
ctx = net.bind(params, data.atoms, torch.float64)
x = data.positions.reshape(128, -1)
gfn = lambda w, wp: (ctx.param_grad_weighted(x, w), ctx.param_grad_weighted(x, wp[None], phase=True)[0])
constants.force_collectives(True)
c0 = constants.ALLREDUCE_CALLS
(l1, a1), g1 = ev.value_and_pmean_grad(params, key, data)
out["pp_calls"] = constants.ALLREDUCE_CALLS - c0
constants.force_collectives(False)
l2, v2, c2, g2, im2 = L.fused_levels(e_l, gfn, 5.0, True, True)
(l3, a3), g3 = ev.value_and_pmean_grad(params, key, data)
out["pp_g"] = np.stack([g1.cpu().numpy(), g2.cpu().numpy(), g3.cpu().numpy()])
out["pp_loss"] = np.array([complex(l1), complex(l2), complex(l3)])
out["pp_imag"] = float(im2)
torch.cuda.synchronize()
np.savez(sys.argv[3], **out)
dist.destroy_process_group()
'''


def test_rccl_one_rank_group_is_bitwise_identity(tmp_path):
    """pmean_stats and the fused training step over a one-rank RCCL group equal the no-group
    results bitwise (the same kernels; a one-rank all-reduce is the identity); the training step
    takes exactly 3 all-reduces (statistics, TV window, clipped sums + gradient); the multi-level
    gradient agrees with the one-rank fused kernel (aiqmc_loss_weights) to rounding."""
    f = tmp_path / "rccl.npz"
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", _RCCL_WORKER, ROOT, PKG, str(f), str(_free_port())], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    o = dict(np.load(f))
    st = o["stats"]
    assert int(o["stats_calls"]) == 1
    assert st[0] == st[2] and st[1] == st[3]          # 4096 energies: n m / n == m exactly
    for tag, tol in (("f64", 1e-10), ("f32", 2e-4)):
        assert int(o[tag + "_calls"]) == 3 and int(o[tag + "_step_calls"]) == 3, tag
        g = o[tag + "_g"]
        np.testing.assert_array_equal(g[0], g[1])                         # RCCL group == no group
        scale = np.abs(g[2]).max()
        np.testing.assert_allclose(g[0], g[2], rtol=0, atol=tol * scale)  # == the one-rank kernel
        lo = o[tag + "_loss"]
        assert lo[0] == lo[1] and abs(lo[0] - lo[2]) <= 1e-12 * abs(lo[2]) * (1 if tag == "f64" else 1e5)
        v = o[tag + "_var"]
        assert v[0] == v[1] and abs(v[0] - v[2]) <= (1e-10 if tag == "f64" else 1e-4) * v[2]
        c = o[tag + "_clipped"]
        np.testing.assert_array_equal(c[0], c[1])
        np.testing.assert_allclose(c[0], c[2], rtol=1e-6 if tag == "f32" else 1e-12)
        p = o[tag + "_params"]
        if tag == "f64":
            np.testing.assert_allclose(p[0], p[1], rtol=0, atol=1e-9)
    # complex energies: phase weights in the same three all-reduces
    assert int(o["pp_calls"]) == 3 and o["pp_imag"] > 0
    g = o["pp_g"]
    np.testing.assert_array_equal(g[0], g[1])
    np.testing.assert_allclose(g[0], g[2], rtol=0, atol=1e-10 * np.abs(g[2]).max())
    lo = o["pp_loss"]
    assert lo[0] == lo[1] and abs(lo[0] - lo[2]) <= 1e-12 * abs(lo[2])


def test_bench_force_collectives_over_rccl_under_torchrun(tmp_path):
    """bench.py under torch.distributed.run --nproc-per-node 1 with --force-collectives: the VMC
    statistics all-reduce and the Be Adam side measurement's fused training step run in RCCL."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "1",
           "--force-collectives", "--dist-backend", "nccl", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
           "--no-ecp", "--no-dmc", "--no-per-rank"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path),
                         env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 1 and r["finite"]
    c = r["collectives"]
    assert c["process_group"] and c["backend"] == "nccl" and c["forced_at_world_1"]
    assert c["allreduce_calls_before_side_benches"] >= 3     # one statistics all-reduce per iteration
    a = r["adam_be_atom"]
    assert "error" not in a, a
    assert a["allreduce_calls"] == 3 * 7 and a["finite"]    # 2 warm-up + 5 timed training steps


_ADAM_WORKER = r'''
import os, sys
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2]); sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
import numpy as np, torch, torch.distributed as dist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
import test_gpu_rccl as T
from aiqmc import constants
from aiqmc.wavefunction_Ynlm import nn
B = int(sys.argv[4]); n = B // world
s, network, params, data, ev, step, le = T._be_training(B, torch.float64, rank * n, (rank + 1) * n)
c0 = constants.ALLREDUCE_CALLS
_, p1, state, loss, aux = step(data, params, None, 0)
calls = constants.ALLREDUCE_CALLS - c0
np.savez(os.path.join(sys.argv[3], f"adam{rank}.npz"), p=nn.flatten_params(p1), loss=complex(loss),
         var=float(aux.variance), calls=calls, clipped=aux.clipped_energy.cpu().numpy())
dist.barrier()
dist.destroy_process_group()
'''


@pytest.mark.parametrize("world", [2])
def test_two_rank_adam_step_equals_concatenated_batch(tmp_path, world):
    """One training step of the all-electron multi-GPU driver (Be, fp64) on two gloo ranks, each
    with a contiguous half of 128 walkers: 3 all-reduces per rank, and the parameters, loss,
    variance and clipped energies equal one process on all 128 walkers."""
    B = 128
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, "-c", _ADAM_WORKER, ROOT, PKG, str(tmp_path), str(B)], env=env))
    for p in procs:
        assert p.wait(timeout=240) == 0
    from aiqmc.wavefunction_Ynlm import nn
    s, network, params, data, ev, step, le = _be_training(B, torch.float64)
    _, p_ref, _, loss_ref, aux_ref = step(data, params, None, 0)
    p_ref = nn.flatten_params(p_ref)
    cl_ref = aux_ref.clipped_energy.cpu().numpy()
    n = B // world
    for r in range(world):
        o = dict(np.load(tmp_path / f"adam{r}.npz"))
        assert int(o["calls"]) == 3
        assert abs(complex(o["loss"]) - complex(loss_ref)) <= 1e-12 * abs(complex(loss_ref))
        assert abs(float(o["var"]) - float(aux_ref.variance)) <= 1e-10 * float(aux_ref.variance)
        np.testing.assert_allclose(o["clipped"], cl_ref[r * n:(r + 1) * n], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(o["p"], p_ref, rtol=0, atol=1e-9)


def test_complex_energies_need_complex_output_checked_after_the_step():
    """Complex local energies with complex_output=False are the reference's error (loss.py:256-265).
    The check is a device count carried in aux (no host read inside the loss) and raised by
    make_training_step after its NaN test."""
    from aiqmc.Loss import loss as L
    from aiqmc.Optimizer import adam, optax_like as optax
    ev, params, data, key, net = _pp_training(32)
    le = ev._aiqmc_local_energy
    bad = L.make_loss(network=le, local_energy=le,
                      clip_local_energy=5.0, clip_from_median=False, center_at_clipped_energy=True,
                      complex_output=False)
    (loss, aux), g = bad.value_and_pmean_grad(params, key, data)
    assert aux.imag_check is not None and int(aux.imag_check) > 0
    opt = optax.chain(optax.scale_by_adam(b1=0.9, b2=0.999, eps=1e-8, eps_root=0.0), optax.scale(-1.))
    step = adam.make_training_step(adam.make_opt_update_step(bad, opt))
    with pytest.raises(NotImplementedError):
        step(data, params, None, key)
