#!/usr/bin/env python3
"""VMC inner-loop benchmark: N2 (14 e-), 4096 walkers per GPU, MI355X.

One benchmark "step" = one VMC iteration of the reference driver's sampling
loop (main_all_electrons_adam_muti_GPU.py:177-197 / VMC/VMCmain.py:83-91):
  mc_step with nsteps drift-diffusion Metropolis sweeps (VMCmcstep.py:121-140),
  local energy of every walker (hamiltonian.local_energy, complex_output=False),
  energy statistics pmean (loss.py:206-208) as ONE all-reduce over RCCL.
Walkers are sharded in contiguous blocks; only the statistics cross ranks.  With N > 1 ranks
the headline is SURVEY 8(d)'s strong-scaling curve: 4096 walkers IN TOTAL (512 per GPU at
N = 8); a weak-scaling run at 4096 walkers per GPU is reported beside it (``weak_scaling``).
``--weak`` makes the weak run the headline.  With N = 1 both are the same 4096-walker run, and
``strong_scaling_per_rank`` times the per-rank workloads of N = 2, 4, 8 (2048/1024/512
walkers) on the one GPU.

Usage: python bench.py [--gpus N --steps K --warmup W].  With N > 1 and no launcher, bench.py
starts the N ranks itself (torch.distributed.run as a child process, before any GPU call) and
relays rank 0's line; under an external launcher
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W
each rank runs directly (a WORLD_SIZE different from --gpus is an error).
Rank 0 prints one JSON line.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd")
sys.path.insert(0, PKG)

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]

# Algorithmic FLOP model of SURVEY.md 8(d) (N2, hand-counted from the nn.py layer dims)
F_FWD_N2 = 4.9e4                 # one wavefunction forward, FLOP/config
F_VG_N2 = 3 * F_FWD_N2           # value + gradient (bwd ~ 2x fwd), FLOP/config
F_MC_N2 = 2.2e6                  # one walker-step = (N+1) value+gradient passes
F_EL_N2 = 2.55e6                 # one local-energy evaluation
PEAK_FP32_TFLOPS = 157.3         # MI355X FP32 vector peak (MI355X_MICROARCH.md)
PEAK_FP64_TFLOPS = 78.6          # FP64 vector peak (spec)
PEAK_HBM_GBS = 8000.0


# General algorithmic FLOP model of one wavefunction forward for N electrons, A atoms (the side
# configurations' rooflines; DESIGN.md 5, "FLOP models"), hand-counted from nn.py / Jastrow.py /
# envelope.py with an FMA = 2 FLOP and a transcendental = 1:
#   ae / ee features 9NA + 9N^2, Ylm terms and their means 86NA, Ylm stream N(48A + 240),
#   Yt = y W^ 12N^2, h stream: per electron 65A + 292 (three conv + single layers with their group
#   means), pair stream 108N^2, Phi 18N^2, envelope 20NA, Jastrows 2N^2 + 8NA, M = Phi Yt e^J 4N^2,
#   complex LU (8/3)N^3  ->  F_fwd = 236NA + 532N + 153N^2 + (8/3)N^3.
# For N2 it gives 5.14e4 against SURVEY 8(d)'s hand count 4.9e4; the headline keeps SURVEY's
# constants (F_FWD_N2, F_EL_N2) so that its fraction stays comparable across rounds.
def f_fwd(n, a):
    return 236.0 * n * a + 532.0 * n + 153.0 * n * n + 8.0 / 3.0 * n ** 3


def f_el(n, a):
    """SURVEY 8(d)'s local-energy model on f_fwd: (F_fwd - F_LU)(3N + 2) + 16N^3 + 3N (8N^3 + 8N^2)."""
    k = 3 * n
    return (f_fwd(n, a) - 8.0 / 3.0 * n ** 3) * (k + 2) + 16.0 * n ** 3 + k * 8.0 * n ** 3 + k * 8.0 * n * n


def load_pmc_side(lib_sha):
    """Per-launch HBM bytes of the side configurations' dominant kernels (tools/gpu_side_prof.sh ->
    profiles/pmc_side_rNN.json), used only when taken on THIS library build."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_side_r[0-9][0-9].json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("lib_sha16") == lib_sha:
            d["pmc_file"] = os.path.relpath(f, ROOT)
            return d
    return None


def side_roofline(kernel, flop_per_launch, avg_ms, launches, flop_model, pmc_side, side, peak=None, note=None):
    """A roofline object for a side configuration's dominant kernel (fp32 VALU bound, as the headline)."""
    peak = peak or PEAK_FP32_TFLOPS
    achieved = flop_per_launch / (avg_ms * 1e-3) / 1e12 if avg_ms else None
    rec = (pmc_side or {}).get("sides", {}).get(side) or {}
    traffic = rec.get("hbm_bytes_per_launch")
    out = {"kernel": kernel, "bound": "valu", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
           "frac": achieved / peak if achieved else None, "traffic": traffic,
           "hbm_gbs": traffic / (avg_ms * 1e-3) / 1e9 if (traffic and avg_ms) else None,
           "avg_launch_ms": avg_ms, "launches": launches, "flop_per_launch": flop_per_launch,
           "flop_model": flop_model, "pmc_file": (pmc_side or {}).get("pmc_file"),
           "pmc_null_reason": None if traffic else "no profiles/pmc_side_rNN.json taken on this library build"}
    if note:
        out["note"] = note
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--walkers", type=int, default=4096, help="walkers per GPU of a weak-scaling run")
    ap.add_argument("--global-walkers", type=int, default=4096,
                    help="strong scaling: this many walkers in total, split over the ranks (SURVEY 8(d): 4096)")
    ap.add_argument("--weak", action="store_true",
                    help="headline = weak scaling (--walkers per GPU) instead of SURVEY 8(d)'s 4096 in total")
    ap.add_argument("--no-per-rank", action="store_true",
                    help="N=1: skip timing the 2048/1024/512-walker per-rank workloads of N=2/4/8")
    ap.add_argument("--nsteps", type=int, default=10, help="Metropolis sweeps per iteration")
    ap.add_argument("--tstep", type=float, default=0.05)
    ap.add_argument("--dtype", choices=["f32", "f64"], default="f32")
    ap.add_argument("--system", default="N2")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-walkers", type=int, default=256, help="SURVEY 8(d): 256 walkers")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) or gloo (rehearsal)")
    ap.add_argument("--force-collectives", action="store_true",
                    help="keep a process group (and every all-reduce) at --gpus 1: the statistics and the "
                         "fused training-step all-reduces run over --dist-backend on a one-rank group")
    ap.add_argument("--no-ecp", action="store_true", help="skip the C-atom ccECP local-energy side measurement")
    ap.add_argument("--no-adam", action="store_true", help="skip the Be-atom Adam training-step side measurement")
    ap.add_argument("--no-dmc", action="store_true", help="skip the C-atom DMC side measurement")
    return ap.parse_args()


def build(name, dtype, device):
    from aiqmc import systems
    s = systems.make_system(name)
    network = s.make_network()
    params = network.init(1)
    net = network.apply._aiqmc_network
    ctx = net.bind(params, s.atoms, dtype, device)
    return s.atoms, s.charges, s.spins, network, params, ctx


def host_cpu_info():
    """The host this runs on: machine CPUs, the CPUs this process may use (affinity and cgroup
    quota), and the CPU model from /proc/cpuinfo."""
    machine = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = machine
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = min(affinity, quota) if quota else affinity
    return {"machine_cpus": machine, "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "usable_cpus": usable, "model": model}


def cpu_baseline(name, params, atoms, charges, nsteps_unused, tstep, sample_walkers):
    """Time the float64 oracle (reference algorithms) on host cores on a bounded sample, with
    every CPU this process may use (affinity / cgroup quota: os.cpu_count() on the GPU box is
    the whole machine, of which a one-GPU job gets a share)."""
    sys.path.insert(0, ROOT)
    from oracle import hamiltonian, mcstep, network, system
    host = host_cpu_info()
    threads = host["usable_cpus"]
    torch.set_num_threads(threads)
    s = system.make_system(name)
    net = network.Network(s)
    pt = network.to_torch(params)
    rng = np.random.default_rng(5)
    B = sample_walkers
    N = s.nelectrons
    x = torch.tensor(system.init_electrons(rng, s.atoms, s.charges, B, 1.0))
    g1 = torch.tensor(rng.standard_normal((B, 3 * N)))
    g2 = torch.tensor(rng.standard_normal((B, N, 3 * N)))
    u = torch.tensor(rng.uniform(size=(B, N)))
    # time-bounded sample (~10 s per leg): whole sweeps of B walkers until the leg has run >= target s
    target = 10.0
    t_mc, n_mc = 0.0, 0
    while t_mc < target:
        t0 = time.perf_counter()
        mcstep.walkers_update(net, pt, x, g1, g2, u, tstep)
        t_mc += time.perf_counter() - t0
        n_mc += B
    be = 8
    t_el, n_el = 0.0, 0
    while t_el < target:
        t0 = time.perf_counter()
        hamiltonian.batch_local_energy(net, pt, x[:be])
        t_el += time.perf_counter() - t0
        n_el += be
    return {
        "value": n_mc / t_mc, "unit": "walker*steps/s", "cores": threads, "kind": "port",
        "local_energy_evals_per_s": n_el / t_el, "host": host, "torch_threads": torch.get_num_threads(),
        "sample": f"float64 oracle (torch CPU, jvp-of-grad Laplacian, per-electron-config MH) on {name}: "
                  f"{n_mc // B} Metropolis sweeps of {B} walkers ({t_mc:.1f}s) + local energy of {n_el} "
                  f"walkers in batches of {be} ({t_el:.1f}s); {threads} threads = the CPUs usable by this "
                  f"process ({host['machine_cpus']} on the machine, model {host['model']})",
    }


def ecp_side_bench(dtype, device, walkers, steps, cpu_baseline_on, name="C_ecp", pmc_side=None):
    """BASELINE.json config 'C atom with ccECP pseudopotential, 4096 walkers, 1xMI355X': complex
    pp local energy (pphamiltonian.py:177-188) of the whole batch, Philox grid rotations.
    name="C2_ecp": the reference's example/C2 (8 pseudo-valence electrons, two atoms)."""
    from aiqmc import _lib, systems
    from aiqmc.initial_electrons_positions.init import init_electrons
    from aiqmc.wavefunction_Ynlm.nn import flatten_params
    s = systems.make_system(name)
    ctx = s.context(dtype=dtype, device=device.index)
    params = s.make_network().init(1)
    ctx.set_params(flatten_params(params))
    e = systems.ccecp_tables(name)
    ctx.set_ecp(e.rn_local, e.local_coes, e.local_exps, e.rn_non_local, e.non_local_coes, e.non_local_exps, e.list_l)
    pos, _ = init_electrons(77, None, s.atoms, s.charges, s.spins, walkers, 1.0)
    pos = pos.to(device, dtype).contiguous()
    for k in range(2):
        ctx.local_energy_ecp(pos, seed=3, offset=k)
    torch.cuda.synchronize()
    ctx.profile(True)
    t0 = time.perf_counter()
    for k in range(steps):
        out = ctx.local_energy_ecp(pos, seed=3, offset=100 + k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ctx.profile(False)
    q_ms, q_n = ctx.profile_read(_lib.PROF_ECP_QUAD)
    nq = walkers * s.nelectrons * s.natoms * _lib.ECP_NQ
    cfg = ("C atom ccECP (Z_eff=4, 4 e-, list_l=2)" if name == "C_ecp" else
           f"{name}: {s.nelectrons} e-, {s.natoms} atoms, ccECP") + ", complex E_L incl. 50-point nonlocal quadrature"
    N, A = s.nelectrons, s.natoms
    qavg = q_ms / max(q_n, 1)
    res = {"config": cfg,
           "walkers": walkers, "local_energy_evals_per_s": walkers * steps / dt, "ms_per_eval_batch": 1e3 * dt / steps,
           "quadrature_configs_per_launch": nq, "quadrature_launch_avg_ms": qavg,
           "mean_energy_re": float(out.real.mean()), "finite": bool(torch.isfinite(out.real).all()),
           # the quadrature's value-only forwards of the displaced configurations (pseudopotential.py:
           # 298-314 evaluates the network at every point; the kernel reuses the walker's cache)
           "roofline": side_roofline(f"k_quad_value<float,{N},{A}> (value-only quadrature configurations)",
                                     nq * f_fwd(N, A), qavg, q_n, f"configs x F_fwd({N},{A}) = {nq} x {f_fwd(N, A):.0f}",
                                     pmc_side, "ecp_c" if name == "C_ecp" else "ecp_c2")}
    if cpu_baseline_on and name == "C_ecp":
        sys.path.insert(0, ROOT)
        from oracle import network as onet, pphamiltonian as opp, system as osys
        net = onet.Network(osys.make_system("C_ecp"))
        pt = onet.to_torch(params)
        rng = np.random.default_rng(9)
        x = torch.tensor(osys.init_electrons(rng, s.atoms, s.charges, 2, 1.0))
        rots = opp.haar_rotations(rng, 2)
        t0 = time.perf_counter()
        opp.batch_local_energy_pp(net, pt, opp.c_atom_ccecp(), x, rots)
        tc = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": 2 / tc, "unit": "local-energy evals/s", "cores": torch.get_num_threads(),
                               "kind": "port", "sample": f"float64 oracle, 2 walkers ({tc:.1f}s)"}
    return res


def pp_adam_side_bench(dtype, device, walkers, steps):
    """main_pp_adam_muti_GPU.py:150-190 on the C-atom ccECP config: one training iteration =
    mc_step (10 sweeps) + complex pp local energy + complex-E_L energy gradient (d log|psi| and
    d phase parameter gradients) + Adam update, through the drop-in API."""
    from aiqmc import spin_indices
    from aiqmc.Energy import pphamiltonian
    from aiqmc.Loss import loss as L
    from aiqmc.Optimizer import adam, optax_like as optax
    from aiqmc.VMC import VMCmcstep
    from aiqmc.wavefunction_Ynlm import nn
    from aiqmc.initial_electrons_positions.init import init_electrons
    from aiqmc import systems
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
    opt = optax.chain(optax.scale_by_adam(b1=0.9, b2=0.999, eps=1e-8, eps_root=0.0),
                      optax.scale_by_schedule(lambda t: 0.05 * (1.0 / (1.0 + t)) ** 10000), optax.scale(-1.))
    step = adam.make_training_step(adam.make_opt_update_step(ev, opt))
    mc_step = VMCmcstep.main_monte_carlo(f=network.apply, tstep=0.05, ndim=3, nelectrons=4, nsteps=10,
                                         batch_size=walkers)
    pos, sp = init_electrons(17, None, s.atoms, s.charges, s.spins, walkers, 1.0)
    data = nn.AINetData(positions=pos.to(device, dtype).contiguous(), spins=sp, atoms=s.atoms, charges=s.charges)
    state = None
    for t in range(2):
        data = mc_step(params, data, VMCmcstep.PhiloxKey(19, 10 * t))
        data, params, state, loss_v, aux = step(data, params, state, VMCmcstep.PhiloxKey(23, t))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(steps):
        data = mc_step(params, data, VMCmcstep.PhiloxKey(19, 100 + 10 * t))
        data, params, state, loss_v, aux = step(data, params, state, VMCmcstep.PhiloxKey(23, 100 + t))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    lv = float(loss_v.real) if torch.is_tensor(loss_v) else float(loss_v)
    return {"config": "C atom ccECP, Adam: mc_step (10 sweeps) + complex pp E_L + complex energy gradient + Adam",
            "walkers": walkers, "ms_per_iteration": 1e3 * dt, "iterations_per_s": 1.0 / dt,
            "energy": lv, "finite": bool(math.isfinite(lv))}


def dmc_side_bench(dtype, device, walkers, steps, system="C_ecp", pmc_side=None):
    """DMC propagation through the drop-in API (DMC/dmc.py:72-93 + branch.py, as main_dmc.py:160-210
    drives it): T-moves, drift-diffusion, pp local energies before/after, weight update, stochastic
    comb.  system "C_ecp": the C-atom ccECP tables (the only ones the reference ships);
    "Ne": all-electron Ne through the same pp-only step with zero tables (BASELINE's "Ne + DMC",
    DESIGN.md 4d)."""
    from aiqmc import spin_indices
    from aiqmc.DMC import dmc
    from aiqmc.DMC.Tmoves import compute_tmoves
    from aiqmc.VMC.VMCmcstep import PhiloxKey
    from aiqmc.wavefunction_Ynlm import nn
    from aiqmc.initial_electrons_positions.init import init_electrons
    from aiqmc import systems
    s = systems.make_system(system)
    N, A = s.nelectrons, s.natoms
    network = s.make_network()
    params = network.init(3)
    e = systems.ccecp_tables(system) if system.endswith("_ecp") else systems.all_electron_tables(system)
    tstep = 0.01
    run = dmc.dmc_propagate(network.apply, nn.make_log_network(network.apply), network.apply, e.list_l, N, A, 3,
                            walkers, tstep, 1, s.charges, s.spins, e.rn_local, e.local_coes, e.local_exps,
                            e.rn_non_local, e.non_local_coes, e.non_local_exps)
    tm = compute_tmoves(e.list_l, tstep, N, A, 3, nn.make_log_network(network.apply), e.rn_non_local,
                        e.non_local_coes, e.non_local_exps)
    pos, sp = init_electrons(11, None, s.atoms, s.charges, s.spins, walkers, 1.0)
    data = nn.AINetData(positions=pos.to(device, dtype).contiguous(), spins=sp, atoms=s.atoms, charges=s.charges)
    ctx = network.apply._aiqmc_network.bind(params, s.atoms, dtype)
    w = torch.ones(walkers, dtype=dtype, device=device)
    bc = torch.full((walkers,), 10.0)

    e_ref = -5.4 if system == "C_ecp" else -128.9   # rough ground-state energies (trial/estimate)

    def one(k):
        nonlocal data, w
        eloc, w, data = run(params, PhiloxKey(21, k), data, w, bc, e_ref, e_ref)
        wn, idx = ctx.dmc_branch(w, 0.37)
        data = nn.AINetData(positions=data.positions[idx.long()].contiguous(), spins=data.spins, atoms=data.atoms,
                            charges=data.charges)
        w = wn.expand(walkers).contiguous()
        return eloc

    for k in range(2):
        one(k)
    torch.cuda.synchronize()
    ctx.profile(True)
    t0 = time.perf_counter()
    for k in range(steps):
        eloc = one(100 + k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ctx.profile(False)
    from aiqmc import _lib
    l_ms, l_n = ctx.profile_read(_lib.PROF_LOCAL_ENERGY)
    lavg = l_ms / max(l_n, 1)
    fe, ff = f_el(N, A), f_fwd(N, A)
    # one DMC step: a drift-diffusion sweep ((N + 1) value+gradient passes), two local energies,
    # and with ccECP tables the T-move / nonlocal quadratures (N A 50 value-only configurations each)
    nq = N * A * _lib.ECP_NQ if system.endswith("_ecp") else 0
    it_flop = walkers * ((N + 1) * 3 * ff + 2 * fe + 3 * nq * ff)
    rf = side_roofline(f"k_walker_rev<float,{N},{A},PREP> + k_walker_lap<float,{N},{A}> (local energy, 2 launches)",
                       walkers * fe, lavg, l_n, f"B*F_EL({N},{A}) = {walkers}*{fe:.3g}", pmc_side,
                       "dmc_ne" if system == "Ne" else "dmc_c")
    rf["iteration_achieved"] = it_flop / (dt / steps) / 1e12
    rf["iteration_frac"] = rf["iteration_achieved"] / PEAK_FP32_TFLOPS
    rf["iteration_flop_model"] = "B*((N+1)*3*F_fwd + 2*F_EL + 3*N*A*50*F_fwd [ccECP only]) per DMC step"
    t0 = time.perf_counter()
    for k in range(steps):
        tm(data, params, PhiloxKey(5, k))
    torch.cuda.synchronize()
    dtm = time.perf_counter() - t0
    label = "C atom ccECP" if system == "C_ecp" else f"{system} all-electron (zero pp tables)"
    return {"config": f"{label} DMC step: T-moves + drift-diffusion + 2x pp E_L + weights + comb, drop-in API",
            "walkers": walkers, "tstep": tstep, "ms_per_dmc_step": 1e3 * dt / steps,
            "walker_steps_per_s": walkers * steps / dt, "tmoves_ms": 1e3 * dtm / steps,
            "mean_energy_re": float(eloc.real.mean()),
            # random-init wavefunction: E_L has heavy tails near the nodes of psi, so the mean is
            # carried by a few walkers; the quantiles show the bulk
            "energy_re_quantiles": {q: float(v) for q, v in zip(
                ("p01", "p10", "p50", "p90", "p99"),
                torch.quantile(eloc.real.double().cpu(), torch.tensor([0.01, 0.1, 0.5, 0.9, 0.99], dtype=torch.float64)))},
            "finite": bool(torch.isfinite(eloc.real).all()), "roofline": rf}


def adam_side_bench(dtype, device, walkers, steps, pmc_side=None):
    """BASELINE.json config 'Be atom (4e-), 4096 walkers, Adam, 1xMI355X': one training iteration
    of main_all_electrons_adam_muti_GPU.py:177-190 = mc_step (nsteps=10) + make_loss energy gradient
    (local energy, clipping, GPU parameter gradient) + Adam update, through the drop-in API."""
    from aiqmc import spin_indices
    from aiqmc.Energy import hamiltonian as H
    from aiqmc.Loss import loss as L
    from aiqmc.Optimizer import adam, optax_like as optax
    from aiqmc.VMC import VMCmcstep
    from aiqmc.wavefunction_Ynlm import nn
    from aiqmc.initial_electrons_positions.init import init_electrons
    from aiqmc import systems
    sb = systems.make_system("Be")
    atoms, charges, spins, n = sb.atoms, sb.charges, sb.spins, sb.nelectrons
    network = sb.make_network()
    params = network.init(2)
    pos, sp = init_electrons(5, None, atoms, charges, spins, walkers, 1.0)
    data = nn.AINetData(positions=pos.to(device, dtype).contiguous(), spins=sp, atoms=atoms, charges=charges)
    mc_step = VMCmcstep.main_monte_carlo(f=network.apply, tstep=0.05, ndim=3, nelectrons=n, nsteps=10,
                                         batch_size=walkers)
    le = H.local_energy(f=network.apply, charges=charges, nspins=spins)
    ev = L.make_loss(network=network.apply, local_energy=le, clip_local_energy=5.0, clip_from_median=False,
                     center_at_clipped_energy=True, complex_output=True)
    opt = optax.chain(optax.scale_by_adam(b1=0.9, b2=0.999, eps=1e-8, eps_root=0.0),
                      optax.scale_by_schedule(lambda t: 0.05 * (1.0 / (1.0 + t)) ** 10000), optax.scale(-1.))
    step = adam.make_training_step(adam.make_opt_update_step(ev, opt))
    state = None
    for t in range(2):
        data = mc_step(params, data, VMCmcstep.PhiloxKey(9, 10 * t))
        data, params, state, loss_v, aux = step(data, params, state, t)
    torch.cuda.synchronize()
    from aiqmc import _lib
    ctx = network.apply._aiqmc_network.context(atoms, dtype, None)   # the drop-in's context (nn.bind)
    ctx.profile(True)
    t0 = time.perf_counter()
    for t in range(steps):
        data = mc_step(params, data, VMCmcstep.PhiloxKey(9, 100 + 10 * t))
        data, params, state, loss_v, aux = step(data, params, state, 2 + t)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    ctx.profile(False)
    p_ms, p_n = ctx.profile_read(_lib.PROF_MC_PROPOSAL)
    pavg = p_ms / max(p_n, 1)
    ff = f_fwd(n, 1)
    # whole iteration: 10 sweeps of (N + 1) value+gradient passes, the local energy, the parameter
    # gradient (one value+gradient pass per walker), per walker
    it_flop = walkers * (10 * (n + 1) * 3 * ff + f_el(n, 1) + 3 * ff)
    rf = side_roofline(f"k_quad_grad<float,{n},1,false> (Metropolis proposals, 4 configurations per wave)",
                       walkers * n * 3 * ff, pavg, p_n, f"B*N*3*F_fwd({n},1) = {walkers}*{n}*3*{ff:.0f}",
                       pmc_side, "adam_be")
    rf["iteration_achieved"] = it_flop / dt / 1e12
    rf["iteration_frac"] = rf["iteration_achieved"] / PEAK_FP32_TFLOPS
    rf["iteration_flop_model"] = "B*(10*(N+1)*3*F_fwd + F_EL + 3*F_fwd) per iteration / ms_per_iteration"
    return {"config": "Be atom (4 e-), Adam: mc_step (10 sweeps) + energy gradient + Adam update, drop-in API",
            "walkers": walkers, "ms_per_iteration": 1e3 * dt, "iterations_per_s": 1.0 / dt,
            "walker_steps_per_s": walkers * 10 / dt, "energy": float(loss_v), "finite": bool(math.isfinite(float(loss_v))),
            "roofline": rf}


def load_pmc(lib_sha):
    """PMC-derived per-launch figures of the proposal kernel (rocprofv3 --pmc passes, one counter
    group per run, corrected per MI355X_MICROARCH.md; tools/gpu_pmc3.sh -> profiles/pmc_rNN.json,
    one file per round).  They are used only if a file was taken on THIS library build
    (``lib_sha16`` equal to the loaded .so's hash; the newest round's file is checked first);
    otherwise every counter-derived field is null and the reason is given."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_r[0-9][0-9].json")), reverse=True)
    if not files:
        return {}, "no PMC summary committed (profiles/pmc_rNN.json)"
    seen = []
    for f in files:
        try:
            pmc = json.load(open(f))
        except Exception as e:
            seen.append(f"{os.path.basename(f)} unreadable ({e!r})")
            continue
        if pmc.get("lib_sha16") == lib_sha:
            pmc["pmc_file"] = os.path.relpath(f, ROOT)
            return pmc, None
        seen.append(f"{os.path.basename(f)} taken on library {pmc.get('lib_sha16')}")
    return {}, (f"this run loads library {lib_sha}; " + "; ".join(seen) +
                ": counters not reported for a different build")


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """``--gpus N`` without a launcher: start N ranks (one process per GPU) under
    torch.distributed.run as a CHILD process -- never exec, and before this process touches the
    GPU -- relay rank 0's JSON line on stdout and exit with the child's return code.  The
    reference shards over every local device by itself (main_all_electrons_adam_muti_GPU.py:58-66)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this host driver
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, bufsize=1)
    for line in proc.stdout:       # streamed: progress reaches the caller while the ranks run
        s = line.strip()
        if s.startswith("{") and '"metric"' in s:
            print(s, flush=True)
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    return proc.wait()


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus and "--gpus" in " ".join(sys.argv):
        sys.stderr.write(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}: launch one rank per GPU "
                         f"(torch.distributed.run --nproc-per-node {args.gpus}) or drop the launcher\n")
        sys.exit(2)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; if fewer GPUs than ranks are visible (a rehearsal), ranks share devices.
    # The device is bound before the process group so RCCL's communicator uses it.
    local_dev = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_dev)
    dist_on = world > 1 or args.force_collectives
    backend = args.dist_backend if torch.cuda.is_available() else "gloo"
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if env_world is None:   # --force-collectives without a launcher: a one-rank group of its own
            dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1)
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local_dev)
    dtype = torch.float32 if args.dtype == "f32" else torch.float64
    from aiqmc import constants, _lib
    if args.force_collectives:
        constants.force_collectives(True)
    from aiqmc.initial_electrons_positions.init import init_electrons

    atoms, charges, spins, network, params, ctx = build(args.system, dtype, local_dev)
    N = int(charges.sum())
    if args.global_walkers % world:
        raise SystemExit("--global-walkers must be divisible by the number of ranks")

    def walkers_of(strong):
        if strong:   # contiguous blocks of one global batch (main_all_electrons_adam_muti_GPU.py:86-97)
            B = args.global_walkers // world
            pos0, _ = init_electrons(1000, None, atoms, charges, spins, args.global_walkers, 1.0)
            return B, pos0[rank * B:(rank + 1) * B]
        pos0, _ = init_electrons(1000 + rank, None, atoms, charges, spins, args.walkers, 1.0)
        return args.walkers, pos0

    def measure(B, pos0, steps, warmup, tag):
        """warmup + `steps` timed VMC iterations on this rank's B walkers; the job time is the max
        over ranks (barrier + synchronize on both sides of the timed region)."""
        pos = pos0.to(dev, dtype).contiguous()
        el = torch.empty(B, dtype=dtype, device=dev)
        seed = 12345 + rank + 7919 * tag
        offset = [0]

        def iteration(record=None):
            if record is not None:
                record[0].record()
            ctx.mc_step(pos, args.nsteps, args.tstep, seed=seed, offset=offset[0])
            offset[0] += args.nsteps
            if record is not None:
                record[1].record()
            ctx.local_energy(pos, out=el)
            if record is not None:
                record[2].record()
            return constants.pmean_stats(el)

        for _ in range(warmup):
            iteration()
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        # HIP events around the launches cost GPU time (round 4, N2: 3.07 -> 3.20 ms per iteration
        # at 4096 walkers and 0.78 -> 0.92 ms at 512 with events around every launch), so the
        # kernel averages and the mc_step / local-energy split are taken in the LAST timed
        # iteration only, still inside the timed region and on the launch stream
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        t0 = time.perf_counter()
        stats = None
        for k in range(steps):
            last = k == steps - 1
            if last:
                ctx.profile(True)
            stats = iteration(evs if last else None)
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        t_local = time.perf_counter() - t0
        ctx.profile(False)
        mc_ms = evs[0].elapsed_time(evs[1])   # one iteration
        el_ms = evs[1].elapsed_time(evs[2])
        prop_ms, prop_n = ctx.profile_read(_lib.PROF_MC_PROPOSAL)
        walk_ms, walk_n = ctx.profile_read(_lib.PROF_MC_WALKER)
        lap_ms, lap_n = ctx.profile_read(_lib.PROF_LOCAL_ENERGY)
        tt = torch.tensor([t_local, mc_ms, el_ms], dtype=torch.float64, device=dev)
        if dist_on:
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_job, mc_ms_max, el_ms_max = tt.tolist()
        mean_e, var_e = (float(stats[0]), float(stats[1]))
        finite = bool(torch.isfinite(pos).all().item()) and math.isfinite(mean_e)
        total = world * B
        return {"B": B, "total_walkers": total, "t_job": t_job, "steps": steps,
                "value": total * args.nsteps * steps / t_job, "ms_per_step": 1e3 * t_job / steps,
                "local_energy_evals_per_s": total / (el_ms_max * 1e-3),
                "mc_walker_steps_per_s": total * args.nsteps / (mc_ms_max * 1e-3),
                "prop_avg_ms": prop_ms / max(prop_n, 1), "prop_n": prop_n,
                "walk_avg_ms": walk_ms / max(walk_n, 1), "lap_avg_ms": lap_ms / max(lap_n, 1), "lap_n": lap_n,
                "mean_e": mean_e, "var_e": var_e, "finite": finite}

    peak = PEAK_FP32_TFLOPS if dtype == torch.float32 else PEAK_FP64_TFLOPS
    lib_sha = _lib.library_sha16()
    pmc, pmc_reason = load_pmc(lib_sha)
    pmc_side = load_pmc_side(lib_sha)

    def rooflines(m):
        B = m["B"]
        flop_prop = B * N * F_VG_N2 if args.system == "N2" else None
        achieved = (flop_prop / (m["prop_avg_ms"] * 1e-3) / 1e12) if flop_prop else None
        achieved_el = (B * F_EL_N2 / (m["lap_avg_ms"] * 1e-3) / 1e12) if args.system == "N2" else None
        # counters were taken at 4096 walkers per GPU; per-launch bytes scale with the launch size
        use_pmc = pmc and B == pmc.get("walkers", 4096)
        traffic = pmc.get("proposal_hbm_bytes_per_launch") if use_pmc else None
        el_traffic = pmc.get("local_energy_hbm_bytes_per_pair") if use_pmc else None
        why = pmc_reason if not pmc else (None if use_pmc else f"PMC passes were taken at {pmc.get('walkers', 4096)} "
                                                                  f"walkers per GPU, this run has {B}")
        prop = {
            "kernel": "k_walker_rev<float,14,2,PROP> proposal launch (B*N value+gradient configs)",
            # the bound is the fp32 vector ALU (157.3 TF = 64 FLOP/clk/SIMD, MI355X_MICROARCH.md; f32
            # MFMA shares that peak on gfx950): F5 forms Phi = h3 W + b with four
            # v_mfma_f32_16x16x4f32 per configuration (round 4), the rest is VALU; HBM at a few % of 8 TB/s
            "bound": "valu", "compute_unit": "VALU fp32 + MFMA f32 (Phi in F5)",
            "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
            "frac": (achieved / peak) if achieved else None, "traffic": traffic,
            "hbm_gbs": (traffic / (m["prop_avg_ms"] * 1e-3) / 1e9) if traffic else None,
            "hbm_frac": (traffic / (m["prop_avg_ms"] * 1e-3) / 1e9 / PEAK_HBM_GBS) if traffic else None,
            "mfma_util": pmc.get("proposal_mfma_util") if use_pmc else None,
            "valu_insts_per_wave": pmc.get("proposal_valu_insts_per_wave") if use_pmc else None,
            "nonfp_valu_insts_per_wave": pmc.get("proposal_nonfp_valu_insts_per_wave") if use_pmc else None,
            "pmc_lib_sha16": pmc.get("lib_sha16") if pmc else None, "lib_sha16": lib_sha,
            "pmc_file": pmc.get("pmc_file") if pmc else None,
            "pmc_null_reason": why,
            "avg_launch_ms": m["prop_avg_ms"], "launches": m["prop_n"],
            "flop_per_launch": flop_prop,
            "flop_model": "B*N*3*F_fwd, F_fwd=4.9e4 (SURVEY 8d)"}
        lap = {
            "kernel": "k_walker_rev<float,14,2,PREP> + k_walker_lap<float,14,2> (local energy, 2 launches)",
            # fp32 VALU and MFMA share the 157.3 TF peak on gfx950; the adjoint pass forms
            # Q_f = (W.Yt) B with v_mfma_f32_16x16x4f32, the rest is VALU
            "bound": "valu", "compute_unit": "VALU fp32 + MFMA f32 (Q_f in the adjoint pass)",
            "achieved": achieved_el, "peak": peak, "unit": "TFLOP/s",
            "frac": (achieved_el / peak) if achieved_el else None, "avg_launch_ms": m["lap_avg_ms"],
            "traffic": el_traffic,
            "mfma_util": pmc.get("local_energy_mfma_util") if use_pmc else None,
            "launches": m["lap_n"], "flop_model": "B*2.55e6 (SURVEY 8d)"}
        return prop, lap

    strong = not args.weak
    B, pos0 = walkers_of(strong)
    head = measure(B, pos0, args.steps, args.warmup, 0)
    weak = None
    if world > 1 and strong:
        Bw, posw = walkers_of(False)
        weak = measure(Bw, posw, args.steps, args.warmup, 1)
    per_rank = {}
    if world == 1 and not args.no_per_rank and args.system == "N2":
        for n in (2, 4, 8):
            Bn = args.global_walkers // n
            pn, _ = init_electrons(1000, None, atoms, charges, spins, args.global_walkers, 1.0)
            m = measure(Bn, pn[:Bn], max(args.steps, 5), max(args.warmup, 2), 10 + n)
            pr, lr = rooflines(m)
            per_rank[f"N={n}"] = {
                "walkers": Bn, "ms_per_step": m["ms_per_step"],
                "walker_steps_per_s_one_rank": m["value"],
                "projected_job_walker_steps_per_s": n * m["value"],
                "mc_walker_steps_per_s_one_rank": m["mc_walker_steps_per_s"],
                "local_energy_evals_per_s_one_rank": m["local_energy_evals_per_s"],
                "proposal_avg_ms": m["prop_avg_ms"], "walker_launch_avg_ms": m["walk_avg_ms"],
                "local_energy_pair_avg_ms": m["lap_avg_ms"],
                "roofline_frac": pr["frac"], "roofline_local_energy_frac": lr["frac"]}

    if rank == 0:
        prop, lap = rooflines(head)
        out = {
            "metric": METRIC,
            "value": head["value"],
            "unit": "walker*steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32" if dtype == torch.float32 else "f64",
            "data": "synthetic (init_electrons walkers, random-init network of the reference architecture)",
            "config": {"workload": f"{args.system} VMC iteration: {args.nsteps} Metropolis sweeps + local energy "
                                   f"+ energy-stat all-reduce", "system": args.system, "electrons": N,
                       "walkers_per_gpu": head["B"], "global_walkers": head["total_walkers"], "nsteps": args.nsteps,
                       "tstep": args.tstep, "parallelism": f"walker-sharded dp{world}"},
            "local_energy_evals_per_s": head["local_energy_evals_per_s"],
            "mc_walker_steps_per_s": head["mc_walker_steps_per_s"],
            "roofline": prop,
            "roofline_local_energy": lap,
            "walker_grad_avg_ms": head["walk_avg_ms"],
            "mean_energy": head["mean_e"], "energy_variance": head["var_e"], "finite": head["finite"],
        }
        if weak is not None:
            wp, wl = rooflines(weak)
            out["weak_scaling"] = {"walkers_per_gpu": weak["B"], "global_walkers": weak["total_walkers"],
                                   "value": weak["value"], "ms_per_step": weak["ms_per_step"],
                                   "local_energy_evals_per_s": weak["local_energy_evals_per_s"],
                                   "mc_walker_steps_per_s": weak["mc_walker_steps_per_s"],
                                   "roofline_frac": wp["frac"], "roofline_local_energy_frac": wl["frac"],
                                   "finite": weak["finite"]}
        if per_rank:
            out["strong_scaling_per_rank"] = per_rank
        out["collectives"] = {"process_group": dist_on, "backend": backend if dist_on else None,
                              "forced_at_world_1": bool(args.force_collectives and world == 1),
                              "allreduce_calls_before_side_benches": constants.ALLREDUCE_CALLS}
        if world == 1 and not args.no_ecp:
            try:
                out["ecp_c_atom"] = ecp_side_bench(dtype, dev, 4096, 5, not args.no_cpu_baseline, pmc_side=pmc_side)
            except Exception as e:  # a side measurement, never a failure of the headline bench
                out["ecp_c_atom"] = {"error": repr(e)}
            try:
                out["ecp_c2"] = ecp_side_bench(dtype, dev, 4096, 3, False, name="C2_ecp", pmc_side=pmc_side)
            except Exception as e:  # a side measurement, never a failure of the headline bench
                out["ecp_c2"] = {"error": repr(e)}
        if world == 1 and not args.no_adam:
            try:
                c0 = constants.ALLREDUCE_CALLS
                out["adam_be_atom"] = adam_side_bench(dtype, dev, 4096, 5, pmc_side=pmc_side)
                # forced collectives: the fused training step's 3 all-reduces per iteration (plus the
                # MC loop's none) over the process group's backend
                out["adam_be_atom"]["allreduce_calls"] = constants.ALLREDUCE_CALLS - c0
            except Exception as e:  # a side measurement, never a failure of the headline bench
                out["adam_be_atom"] = {"error": repr(e)}
        if world == 1 and not args.no_adam:
            try:
                out["pp_adam_c_atom"] = pp_adam_side_bench(dtype, dev, 4096, 5)
            except Exception as e:  # a side measurement, never a failure of the headline bench
                out["pp_adam_c_atom"] = {"error": repr(e)}
        if world == 1 and not args.no_dmc:
            try:
                out["dmc_c_atom"] = dmc_side_bench(dtype, dev, 4096, 5, pmc_side=pmc_side)
            except Exception as e:  # a side measurement, never a failure of the headline bench
                out["dmc_c_atom"] = {"error": repr(e)}
            try:
                out["dmc_ne_atom"] = dmc_side_bench(dtype, dev, 4096, 5, system="Ne", pmc_side=pmc_side)
            except Exception as e:  # a side measurement, never a failure of the headline bench
                out["dmc_ne_atom"] = {"error": repr(e)}
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(args.system, params, atoms, charges, args.nsteps, args.tstep,
                                                   args.cpu_sample_walkers)
            except Exception as e:  # the baseline is a report, never a failure of the bench
                out["cpu_baseline"] = {"value": None, "error": repr(e)}
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
