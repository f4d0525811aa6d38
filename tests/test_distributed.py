"""Multi-rank host logic over torch.distributed gloo (CPU, world_size 2 and 4).

The data path shards walkers with no collective (VMCmcstep has none);
the only exchange is the energy-statistics pmean (loss.py:206-208), done by
aiqmc.constants.pmean_stats as ONE all-reduce.  These tests check it equals the
single-process statistics of the concatenated walker set, and that
psum/pmean/all_gather follow the reference's constants.py semantics.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from aiqmc import constants
    rng = np.random.default_rng(rank)
    e = torch.tensor(rng.normal(-109.0, 3.0, size=64))
    mean, var = constants.pmean_stats(e)
    x = torch.tensor([float(rank + 1)])
    s = constants.psum(x)
    m = constants.pmean(x)
    g = constants.all_gather(x)
    q.put((rank, e.numpy(), float(mean), float(var), float(s), float(m), g.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_pmean_stats_matches_global(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda t: t[0])
    allE = np.concatenate([r[1] for r in res])
    for r in res:
        np.testing.assert_allclose(r[2], allE.mean(), rtol=1e-12)
        np.testing.assert_allclose(r[3], allE.var(), rtol=1e-9)
        assert r[4] == sum(range(1, world + 1))
        np.testing.assert_allclose(r[5], sum(range(1, world + 1)) / world)
        np.testing.assert_array_equal(r[6].reshape(-1), np.arange(1, world + 1))


def test_single_process_collectives_are_identity():
    from aiqmc import constants
    x = torch.tensor([1.0, 2.0])
    assert torch.equal(constants.pmean(x), x)
    assert torch.equal(constants.psum(x), x)
    assert constants.all_gather(x).shape == (1, 2)
    m, v = constants.pmean_stats(torch.tensor([1.0, 3.0]))
    assert float(m) == 2.0 and float(v) == 1.0


def _clip_worker(rank, world, port, q):
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from aiqmc import constants
    from aiqmc.Loss.loss import clip_local_values
    e_all = np.random.default_rng(11).normal(-14.6, 0.5, size=64 * world)
    e_all[5] = 3.0                                                      # outlier clipped by the 5-TV window
    e = torch.tensor(e_all[64 * rank:64 * (rank + 1)])
    loss = constants.pmean(torch.mean(e))
    center, diff = clip_local_values(e, loss, 5.0, False, True)
    g = constants.pmean(torch.tensor(np.full(7, float(rank))))          # the gradient pmean (adam.py:55)
    q.put((rank, float(loss), float(center), diff.numpy(), g.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_clipping_and_gradient_pmean_match_global(world):
    """loss.py:73-135 statistics over ranks (pmean'd mean, TV and clipped mean) equal the
    single-device computation on the concatenated batch; the gradient pmean is the rank mean."""
    from oracle import loss as oloss
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_clip_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
    e_all = np.random.default_rng(11).normal(-14.6, 0.5, size=64 * world)
    e_all[5] = 3.0
    center, diff = oloss.clip_local_values(e_all, e_all.mean(), 5.0)
    for r in res:
        assert abs(r[1] - e_all.mean()) < 1e-12 and abs(r[2] - center) < 1e-12
        np.testing.assert_allclose(r[3], diff[64 * r[0]:64 * (r[0] + 1)], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(r[4], np.full(7, (world - 1) / 2.0))


def _ckpt_worker(rank, world, port, out_dir, q):
    """DMC checkpoint cadence on world ranks whose clocks disagree (each rank used
    its own wall clock, so one rank could enter the gather + barrier while another skipped it)."""
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from aiqmc.DMC import main_dmc
    from aiqmc.wavefunction_Ynlm.nn import AINetData
    # per-rank fake clocks in seconds (save_frequency 1 min): rank 0 is first due at block 1,
    # rank 1 already at block 0
    clock_vals = [0, 0, 100, 100, 200, 200, 300, 300, 400, 400] if rank == 0 else \
        [0, 100, 100, 200, 200, 300, 300, 400, 400, 500]
    calls = [0]

    def clock():
        v = clock_vals[min(calls[0], len(clock_vals) - 1)]
        calls[0] += 1
        return float(v)

    hook = main_dmc.make_checkpoint_hook(out_dir, {"w": np.ones(2)}, {"count": np.int64(0)},
                                         save_frequency=1.0, clock=clock)
    after = []
    for block in range(4):
        pos = torch.full((3, 6), float(10 * rank + block), dtype=torch.float64)
        data = AINetData(positions=pos, spins=np.ones(2), atoms=np.zeros((1, 3)), charges=np.ones(1))
        hook(block, complex(-1.0), data)
        # the next collective of the driver: must pair with the same call on every rank
        x = torch.tensor([float(block)])
        dist.all_reduce(x)
        after.append(float(x))
    q.put((rank, [os.path.basename(f) for f in hook.saved], after))
    dist.barrier()
    dist.destroy_process_group()


def test_dmc_checkpoint_cadence_is_collective(tmp_path):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ckpt_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # rank 0's clock decides (due at blocks 1, 2, 3; rank 1's clock alone would say 0, 1, 2, 3)
    saved0 = res[0][1]
    assert saved0 == [f"qmcjax_ckpt_{b:06d}.npz" for b in (1, 2, 3)] and res[1][1] == []
    for r in res:
        assert r[2] == [float(world * b) for b in range(4)]          # collectives stayed paired
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
    from aiqmc import checkpoint
    for f in saved0:
        t, data, _, _ = checkpoint.restore(str(tmp_path / f))
        block = t - 1
        pos = np.asarray(data.positions)
        assert pos.shape == (6, 6)                                   # both ranks' walkers, rank-major
        np.testing.assert_array_equal(pos[:3], block)
        np.testing.assert_array_equal(pos[3:], 10 + block)


def _run_bench(args, env_extra):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, capture_output=True, text=True,
                          timeout=120, env=env)


@pytest.mark.parametrize("world,gpus", [("2", "8"), ("4", "1"), ("8", "2")])
def test_bench_world_size_mismatch_exits_nonzero(world, gpus):
    """bench.py under a launcher whose WORLD_SIZE differs from --gpus must fail before any GPU call
    instead of measuring a different number of ranks than asked for."""
    out = _run_bench(["--gpus", gpus, "--steps", "1", "--warmup", "0"],
                     {"WORLD_SIZE": world, "RANK": "0", "LOCAL_RANK": "0"})
    assert out.returncode == 2, (out.returncode, out.stderr[-1000:])
    assert f"--gpus {gpus}" in out.stderr and f"WORLD_SIZE={world}" in out.stderr
    assert not out.stdout.strip()
