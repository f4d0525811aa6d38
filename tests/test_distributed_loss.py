"""The multi-rank training step's collectives, fused per dependency level, over
torch.distributed gloo on the CPU (world 2 and 4).

The reference pmeans the loss statistics and the gradient one value at a time: mean E and its
variance (Loss/loss.py:206,208), the total-variation window of the clipping and the clipped mean
(:107, twice for complex energies), then the parameter gradient (Optimizer/adam.py:55).
``aiqmc.Loss.loss.fused_levels`` does the same arithmetic with ONE packed all-reduce per level:
[Chan 6-vector] -> [TV sums] -> [clipped sums, G, G0].  Each rank here holds a contiguous block
of a global batch and a synthetic per-walker Jacobian (d log|psi| and d phase rows); the
pmean'd gradient, the loss, the variance and the clipped energies must equal the reference's
formulas on the concatenated batch (oracle.loss.energy_gradient_complex, a literal restatement
of loss.py:220-270) to 1e-12, with exactly 3 all-reduces per step (2 without clipping).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

B_RANK, P = 48, 37


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_batch(world, complex_e):
    rng = np.random.default_rng(31)
    n = B_RANK * world
    e = rng.normal(-14.6, 0.5, size=n)
    e[3] = 9.0                    # outliers the 5-TV window clips
    e[n - 2] = -40.0
    if complex_e:
        ei = rng.normal(0.0, 0.2, size=n)
        ei[7] = 4.0
        e = e + 1j * ei
    o_abs = rng.normal(size=(n, P))
    o_ph = rng.normal(size=(n, P))
    return e, o_abs, o_ph


CASES = [  # (clip, center_at_clipped, complex_output, complex energies, all-reduces per step)
    (5.0, True, True, True, 3),
    (5.0, False, True, True, 3),
    (0.0, True, True, True, 2),
    (5.0, True, False, False, 3),
    (5.0, True, True, False, 3),
]


def _worker(rank, world, port, q):
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from aiqmc import constants
    from aiqmc.Loss.loss import fused_levels
    out = []
    for clip, center, cout, cplx, _ in CASES:
        e, o_abs, o_ph = _global_batch(world, cplx)
        sl = slice(B_RANK * rank, B_RANK * (rank + 1))
        e_r = torch.tensor(e[sl])
        Oa, Op = torch.tensor(o_abs[sl]), torch.tensor(o_ph[sl])

        def grad_fn(w, wp):
            return w @ Oa, (wp @ Op if wp is not None else None)

        c0 = constants.ALLREDUCE_CALLS
        loss, var, clipped, g, imag = fused_levels(e_r, grad_fn, clip, center, cout)
        out.append((complex(loss), float(var), clipped.numpy(), g.numpy(), float(imag),
                    constants.ALLREDUCE_CALLS - c0))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_fused_levels_match_concatenated_batch(world):
    from oracle import loss as oloss
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k, (clip, center, cout, cplx, n_ar) in enumerate(CASES):
        e, o_abs, o_ph = _global_batch(world, cplx)
        l_ref, g_ref = oloss.energy_gradient_complex(e, o_abs, o_ph, clip_scale=clip, clip_from_median=False,
                                                     center_at_clipped_energy=center, complex_output=cout)
        g_ref = np.real(g_ref)
        mean = e.mean()
        var_ref = np.mean(np.abs(e - mean) ** 2)
        if clip > 0:
            c = mean
            tr, ti = np.mean(np.abs(e.real - c.real)), np.mean(np.abs(np.imag(e) - np.imag(c)))
            xc = (np.clip(e.real, c.real - clip * tr, c.real + clip * tr)
                  + 1j * np.clip(np.imag(e), np.imag(c) - clip * ti, np.imag(c) + clip * ti))
        else:
            xc = e
        for rank, out in res:
            loss, var, clipped, g, imag, calls = out[k]
            assert calls == n_ar, (k, calls)
            assert abs(loss - complex(mean)) < 1e-12 * abs(mean), k
            assert abs(var - var_ref) < 1e-12 * var_ref, k
            sl = slice(B_RANK * rank, B_RANK * (rank + 1))
            np.testing.assert_allclose(clipped, xc[sl] if cplx else xc[sl].real, rtol=1e-13, atol=1e-13)
            np.testing.assert_allclose(g, g_ref, rtol=1e-11, atol=1e-12 * np.abs(g_ref).max())
            assert imag == (float(np.count_nonzero(np.imag(e))) if cplx else 0.0)


def test_fused_levels_one_process_without_group():
    """No process group: every all-reduce is the identity (none counted), the result is the
    one-device formula."""
    from oracle import loss as oloss
    from aiqmc import constants
    from aiqmc.Loss.loss import fused_levels
    e, o_abs, o_ph = _global_batch(1, True)
    c0 = constants.ALLREDUCE_CALLS
    loss, var, clipped, g, imag = fused_levels(torch.tensor(e), lambda w, wp: (w @ torch.tensor(o_abs),
                                                                             wp @ torch.tensor(o_ph)),
                                               5.0, True, True)
    assert constants.ALLREDUCE_CALLS == c0
    _, g_ref = oloss.energy_gradient_complex(e, o_abs, o_ph, 5.0)
    np.testing.assert_allclose(g.numpy(), np.real(g_ref), rtol=1e-11, atol=1e-12 * np.abs(g_ref).max())
    assert abs(complex(loss) - e.mean()) < 1e-12 * abs(e.mean())
