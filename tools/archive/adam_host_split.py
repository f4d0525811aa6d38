"""Host time of the pieces of one C-atom ccECP (or Be, AIQMC_SYSTEM=Be) Adam training step, no
device synchronisation inside the step: each wrapped call's wall time on the host (launch and
Python overhead only, since nothing waits for the GPU), summed per iteration."""
import collections, os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
sys.path.insert(0, bench.PKG)
from aiqmc import _lib, constants
from aiqmc.Loss import loss as L
from aiqmc.Optimizer import optax_like as optax, adam
acc = collections.defaultdict(float)


def wrap(obj, name, label):
    f = getattr(obj, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        acc[label] += time.perf_counter() - t0
        return r
    setattr(obj, name, g)


wrap(_lib.Context, "local_energy_ecp", "ctx.local_energy_ecp")
wrap(_lib.Context, "local_energy", "ctx.local_energy")
wrap(_lib.Context, "logpsi_param_grad", "ctx.logpsi_param_grad")
wrap(_lib.Context, "phase_param_grad", "ctx.phase_param_grad")
wrap(_lib.Context, "mc_step", "ctx.mc_step")
wrap(_lib.Context, "set_params_device", "ctx.set_params_device")
wrap(L, "clip_local_values", "loss.clip_local_values")
wrap(constants, "pmean", "constants.pmean")
orig_step = adam.make_training_step


def mts(opt_update):
    s = orig_step(opt_update)

    def step(*a, **k):
        t0 = time.perf_counter()
        r = s(*a, **k)
        acc["training step total"] += time.perf_counter() - t0
        return r
    return step


adam.make_training_step = mts
system = os.environ.get("AIQMC_SYSTEM", "C_ecp")
for rep in range(2):
    acc.clear()
    r = (bench.pp_adam_side_bench if system == "C_ecp" else bench.adam_side_bench)(torch.float32, torch.device("cuda", 0), 4096, 5)
    n = 7   # 2 warm-up + 5 timed iterations
    print(system, "ms/iteration", round(r["ms_per_iteration"], 3), {k: round(1e3 * v / n, 3) for k, v in sorted(acc.items())}, flush=True)
