"""Run only the Be Adam side measurement of bench.py (host-overhead checks of the drop-in API).
AIQMC_DIGEST_BIND=1: AINet.bind re-flattens and digests the parameters on every call (the
behaviour before the identity/version key), for an A/B in one process tree.
AIQMC_HOST_PARAMS=1: the optimiser's parameters round-trip through the host every step (round 4).
AIQMC_PP=1: the C-atom ccECP Adam side measurement instead (complex E_L).
AIQMC_LOSS_TORCH=1: the energy statistics / clipping / weights in torch ops (no fused launch)."""
import hashlib, json, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
sys.path.insert(0, bench.PKG)
from aiqmc.wavefunction_Ynlm import nn  # noqa: E402

if os.environ.get("AIQMC_DIGEST_BIND"):
    def bind(self, params, atoms, dtype=torch.float32, device=None):
        ctx = self.context(atoms, dtype, device)
        flat = nn.flatten_params(params)
        digest = hashlib.sha1(flat.tobytes()).hexdigest()
        k = id(ctx)
        if self._loaded.get(k) != digest:
            ctx.set_params(flat)
            self._loaded[k] = digest
        return ctx
    nn.AINet.bind = bind
if os.environ.get("AIQMC_LOSS_TORCH"):
    from aiqmc.Loss import loss as _L0
    _L0.FUSED_ONE_RANK = False
if os.environ.get("AIQMC_HOST_PARAMS"):
    # the round-4 behaviour: the optimiser's new parameters copied to the host (numpy leaves) and
    # uploaded again by the next bind, for an A/B against the device-resident step
    from aiqmc.Loss import loss as _L
    _orig = _L._unflatten_like
    _L._unflatten_like = lambda t, f: _orig(t, f.detach().cpu().numpy() if isinstance(f, torch.Tensor) else f)
for _ in range(2):
    if os.environ.get("AIQMC_PP"):
        print(json.dumps(bench.pp_adam_side_bench(torch.float32, torch.device("cuda", 0), 4096, 5)), flush=True)
    else:
        print(json.dumps(bench.adam_side_bench(torch.float32, torch.device("cuda", 0), 4096, 5)), flush=True)
