"""Run only the Be Adam side measurement of bench.py (host-overhead checks of the drop-in API).
AIQMC_DIGEST_BIND=1: AINet.bind re-flattens and digests the parameters on every call (the
behaviour before the identity/version key), for an A/B in one process tree."""
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
for _ in range(2):
    print(json.dumps(bench.adam_side_bench(torch.float32, torch.device("cuda", 0), 4096, 5)), flush=True)
