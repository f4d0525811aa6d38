"""Small-batch walker launches on two waves per walker (k_walker_rev<..., SPL>: the per-electron
stage F1 on wave 0 and the pair stream F2 on wave 1 at the same time, handed over through LDS;
the default for fp32 batches of at most 8 walkers per CU) against one wave per walker
(AIQMC_WALK_SPLIT=0, read once per process): walker positions after three mc_step calls of ten
Philox sweeps and the local energies there must be BITWISE equal -- the split moves work between
waves, not arithmetic (J_ee's per-lane partial sums are handed over in lane order)."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("system,walkers", [("N2", 512), ("N2", 2048), ("Ne", 300), ("C2", 96)])
def test_split_walker_launch_is_bitwise_the_one_wave_launch(tmp_path, system, walkers):
    out = {}
    for v in ("0", "1"):
        f = tmp_path / f"pos{v}.npy"
        env = dict(os.environ, AIQMC_WALK_SPLIT=v, HSA_ENABLE_IPC_MODE_LEGACY="0")
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pos_dump.py"), str(f), system, str(walkers)],
                           env=env, capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stderr[-2000:]
        out[v] = np.load(f)
    assert np.isfinite(out["1"]).all()
    np.testing.assert_array_equal(out["0"], out["1"])
