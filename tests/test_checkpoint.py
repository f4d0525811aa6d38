"""checkpoint / writers drop-ins (AIQMCrelease3/checkpoint.py:13-70, utils/writers.py:7-39)."""
import os

import numpy as np
import torch


def test_save_restore_roundtrip(tmp_path):
    from oracle import system
    from aiqmc import checkpoint
    from aiqmc.wavefunction_Ynlm.nn import AINetData
    s = system.make_system("Be")
    params = system.init_params(np.random.default_rng(0), s)
    pos = torch.tensor(system.init_electrons(np.random.default_rng(1), s.atoms, s.charges, 8, 1.0))
    data = AINetData(positions=pos, spins=s.spins, atoms=s.atoms, charges=s.charges)
    path = checkpoint.create_save_path(str(tmp_path / "run"))
    assert checkpoint.find_last_checkpoint(path) is None
    checkpoint.save(path, 3, data, params, {"count": np.int64(3)})
    f7 = checkpoint.save(path, 7, data, params, {"count": np.int64(7)})
    assert os.path.basename(f7) == "qmcjax_ckpt_000007.npz"
    # a truncated newer file is skipped (checkpoint.py:19-23)
    open(os.path.join(path, "qmcjax_ckpt_000009.npz"), "wb").write(b"PK\x03\x04 broken")
    last = checkpoint.find_last_checkpoint(path)
    assert last == f7
    t, d, p, opt = checkpoint.restore(last)
    assert t == 8 and opt["count"] == 7
    np.testing.assert_array_equal(d.positions, pos.numpy())
    np.testing.assert_array_equal(system.flatten_params(p), system.flatten_params(params))
    assert checkpoint.get_restore_path(None) is None and checkpoint.get_restore_path(path) == path


def test_writer_csv(tmp_path):
    from aiqmc.utils.writers import Writer
    import pytest
    with Writer("train_states", ["step", "energy"], directory=str(tmp_path), iteration_key=None, log=False) as w:
        w.write(0, step=0, energy=-14.5)
        w.write(1, step=1, energy=-14.6)
        with pytest.raises(ValueError):
            w.write(2, foo=1)
    lines = open(tmp_path / "train_states.csv").read().splitlines()
    assert lines == ["step,energy", "0,-14.5", "1,-14.6"]
