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


def test_writer_iteration_key_and_missing_columns(tmp_path):
    from aiqmc.utils.writers import Writer
    with Writer("DMC_states", ["block", "energy", "positions"], directory=str(tmp_path / "new"), log=False) as w:
        w.write(4, block=4, energy=-5.25)
    lines = open(tmp_path / "new" / "DMC_states.csv").read().splitlines()
    assert lines == ["t,block,energy,positions", "4,4,-5.25,"]


# A checkpoint in the reference's on-disk layout (checkpoint.py:44-60 run under JAX + optax):
# params / data / opt_state are pickled pytrees of jax arrays (jax._src.array._reconstruct_array
# around numpy's _reconstruct + __setstate__) and optax NamedTuple states.  JAX and optax are
# absent here, so a child process writes the same pickle stream through stand-in modules of the
# same names (placed on its sys.path only); this test process then reads it with the
# weights-only interpreter, which imports none of them.
_FAKE_JAX = '''
import numpy as np
def _reconstruct_array(fun, args, arr_state, aval_state):
    a = fun(*args); a.__setstate__(arr_state); return a
class ArrayImpl:
    def __init__(self, v, weak_type=False):
        self._value = np.asarray(v); self.weak_type = weak_type
    def __reduce__(self):
        fun, args, arr_state = self._value.__reduce__()
        return (_reconstruct_array, (fun, args, arr_state, {"weak_type": self.weak_type}))
'''
_FAKE_OPTAX = '''
from typing import NamedTuple, Any
class ScaleByAdamState(NamedTuple):
    count: Any
    mu: Any
    nu: Any
class ScaleByScheduleState(NamedTuple):
    count: Any
'''
_WRITER = '''
import sys, dataclasses, numpy as np
sys.path.insert(0, sys.argv[1])
from jax._src.array import ArrayImpl
from optax._src.transform import ScaleByAdamState, ScaleByScheduleState
@dataclasses.dataclass
class AINetData:
    positions: object
    spins: object
    atoms: object
    charges: object
rng = np.random.default_rng(0)
J = lambda a: ArrayImpl(np.asarray(a))
params = {"envelope": [{"alpha": J(rng.standard_normal(1).astype(np.float32))}],
          "orbitals": [{"w": J(rng.standard_normal((4, 6)).astype(np.float32)), "b": J(np.arange(6, dtype=np.float32))}]}
data = AINetData(positions=J(rng.standard_normal((3, 12)).astype(np.float32)), spins=J(np.array([1., -1., 1., -1.])),
                 atoms=J(np.zeros((1, 3))), charges=J(np.array([4.0])))
opt = (ScaleByAdamState(count=J(np.int32(9)), mu=params, nu=params), ScaleByScheduleState(count=J(np.int32(9))))
with open(sys.argv[2], "wb") as f:
    # main_all_electrons_adam_muti_GPU.py:204-208: np.asarray(params), np.asarray(opt_state, dtype=object)
    np.savez(f, t=9, data=dataclasses.asdict(data), params=np.asarray(params),
             opt_state=np.asarray(opt, dtype=object))
np.savez(sys.argv[3], w=np.asarray(params["orbitals"][0]["w"]._value),
         pos=np.asarray(data.positions._value))
'''


def test_restore_reference_layout_without_jax(tmp_path):
    import subprocess
    import sys
    from aiqmc import checkpoint
    from aiqmc.utils.safe_npz import Record
    fake = tmp_path / "fake"
    for mod, src in (("jax/_src/array.py", _FAKE_JAX), ("optax/_src/transform.py", _FAKE_OPTAX)):
        f = fake / mod
        f.parent.mkdir(parents=True, exist_ok=True)
        f.write_text(src)
        for d in (f.parent, f.parent.parent):
            (d / "__init__.py").write_text("")
    ck = tmp_path / "Save" / "qmcjax_ckpt_000009.npz"
    ck.parent.mkdir()
    subprocess.run([sys.executable, "-c", _WRITER, str(fake), str(ck), str(tmp_path / "expect.npz")], check=True)
    assert "jax" not in sys.modules and "optax" not in sys.modules
    assert checkpoint.find_last_checkpoint(str(ck.parent)) == str(ck)
    t, data, params, opt = checkpoint.restore(str(ck))
    expect = np.load(str(tmp_path / "expect.npz"))
    assert t == 10
    np.testing.assert_array_equal(params["orbitals"][0]["w"], expect["w"])
    assert params["orbitals"][0]["w"].dtype == np.float32
    np.testing.assert_array_equal(data.positions, expect["pos"])
    assert isinstance(opt[0], Record) and opt[0].type_name == "ScaleByAdamState" and int(opt[0][0]) == 9
    np.testing.assert_array_equal(opt[0][1]["orbitals"][0]["b"], np.arange(6, dtype=np.float32))
    assert "jax" not in sys.modules and "optax" not in sys.modules


def test_safe_loader_refuses_foreign_globals(tmp_path):
    import io
    import zipfile
    import pytest
    from aiqmc.utils.safe_npz import UnsafeCheckpointError, load_npz, loads_pickle_stream
    marker = tmp_path / "pwned"
    evil = (b"\x80\x03cos\nsystem\nX" + len(f"touch {marker}").to_bytes(4, "little") +
            f"touch {marker}".encode() + b"\x85R.")
    with pytest.raises(UnsafeCheckpointError):
        loads_pickle_stream(evil)
    # the same stream as the payload of an object member of an .npz
    hdr = io.BytesIO()
    np.lib.format.write_array_header_1_0(hdr, {"descr": "|O", "fortran_order": False, "shape": ()})
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w") as z:
        z.writestr("params.npy", b"\x93NUMPY\x01\x00" + hdr.getvalue()[8:] + evil)
    with pytest.raises(UnsafeCheckpointError):
        load_npz(io.BytesIO(buf.getvalue()))
    assert not marker.exists()
