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


_REF_C2 = "/root/reference/AIQMCrelease3/example/C2/Save"


def test_restore_reference_release3_kfac_checkpoint():
    """The reference's own release3 checkpoint (example/C2/Save, written by the KFAC
    driver): opt_state pickles kfac_jax.Optimizer.State through builtins.getattr.  Read from
    /root/reference as data only (never executed); skipped where the reference is absent."""
    import pytest
    if not os.path.isdir(_REF_C2):
        pytest.skip("reference tree absent (GPU box)")
    import sys
    from aiqmc import checkpoint
    from aiqmc.utils.safe_npz import StateRecord
    last = checkpoint.find_last_checkpoint(_REF_C2)
    assert os.path.basename(last) == "qmcjax_ckpt_000009.npz"
    t, data, params, opt = checkpoint.restore(last)
    assert t == 10                                  # saved at t = 9, resumes at t + 1 (checkpoint.py:67)
    # pmapped layout [ndev=1, B=4, 3N=24] (C2 ECP: 8 valence electrons, 2 atoms)
    assert data.positions.shape == (1, 4, 24) and data.positions.dtype == np.float32
    assert data.atoms.shape == (1, 4, 2, 3) and data.charges.shape == (1, 4, 2)
    assert data.spins.shape == (1, 4, 8)
    # release2-style network tree: envelope[k] = {pi, sigma}, no convolutional layer
    assert sorted(params) == ["envelope", "jastrow_ee", "layers", "orbitals", "y"]
    assert len(params["envelope"]) == 2 and sorted(params["envelope"][0]) == ["pi", "sigma"]
    assert params["envelope"][0]["pi"].shape == (1, 2, 8)
    assert [sorted(s) for s in params["layers"]["streams"]] == [["double", "single"]] * 2 + [["single"]]
    assert params["orbitals"][0]["w"].shape == (1, 4, 16)
    assert params["jastrow_ee"]["ee_par"].shape == (1, 12) and params["jastrow_ee"]["ee_anti"].shape == (1, 16)
    for leaf in (params["y"][0]["w"], params["layers"]["streams"][2]["single"]["w"]):
        assert np.all(np.isfinite(leaf))
    # kfac_jax optimizer state: a StateRecord tree, the velocities mirroring params
    assert isinstance(opt, StateRecord) and opt.type_name == "Optimizer.State"
    assert sorted(opt) == ["damping", "data_seen", "estimator_state", "step_counter", "velocities"]
    assert int(np.asarray(opt.step_counter).reshape(-1)[0]) == 10
    assert int(np.asarray(opt.data_seen).reshape(-1)[0]) == 40         # 10 steps x 4 walkers
    assert sorted(opt.velocities) == sorted(params)
    assert opt.velocities["orbitals"][0]["w"].shape == params["orbitals"][0]["w"].shape
    est = opt.estimator_state
    assert est.type_name == "BlockDiagonalCurvature.State"
    names = {b.type_name for b in est.blocks_states}
    assert names <= {"Diagonal.State", "KroneckerFactored.State"} and "KroneckerFactored.State" in names
    assert "jax" not in sys.modules and "kfac_jax" not in sys.modules


def test_every_reference_checkpoint_loads():
    """All 45 qmcjax_ckpt files the reference ships (release2 H2/C2/CO2/..., release3 C2) go
    through the weights-only reader."""
    import glob
    import pytest
    files = sorted(glob.glob("/root/reference/**/qmcjax_ckpt_*.npz", recursive=True))
    if not files:
        pytest.skip("reference tree absent (GPU box)")
    from aiqmc.utils.safe_npz import load_npz
    for f in files:
        ck = load_npz(f)
        assert set(ck) == {"t", "data", "params", "opt_state"}, f
        assert ck["data"].item()["positions"].dtype.kind == "f", f


def _npz_with_stream(path, stream, name="params.npy"):
    import zipfile
    hdr = io_mod().BytesIO()
    np.lib.format.write_array_header_1_0(hdr, {"descr": "|O", "fortran_order": False, "shape": ()})
    with zipfile.ZipFile(path, "w") as z:
        z.writestr("t.npy", _npy_int(9))
        z.writestr(name, b"\x93NUMPY\x01\x00" + hdr.getvalue()[8:] + stream)


def io_mod():
    import io
    return io


def _npy_int(v):
    b = io_mod().BytesIO()
    np.save(b, np.int64(v))
    return b.getvalue()


def test_getattr_only_in_the_kfac_state_pattern():
    import pytest
    from aiqmc.utils.safe_npz import StateRecord, UnsafeCheckpointError, loads_pickle_stream
    # getattr(kfac_jax._src.optimizer.Optimizer, "State")() + BUILD({"step_counter": 3})
    good = (b"\x80\x03cbuiltins\ngetattr\nckfac_jax._src.optimizer\nOptimizer\nX\x05\x00\x00\x00State"
            b"\x86R)\x81}X\x0c\x00\x00\x00step_counterK\x03sb.")
    rec = loads_pickle_stream(good)
    assert isinstance(rec, StateRecord) and rec.type_name == "Optimizer.State" and rec.step_counter == 3
    # any other attribute, or getattr on a class outside the allowlist, is refused
    for bad in (good.replace(b"State", b"__new"),
                b"\x80\x03cbuiltins\ngetattr\ncos\nsystem\nX\x05\x00\x00\x00State\x86R.",
                b"\x80\x03cbuiltins\ngetattr\nckfac_jax._src.optimizer\nOptimizer\nX\x05\x00\x00\x00State"
                b"\x86R.",                                             # dangling class marker
                b"\x80\x03cbuiltins\ngetattr\nckfac_jax._src.optimizer\nOptimizer\nX\x05\x00\x00\x00State"
                b"\x86R)\x81K\x01b."):                                 # BUILD with a non-dict state
        with pytest.raises(UnsafeCheckpointError):
            loads_pickle_stream(bad)
    # a non-str attribute name (an array whose == is elementwise) is refused, not a ValueError
    # that find_last_checkpoint would read as a corrupt file
    from aiqmc.utils import safe_npz
    owner = safe_npz._Marker("owner:kfac_jax._src.optimizer Optimizer")
    for name in (np.array(["State", "State"]), 5, b"State"):
        with pytest.raises(UnsafeCheckpointError):
            safe_npz._call(safe_npz._Marker("getattr"), (owner, name))


def test_self_referential_stream_is_refused_not_recursed():
    import pytest
    from aiqmc.utils.safe_npz import UnsafeCheckpointError, loads_pickle_stream
    # memo references back to a list resolve to the same object instead of recursing
    # (the seen-entry is made before descending): L = [L] and L = [(L,)]
    lst = loads_pickle_stream(b"\x80\x03]q\x00h\x00a.")
    assert lst[0] is lst
    lst = loads_pickle_stream(b"\x80\x03]q\x00h\x00\x85q\x01a.")
    assert isinstance(lst[0], tuple) and lst[0][0] is lst
    # deep nesting is refused instead of escaping as a RecursionError
    deep = b"\x80\x03" + b"]" * 5000 + b"a" * 4999 + b"."
    with pytest.raises(UnsafeCheckpointError):
        loads_pickle_stream(deep)


def test_find_last_checkpoint_refused_vs_corrupt(tmp_path):
    import logging
    import pytest
    from aiqmc import checkpoint
    from aiqmc.utils.safe_npz import UnsafeCheckpointError
    d = tmp_path / "Save"
    d.mkdir()
    _npz_with_stream(d / "qmcjax_ckpt_000002.npz", b"\x80\x03]q\x00.")          # loadable
    (d / "qmcjax_ckpt_000003.npz").write_bytes(b"PK\x03\x04 truncated")        # corrupt: skipped
    assert checkpoint.find_last_checkpoint(str(d)) == str(d / "qmcjax_ckpt_000002.npz")
    _npz_with_stream(d / "qmcjax_ckpt_000004.npz", b"\x80\x03cos\nsystem\n)R.")  # refused: raises
    with pytest.raises(UnsafeCheckpointError, match="os.system"):
        checkpoint.find_last_checkpoint(str(d))
    assert checkpoint.find_last_checkpoint(str(d), skip_refused=True) == str(d / "qmcjax_ckpt_000002.npz")
