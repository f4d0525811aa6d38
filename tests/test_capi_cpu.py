"""C-ABI and host-logic checks that need no GPU."""
import ctypes
import re
import os
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "aiqmc.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(aiqmc_\w+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    from aiqmc import _lib
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 13
    for s in syms:
        assert hasattr(lib, s), s
        getattr(lib, s)           # resolves the symbol
    assert set(syms) == set(_lib.EXPORTED_SYMBOLS)


def test_library_is_gfx950_code_object():
    """Every translation unit's offload bundle (zstd-compressed since round 6) holds a gfx950 code
    object and nothing for another GPU target."""
    import subprocess
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_resources
    from aiqmc import _lib
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fb")
        subprocess.run([f"{isa_resources.LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", _lib.LIB_PATH,
                        os.path.join(d, "x")], check=True, capture_output=True)
        pieces = isa_resources.bundles(open(fb, "rb").read())
        assert len(pieces) >= 2
        for i, piece in enumerate(pieces):
            b = os.path.join(d, f"b{i}")
            open(b, "wb").write(piece)
            lst = subprocess.run([f"{isa_resources.LLVM}/clang-offload-bundler", "--list", "--type=o", f"--input={b}"],
                                 capture_output=True, text=True, check=True).stdout.split()
            gpu = [t for t in lst if t.startswith("hip")]
            assert gpu == ["hipv4-amdgcn-amd-amdhsa--gfx950"], lst


def test_supported_shapes_include_benchmark_systems():
    from aiqmc import _lib
    shapes = _lib.supported_shapes()
    for s in [(2, 2), (4, 1), (10, 1), (12, 2), (14, 2)]:
        assert s in shapes


def test_shape_list_is_the_makefiles_and_the_shape_tests_cover_it():
    """The dispatch table (aiqmc_supported_shapes) is generated from csrc/Makefile's SHAPES, and
    tests/test_gpu_shapes.py runs every one of them against the oracle."""
    import os
    import re
    from aiqmc import _lib
    import test_gpu_shapes
    mk = open(os.path.join(os.path.dirname(_lib.__file__), "..", "csrc", "Makefile")).read()
    line = re.search(r"^SHAPES\s*:=\s*(.*)$", mk, re.M).group(1)
    make_shapes = {tuple(int(v) for v in t.split("_")) for t in line.split()}
    assert set(_lib.supported_shapes()) == make_shapes
    assert set(test_gpu_shapes.SHAPES) == {sh for sh in make_shapes if sh[0] >= sh[1]}
    assert {(n, a) for a in (1, 2) for n in range(2, 17)} <= make_shapes


def test_last_error_is_a_string():
    from aiqmc import _lib
    assert isinstance(_lib.last_error(), str)


def test_create_rejects_bad_config_without_touching_gpu():
    from aiqmc import _lib
    lib = _lib.load()
    cfg = _lib.AiqmcCfg()
    cfg.nelectrons = 40
    h = ctypes.c_void_p()
    rc = lib.aiqmc_create(ctypes.byref(cfg), ctypes.byref(h))
    assert rc != 0 and "nelectrons" in _lib.last_error()
    cfg.nelectrons = 4
    cfg.nspins[0], cfg.nspins[1] = 4, 0
    assert lib.aiqmc_create(ctypes.byref(cfg), ctypes.byref(h)) != 0
    assert "spin" in _lib.last_error()
    assert lib.aiqmc_create(None, ctypes.byref(h)) != 0


def test_null_context_calls_fail_cleanly():
    from aiqmc import _lib
    lib = _lib.load()
    assert lib.aiqmc_set_params(None, None, 0, None) != 0
    assert lib.aiqmc_logpsi(None, None, 0, None, None, None) != 0
    assert lib.aiqmc_mc_step(None, None, 0, 0, 0.05, 0, None, None, None, 0, 0, None, None) != 0
    assert lib.aiqmc_param_count(None) == -1


@pytest.mark.parametrize("name", ["H2", "Be", "N2"])
def test_product_flatten_matches_canonical_order(name):
    """aiqmc's tree_flatten == oracle's == JAX tree_flatten order; product init has the reference shapes."""
    from oracle import system
    from aiqmc.wavefunction_Ynlm import nn
    s = system.make_system(name)
    t = s.tables()
    net = nn.make_ai_net(nspins=s.nspins, charges=s.charges, parallel_indices=t["parallel_indices"],
                         antiparallel_indices=t["antiparallel_indices"],
                         spin_up_indices=(t["spin_up_indices"],), spin_down_indices=(t["spin_down_indices"],),
                         n_parallel=t["n_parallel"], n_antiparallel=t["n_antiparallel"], ndim=3,
                         natoms=s.natoms, nelectrons=s.nelectrons)
    p1 = net.init(3)
    ref = system.init_params(np.random.default_rng(0), s)
    assert [a.shape for a in system.tree_flatten(p1)] == [a.shape for a in system.tree_flatten(ref)]
    np.testing.assert_array_equal(nn.flatten_params(p1), system.flatten_params(p1))


def test_local_energy_rejects_foreign_wavefunction():
    from aiqmc.Energy import hamiltonian
    with pytest.raises(TypeError):
        hamiltonian.local_energy(lambda *a: (0, 0), np.ones(1), (1, 0))


def test_unsupported_options_fail_loudly():
    from aiqmc.wavefunction_Ynlm import nn
    from oracle import system
    s = system.make_system("H2")
    t = s.tables()
    kw = dict(nspins=s.nspins, charges=s.charges, parallel_indices=t["parallel_indices"],
              antiparallel_indices=t["antiparallel_indices"], spin_up_indices=t["spin_up_indices"],
              spin_down_indices=t["spin_down_indices"], n_parallel=t["n_parallel"],
              n_antiparallel=t["n_antiparallel"], ndim=3, natoms=2, nelectrons=2)
    with pytest.raises(NotImplementedError):
        nn.make_ai_net(rescale_inputs=True, **kw)
    with pytest.raises(NotImplementedError):
        nn.make_ai_net(hidden_dims=((8, 4),) * 3, **kw)
    # bias_orbitals is accepted and ignored, as in the reference (nn.py:523 is never forwarded)
    a, b = nn.make_ai_net(bias_orbitals=False, **kw), nn.make_ai_net(**kw)
    np.testing.assert_array_equal(nn.flatten_params(a.init(0)), nn.flatten_params(b.init(0)))


def test_spin_tables_product_equals_oracle():
    from aiqmc import spin_indices
    from oracle import system
    for n in [2, 4, 10, 14]:
        s = system.alternating_spins(n)
        a = spin_indices.jastrow_indices_ee(s, n)
        b = system.jastrow_indices_ee(s, n)
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
        up, dn = spin_indices.spin_indices_h(s)
        u2, d2 = system.spin_indices_h(s)
        np.testing.assert_array_equal(up[0], u2)
        np.testing.assert_array_equal(dn[0], d2)


def test_limdrift_matches_reference_formula():
    from aiqmc.VMC.VMCmcstep import limdrift, diag_gauss2
    g = torch.tensor(np.random.default_rng(0).standard_normal((5, 6)))
    v2 = float((g ** 2).sum())
    te = (np.sqrt(1 + 2 * 0.05 * 0.25 * v2) - 1) / (0.25 * v2)
    np.testing.assert_allclose(limdrift(g, 0.05, 0.25).numpy(), g.numpy() * te, rtol=1e-14)
    full = torch.arange(2 * 3 * 9, dtype=torch.float64).reshape(2, 3, 9)
    d = diag_gauss2(full, 3)
    assert d.shape == (2, 3, 3)
    np.testing.assert_array_equal(d[:, 1].numpy(), full[:, 1, 3:6].numpy())
