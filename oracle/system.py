"""System description helpers for the oracle (TEST INFRASTRUCTURE ONLY).

Restates, in numpy float64:
  * ``AIQMCrelease3/spin_indices.py:5-19``  jastrow_indices_ee
  * ``AIQMCrelease3/spin_indices.py:38-45`` spin_indices_h
  * ``AIQMCrelease3/initial_electrons_positions/init.py:7-30`` init_electrons
  * the parameter-tree shapes and init distributions of
    ``wavefunction_Ynlm/nn.py:203-278,370-407``,
    ``network_blocks.py:63-102``, ``Jastrow.py:54-58,95-98``,
    ``envelope.py:11-24``.
"""
from __future__ import annotations

import dataclasses
import math
import re
from typing import Any, Dict, List, Sequence, Tuple

import numpy as np

HIDDEN_DIMS = ((4, 4), (4, 4), (4, 4))   # nn.py:525 default
HIDDEN_DIMS_YNLM = (6, 6, 6)             # nn.py:526 default


def jastrow_indices_ee(spins: np.ndarray, nelectrons: int):
    """spin_indices.py:5-19: upper-triangle same/opposite-spin pair lists.

    Row-major ``jnp.nonzero`` order of the strict upper triangle of s s^T.
    """
    s = np.asarray(spins, dtype=np.float64).reshape(nelectrons)
    tot = np.triu(np.outer(s, s), k=1)
    par = np.array(np.nonzero(np.where(tot > 0, tot, 0.0)), dtype=np.int32)
    anti = np.array(np.nonzero(np.where(tot < 0, tot, 0.0)), dtype=np.int32)
    return par, anti, par.shape[1], anti.shape[1]


def spin_indices_h(spins: np.ndarray):
    """spin_indices.py:38-45: ascending indices of up (+) and down (-) electrons."""
    s = np.asarray(spins, dtype=np.float64)
    return (np.nonzero(s > 0)[0].astype(np.int32),
            np.nonzero(s < 0)[0].astype(np.int32))


def init_electrons(rng: np.random.Generator, atoms: np.ndarray, charges: np.ndarray,
                   batch_size: int, init_width: float) -> np.ndarray:
    """init.py:7-30: electron block i at atom i, charges[i] times, + N(0,1)*width.

    The reference draws the noise with jax threefry; here numpy's generator is
    used (bit compatibility of RNG streams is out of scope).
    """
    block = np.concatenate([np.tile(atoms[i], int(charges[i])) for i in range(len(atoms))])
    pos = np.tile(block[None, :], (batch_size, 1)).astype(np.float64)
    return pos + rng.standard_normal(pos.shape) * init_width


@dataclasses.dataclass
class System:
    """An all-electron molecule as the reference drivers set it up."""
    name: str
    atoms: np.ndarray        # [A,3]
    charges: np.ndarray      # [A]
    spins: np.ndarray        # [N] of +-1
    nspins: Tuple[int, int]

    @property
    def nelectrons(self) -> int:
        return int(self.spins.shape[0])

    @property
    def natoms(self) -> int:
        return int(self.atoms.shape[0])

    def tables(self) -> Dict[str, Any]:
        par, anti, npar, nanti = jastrow_indices_ee(self.spins, self.nelectrons)
        up, dn = spin_indices_h(self.spins)
        return dict(parallel_indices=par, antiparallel_indices=anti,
                    n_parallel=npar, n_antiparallel=nanti,
                    spin_up_indices=up, spin_down_indices=dn)


def alternating_spins(n: int) -> np.ndarray:
    return np.array([1.0 if i % 2 == 0 else -1.0 for i in range(n)])


def make_system(name: str) -> System:
    """Systems used by BASELINE.json configs (all-electron, alternating spins)."""
    if name == "H2":
        atoms = np.array([[0.0, 0.0, -0.7], [0.0, 0.0, 0.7]])
        charges = np.array([1.0, 1.0])
    elif name == "Be":
        atoms = np.zeros((1, 3))
        charges = np.array([4.0])
    elif name == "C":
        atoms = np.zeros((1, 3))
        charges = np.array([6.0])
    elif name == "C_ecp":
        # ccECP carbon: Z_eff = 4 at the origin, 4 valence electrons (single_atom_C.py:9-11)
        atoms = np.zeros((1, 3))
        charges = np.array([4.0])
    elif name == "Ne":
        atoms = np.zeros((1, 3))
        charges = np.array([10.0])
    elif name == "C2":
        atoms = np.array([[0.0, 0.0, -1.0], [0.0, 0.0, 1.0]])   # C2test.py:9
        charges = np.array([6.0, 6.0])
    elif name == "C2_ecp":
        # example/C2/C2.py:8-10: ccECP carbons at z = -+1, Z_eff 4, BLOCK spins [+1]*4 + [-1]*4
        atoms = np.array([[0.0, 0.0, -1.0], [0.0, 0.0, 1.0]])
        charges = np.array([4.0, 4.0])
    elif name == "N2":
        atoms = np.array([[0.0, 0.0, -1.0372], [0.0, 0.0, 1.0372]])
        charges = np.array([7.0, 7.0])
    elif name == "CO2_ecp":
        # AIQMCrelease2/example/CO2/co2_test.py:7-10: C, O, O with ccECP charges, alternating spins
        atoms = np.array([[1.33, 1.0, 1.0], [0.0, 1.0, 1.0], [2.66, 1.0, 1.0]])
        charges = np.array([4.0, 6.0, 6.0])
    elif name == "O2":
        atoms = np.array([[0.0, 0.0, -1.1408], [0.0, 0.0, 1.1408]])
        charges = np.array([8.0, 8.0])
    elif re.fullmatch(r"Z\d+(-\d+){0,4}", name):
        # generic shapes (tests/test_gpu_shapes.py): "Z<z>" one atom of charge z at the origin,
        # "Z<a>-<b>" a diatomic of charges a, b at z = -1, +1 bohr, up to five atoms "Z<a>-...-<e>"
        # (the third to fifth off the axis, no symmetry); neutral, alternating spins
        zs = [float(z) for z in name[1:].split("-")]
        sites = np.array([[0.0, 0.0, -1.0], [0.0, 0.0, 1.0], [1.2, 0.7, 0.3], [-0.9, 1.1, -0.4], [0.3, -1.3, 0.8]])
        atoms = np.zeros((1, 3)) if len(zs) == 1 else sites[:len(zs)]
        charges = np.array(zs)
    else:
        raise KeyError(name)
    n = int(charges.sum())
    spins = alternating_spins(n) if name != "C2_ecp" else np.array([1.0] * (n // 2) + [-1.0] * (n - n // 2))
    nup = int((spins > 0).sum())
    return System(name, atoms.astype(np.float64), charges.astype(np.float64), spins, (nup, n - nup))


# ----------------------------------------------------------------------------
# parameters
# ----------------------------------------------------------------------------

def _lin(rng, i, o, bias=True):
    """network_blocks.py:63-86: w ~ N(0,1)/sqrt(in), b ~ N(0,1)."""
    p = {"w": rng.standard_normal((i, o)) / math.sqrt(float(i))}
    if bias:
        p["b"] = rng.standard_normal((o,))
    return p


def init_params(rng: np.random.Generator, system: System, randomize_aux: bool = False,
                hidden_dims=HIDDEN_DIMS, hidden_dims_ynlm=HIDDEN_DIMS_YNLM) -> Dict[str, Any]:
    """Parameter tree of ``make_ai_net`` (nn.py:203-278, 370-407).

    ``randomize_aux`` replaces the all-ones Jastrow/envelope initialisation with
    values in [0.5, 1.5] so that parity tests exercise every parameter.
    """
    N, A = system.nelectrons, system.natoms
    nch = len([s for s in system.nspins if s > 0])
    t = system.tables()
    d1, d2, dy = 4 * A, 4, 4 * A + 2
    streams, streams_y = [], []
    for l in range(len(hidden_dims)):
        din = (nch + 1) * d1 + nch * d2                    # nn.py:209-210,226
        layer = {"convolutional": {                        # network_blocks.py:88-102
            "w": rng.standard_normal((N, din)) / math.sqrt(float(N)),
            "b": rng.standard_normal((N, din // 4))}}
        layer["single"] = _lin(rng, din // 4, hidden_dims[l][0])
        if l < len(hidden_dims) - 1:
            layer["double"] = _lin(rng, d2, hidden_dims[l][1])
        streams.append(layer)
        streams_y.append({"single_Ynlm": _lin(rng, dy, hidden_dims_ynlm[l])})
        d1, d2, dy = hidden_dims[l][0], hidden_dims[l][1], hidden_dims_ynlm[l]
    orbitals = [_lin(rng, d1, 2 * N) for _ in range(nch)]
    y = [{"w": rng.standard_normal((dy, N)) / math.sqrt(float(dy))}]

    def aux(shape):
        if randomize_aux:
            return rng.uniform(0.5, 1.5, size=shape)
        return np.ones(shape)

    params = {
        "layers": {"input": {}, "streams": streams, "streams_y": streams_y},
        "orbitals": orbitals,
        "y": y,
        "jastrow_ee": {"ee_par": aux((t["n_parallel"],)), "ee_anti": aux((t["n_antiparallel"],))},
        "jastrow_ae": {"ae": aux((N, A))},
        "envelope": [{"pi": aux((A, 3)), "sigma": aux((A, 3)), "alpha": aux((1,)),
                      "beta": aux((A,)), "xi": aux((1,)), "eplion": np.ones((A, 3)),
                      "mu": np.ones((A,)), "nu": np.ones((A,))} for _ in range(N)],
    }
    return params


def tree_flatten(tree) -> List[np.ndarray]:
    """JAX tree_flatten order: dict keys sorted, lists in order, leaves C-order."""
    out: List[np.ndarray] = []
    if isinstance(tree, dict):
        for k in sorted(tree.keys()):
            out.extend(tree_flatten(tree[k]))
    elif isinstance(tree, (list, tuple)):
        for v in tree:
            out.extend(tree_flatten(v))
    else:   # numpy / python leaves, or device tensors (a drop-in optimiser step keeps them on the GPU)
        out.append(np.asarray(tree.detach().cpu() if hasattr(tree, "detach") else tree, dtype=np.float64))
    return out


def flatten_params(params) -> np.ndarray:
    """Canonical flat parameter vector (what the C-ABI ``aiqmc_set_params`` takes)."""
    return np.concatenate([a.reshape(-1) for a in tree_flatten(params)])


def param_count(params) -> int:
    return int(sum(a.size for a in tree_flatten(params)))


def map_tree(fn, tree):
    if isinstance(tree, dict):
        return {k: map_tree(fn, v) for k, v in tree.items()}
    if isinstance(tree, list):
        return [map_tree(fn, v) for v in tree]
    if isinstance(tree, tuple):
        return tuple(map_tree(fn, v) for v in tree)
    return fn(tree)


def unflatten_params(template, flat: np.ndarray):
    """Inverse of flatten_params for a tree with the template's structure/shapes."""
    flat = np.asarray(flat, dtype=np.float64)
    pos = [0]

    def build(tree):
        if isinstance(tree, dict):
            return {k: build(tree[k]) for k in sorted(tree.keys())}
        if isinstance(tree, (list, tuple)):
            return [build(v) for v in tree]
        a = np.asarray(tree)
        out = flat[pos[0]:pos[0] + a.size].reshape(a.shape)
        pos[0] += a.size
        return out
    out = build(template)
    if pos[0] != flat.size:
        raise ValueError(f"flat vector has {flat.size} entries, template needs {pos[0]}")
    return out
