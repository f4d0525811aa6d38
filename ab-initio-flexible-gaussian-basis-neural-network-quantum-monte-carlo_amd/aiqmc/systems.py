"""Systems and pseudopotential tables of the reference's example configurations.

The reference has no config system: each example script builds ``atoms``, ``charges``,
``spins`` and, for ccECP runs, the ``Rn_local / Local_coes / ...`` tables inline and calls a
driver ``main(...)`` ("Config / flags").  This module holds those values as data
so that drivers, benchmarks and tests build the same systems:

* ``C_ecp``  example/single_atom_C/single_atom_C.py:9-23 (C atom, ccECP, Z_eff = 4, spins +-);
* ``C2_ecp`` example/C2/C2.py:8-27 (C2 at z = +-1 bohr, ccECP on both atoms, BLOCK spins
  [+1]*4 + [-1]*4, nspins (4, 4));
* ``C2``     example/C2_muti_GPU_all_electrons/C2test.py (all-electron C2, alternating spins);
* ``N2``     the benchmark molecule of BASELINE.json (R = 2.0744 bohr);
* ``H2``, ``Be``, ``C``, ``Ne``: the remaining BASELINE.json systems (all-electron atoms /
  molecule, alternating spins as every reference example uses);
* ``O2``     16 electrons (the largest shape built), alternating spins;
* ``CO2_ecp`` example/CO2/co2_test.py:7-19 (AIQMCrelease1/2; C, O, O with ccECP, 16 valence
  electrons, alternating spins): the three-atom shape (16, 3).
"""
from __future__ import annotations

import dataclasses
from typing import Any, Dict, Tuple

import numpy as np

from .spin_indices import jastrow_indices_ee, spin_indices_h

__all__ = ["System", "EcpTables", "make_system", "ccecp_tables", "SYSTEM_NAMES"]


@dataclasses.dataclass
class System:
    """One molecule as a reference driver sets it up."""
    name: str
    atoms: np.ndarray        # [A, 3] bohr
    charges: np.ndarray      # [A]   (Z, or Z_eff for ccECP systems)
    spins: np.ndarray        # [N]   +-1
    nspins: Tuple[int, int]

    @property
    def nelectrons(self) -> int:
        return int(self.spins.shape[0])

    @property
    def natoms(self) -> int:
        return int(self.atoms.shape[0])

    def tables(self) -> Dict[str, Any]:
        """The closure tables of make_ai_net (spin_indices.py:5-45)."""
        par, anti, npar, nanti = jastrow_indices_ee(self.spins, self.nelectrons)
        (up,), (dn,) = spin_indices_h(self.spins)
        return dict(parallel_indices=np.asarray(par), antiparallel_indices=np.asarray(anti), n_parallel=int(npar),
                    n_antiparallel=int(nanti), spin_up_indices=np.asarray(up), spin_down_indices=np.asarray(dn))

    def context(self, dtype=None, device: int = 0):
        """A HIP context (libaiqmc_hip.so) for this system."""
        import torch
        from . import _lib
        t = self.tables()
        return _lib.Context(self.nelectrons, self.natoms, self.nspins, self.atoms, self.charges,
                            t["spin_up_indices"], t["spin_down_indices"], t["parallel_indices"],
                            t["antiparallel_indices"], dtype=dtype or torch.float32, device=device)

    def make_network(self):
        """nn.make_ai_net with this system's closure tables (the drivers' call, e.g.
        main_all_electrons_adam_muti_GPU.py:108-120)."""
        from .wavefunction_Ynlm import nn
        t = self.tables()
        return nn.make_ai_net(nspins=self.nspins, charges=self.charges, parallel_indices=t["parallel_indices"],
                              antiparallel_indices=t["antiparallel_indices"], spin_up_indices=t["spin_up_indices"],
                              spin_down_indices=t["spin_down_indices"], n_parallel=t["n_parallel"],
                              n_antiparallel=t["n_antiparallel"], ndim=3, natoms=self.natoms,
                              nelectrons=self.nelectrons)


def _alternating(n: int) -> np.ndarray:
    return np.array([1.0 if i % 2 == 0 else -1.0 for i in range(n)])


_GEOMETRY = {
    "H2": ([[0.0, 0.0, -0.7], [0.0, 0.0, 0.7]], [1.0, 1.0]),
    "Be": ([[0.0, 0.0, 0.0]], [4.0]),
    "C": ([[0.0, 0.0, 0.0]], [6.0]),
    "C_ecp": ([[0.0, 0.0, 0.0]], [4.0]),
    "Ne": ([[0.0, 0.0, 0.0]], [10.0]),
    "C2": ([[0.0, 0.0, -1.0], [0.0, 0.0, 1.0]], [6.0, 6.0]),
    "C2_ecp": ([[0.0, 0.0, -1.0], [0.0, 0.0, 1.0]], [4.0, 4.0]),
    "N2": ([[0.0, 0.0, -1.0372], [0.0, 0.0, 1.0372]], [7.0, 7.0]),
    "O2": ([[0.0, 0.0, -1.1408], [0.0, 0.0, 1.1408]], [8.0, 8.0]),
    "CO2_ecp": ([[1.33, 1.0, 1.0], [0.0, 1.0, 1.0], [2.66, 1.0, 1.0]], [4.0, 6.0, 6.0]),
}
SYSTEM_NAMES = tuple(_GEOMETRY)


def make_system(name: str) -> System:
    atoms, charges = _GEOMETRY[name]
    atoms = np.asarray(atoms, np.float64)
    charges = np.asarray(charges, np.float64)
    n = int(round(charges.sum()))
    if name == "C2_ecp":   # example/C2/C2.py:10 -- block spins
        spins = np.array([1.0] * (n // 2) + [-1.0] * (n - n // 2))
    else:
        spins = _alternating(n)
    nup = int((spins > 0).sum())
    return System(name, atoms, charges, spins, (nup, n - nup))


@dataclasses.dataclass
class EcpTables:
    """Pseudopotential tables in the drivers' shapes (single_atom_C.py:13-23):
    rn_local / local_coes / local_exps [A, KL]; rn_non_local / ... [A, list_l + 1, KN]."""
    rn_local: np.ndarray
    local_coes: np.ndarray
    local_exps: np.ndarray
    rn_non_local: np.ndarray
    non_local_coes: np.ndarray
    non_local_exps: np.ndarray
    list_l: int


# carbon ccECP as the examples write it (single_atom_C.py:13-23, C2.py:12-27)
_C_LOCAL = ([1.0, 3.0, 2.0], [4.00000, 57.74008, -25.81955], [14.43502, 8.39889, 7.38188])
_C_NONLOCAL = ([[2.0, 2.0], [2.0, 2.0], [2.0, 2.0]], [[52.13345, 0], [0, 0], [0, 0]],
               [[7.76079, 0], [0, 0], [0, 0]])


def all_electron_tables(name: str, list_l: int = 2) -> EcpTables:
    """Zero pseudopotential tables: the pp local energy and T-moves of dmc_propagate (which is
    pp-only, DMC/dmc.py:13-94) reduce to the all-electron Hamiltonian -- zero local coefficients
    leave the -Z/r part of local_pp_energy (pseudopotential.py:86-117), zero nonlocal
    coefficients make E_nl = 0 and every T-move amplitude 0.  How "Ne + DMC" runs."""
    A = make_system(name).natoms
    one = lambda v: np.full((A, 1), v, np.float64)
    nl = lambda v: np.full((A, list_l + 1, 1), v, np.float64)
    return EcpTables(one(1.0), one(0.0), one(1.0), nl(2.0), nl(0.0), nl(1.0), list_l)


# oxygen ccECP of the CO2 example (co2_test.py:11-19: Z_eff 6, one l = 0 projector), in release
# 3's table shapes (the l = 0 term first, zero-padded as the carbon block)
_O_LOCAL = ([1.0, 3.0, 2.0], [6.000000, 73.85984, -47.87600], [12.30997, 14.76962, 13.71419])
_O_NONLOCAL = ([[2.0, 2.0], [2.0, 2.0], [2.0, 2.0]], [[85.86406, 0], [0, 0], [0, 0]],
               [[13.65512, 0], [0, 0], [0, 0]])


def ccecp_tables(name: str) -> EcpTables:
    """The ccECP tables of a pseudopotential example system (a carbon or oxygen block per atom)."""
    blocks = {"C_ecp": "C", "C2_ecp": "CC", "CO2_ecp": "COO"}
    if name not in blocks:
        raise KeyError(f"{name} has no pseudopotential tables")
    loc = {"C": _C_LOCAL, "O": _O_LOCAL}
    nl = {"C": _C_NONLOCAL, "O": _O_NONLOCAL}
    rows = lambda tab, k: np.asarray([tab[e][k] for e in blocks[name]], np.float64)
    return EcpTables(rows(loc, 0), rows(loc, 1), rows(loc, 2), rows(nl, 0), rows(nl, 1), rows(nl, 2), 2)
