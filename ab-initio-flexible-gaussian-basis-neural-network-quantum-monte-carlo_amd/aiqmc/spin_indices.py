"""Spin / pair index tables (AIQMCrelease3/spin_indices.py).

Same semantics and ordering as the reference (row-major ``nonzero`` order),
computed with numpy on the host once per system.
"""
import numpy as np


def jastrow_indices_ee(spins, nelectrons: int):
    """spin_indices.py:5-19 -> (parallel_indices[2,P], antiparallel_indices[2,Q], P, Q)."""
    s = np.asarray(spins, dtype=np.float64).reshape(nelectrons)
    tot = np.triu(np.outer(s, s), k=1)
    par = np.array(np.nonzero(np.where(tot > 0, tot, 0.0)), dtype=np.int32)
    anti = np.array(np.nonzero(np.where(tot < 0, tot, 0.0)), dtype=np.int32)
    return par, anti, int(par.shape[1]), int(anti.shape[1])


def spin_indices_h(spins):
    """spin_indices.py:38-45 -> (indices_up, indices_down), each a 1-tuple like jnp.nonzero."""
    s = np.asarray(spins, dtype=np.float64)
    return (np.nonzero(s > 0)[0].astype(np.int32),), (np.nonzero(s < 0)[0].astype(np.int32),)
