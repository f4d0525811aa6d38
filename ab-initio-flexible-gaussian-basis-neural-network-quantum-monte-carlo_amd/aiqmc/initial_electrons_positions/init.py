"""Walker initialisation (AIQMCrelease3/initial_electrons_positions/init.py:7-30)."""
from typing import Tuple

import numpy as np
import torch


def init_electrons(key, structure, atoms, charges, electrons, batch_size: int,
                   init_width: float) -> Tuple[torch.Tensor, np.ndarray]:
    """Electron block i sits on atom i, charges[i] times, plus N(0,1)*init_width.

    ``key`` is an int seed or a numpy Generator (the reference uses a JAX key;
    RNG-stream bit compatibility is out of scope).  ``structure`` is unused, as
    in the reference.  Returns (positions [batch_size, 3N] float64 tensor, spins).
    """
    del structure
    rng = key if isinstance(key, np.random.Generator) else np.random.default_rng(int(key))
    atoms = np.asarray(atoms, dtype=np.float64)
    charges = np.asarray(charges)
    block = np.concatenate([np.tile(atoms[i], int(charges[i])) for i in range(len(atoms))])
    pos = np.tile(block[None, :], (batch_size, 1))
    pos = pos + rng.standard_normal(pos.shape) * init_width
    return torch.from_numpy(pos), np.asarray(electrons)
