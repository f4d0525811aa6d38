"""Checkpoints (drop-in for AIQMCrelease3/checkpoint.py:13-70).

``save`` writes ``qmcjax_ckpt_{t:06d}.npz`` with the reference's keys (t, data as a
dict, params, opt_state) via ``np.savez``; device tensors are copied to host numpy
first, so a file written here holds plain numpy leaves.  ``restore`` returns
``(t + 1, AINetData, params, opt_state)`` as the reference does (:63-70).  Reading never
unpickles: ``restore``/``find_last_checkpoint`` go through the weights-only interpreter of
``utils.safe_npz`` (numpy/JAX arrays, numpy scalars, containers, optax state records and
kfac_jax optimizer states; anything else in the file is refused), so the reference's own
pickled-pytree checkpoints -- e.g. ``AIQMCrelease3/example/C2/Save/qmcjax_ckpt_000009.npz``,
whose ``opt_state`` is a ``kfac_jax.Optimizer.State`` -- load without JAX and without
executing anything from the file.

``find_last_checkpoint`` keeps the reference's "try the next file" rule for files that are
truncated or corrupt (checkpoint.py:19-23), but a file the weights-only interpreter REFUSES
(a global outside its vocabulary) raises :class:`UnsafeCheckpointError` naming the file and
the global: silently starting from scratch next to a checkpoint that exists would hide it.
``skip_refused=True`` restores the plain skip (logged at ERROR level).
"""
from __future__ import annotations

import dataclasses
import datetime
import logging
import os
import zipfile
from typing import Any, Optional

import numpy as np
import torch

from .utils.safe_npz import UnsafeCheckpointError, load_npz
from .wavefunction_Ynlm.nn import AINetData


def _host(tree: Any) -> Any:
    """Tensors -> numpy, recursively (dict / list / tuple leaves)."""
    if isinstance(tree, torch.Tensor):
        return tree.detach().cpu().numpy()
    if isinstance(tree, dict):
        return {k: _host(v) for k, v in tree.items()}
    if isinstance(tree, (list, tuple)):
        return type(tree)(_host(v) for v in tree)
    return tree


def find_last_checkpoint(ckpt_path: Optional[str] = None, skip_refused: bool = False) -> Optional[str]:
    """checkpoint.py:13-24: newest loadable qmcjax_ckpt file, or None.  Corrupt files are
    skipped as in the reference; a refused one raises unless ``skip_refused``."""
    if ckpt_path and os.path.exists(ckpt_path):
        files = [f for f in os.listdir(ckpt_path) if "qmcjax_ckpt" in f]
        for file in sorted(files, reverse=True):
            fname = os.path.join(ckpt_path, file)
            try:
                with open(fname, "rb") as f:
                    load_npz(f)
                return fname
            except UnsafeCheckpointError as e:
                if not skip_refused:
                    raise UnsafeCheckpointError(f"{fname}: {e}") from e
                logging.error("Checkpoint %s refused by the weights-only reader (%s). Trying next checkpoint...",
                              fname, e)
            except (OSError, EOFError, zipfile.BadZipFile, ValueError, KeyError):
                logging.info("Error loading checkpoint %s. Trying next checkpoint...", fname)
    return None


def create_save_path(save_path: Optional[str]) -> str:
    """checkpoint.py:27-33."""
    timestamp = datetime.datetime.now().strftime("%Y_%m_%d_%H:%M:%S")
    path = save_path or os.path.join(os.getcwd(), f"AInet_{timestamp}")
    if path and not os.path.isdir(path):
        os.makedirs(path)
    return path


def get_restore_path(restore_path: Optional[str] = None) -> Optional[str]:
    """checkpoint.py:36-41."""
    return restore_path if restore_path else None


def _object0(tree) -> np.ndarray:
    """A 0-d object array holding `tree` (what np.savez makes of a pytree argument)."""
    if isinstance(tree, np.ndarray):
        return tree
    a = np.empty((), dtype=object)
    a[()] = tree
    return a


def save(save_path: str, t: int, data: AINetData, params, opt_state) -> str:
    """checkpoint.py:44-60.  Written to a temporary name and renamed, so a reader never sees
    a partial file (multi-rank drivers: rank 0 alone writes, see DMC.main_dmc)."""
    fname = os.path.join(save_path, f"qmcjax_ckpt_{t:06d}.npz")
    logging.info("Saving checkpoint %s", fname)
    d = {f.name: _host(getattr(data, f.name)) for f in dataclasses.fields(data)}
    tmp = os.path.join(save_path, f".partial_{t:06d}_{os.getpid()}.npz")   # no 'qmcjax_ckpt' in the name
    with open(tmp, "wb") as f:
        np.savez(f, t=t, data=_object0(d), params=_object0(_host(params)), opt_state=_object0(_host(opt_state)))
    os.replace(tmp, fname)
    return fname


def restore(restore_filename: str, batch_size: Optional[int] = None):
    """checkpoint.py:63-70: (t + 1, data, params, opt_state)."""
    del batch_size
    logging.info("Loading checkpoint %s", restore_filename)
    with open(restore_filename, "rb") as f:
        ck = load_npz(f)
    t = ck["t"].tolist() + 1
    data = AINetData(**ck["data"].item())
    params = ck["params"].tolist()
    opt_state = ck["opt_state"].tolist()
    return t, data, params, opt_state
