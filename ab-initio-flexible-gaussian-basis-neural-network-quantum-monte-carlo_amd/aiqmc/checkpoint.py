"""Checkpoints (drop-in for AIQMCrelease3/checkpoint.py:13-70).

``save`` writes ``qmcjax_ckpt_{t:06d}.npz`` with the reference's keys (t, data as a
dict, params, opt_state) via ``np.savez``; device tensors are copied to host numpy
first, so a file written here holds plain numpy leaves.  ``restore`` returns
``(t + 1, AINetData, params, opt_state)`` as the reference does (:63-70).  Like the
reference, ``restore``/``find_last_checkpoint`` read object arrays, i.e. pickles:
only load files this package (or a trusted run of the reference) wrote.
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


def find_last_checkpoint(ckpt_path: Optional[str] = None) -> Optional[str]:
    """checkpoint.py:13-24: newest loadable qmcjax_ckpt file, or None."""
    if ckpt_path and os.path.exists(ckpt_path):
        files = [f for f in os.listdir(ckpt_path) if "qmcjax_ckpt" in f]
        for file in sorted(files, reverse=True):
            fname = os.path.join(ckpt_path, file)
            with open(fname, "rb") as f:
                try:
                    np.load(f, allow_pickle=True)
                    return fname
                except (OSError, EOFError, zipfile.BadZipFile, ValueError):
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


def save(save_path: str, t: int, data: AINetData, params, opt_state) -> str:
    """checkpoint.py:44-60."""
    fname = os.path.join(save_path, f"qmcjax_ckpt_{t:06d}.npz")
    logging.info("Saving checkpoint %s", fname)
    d = {f.name: _host(getattr(data, f.name)) for f in dataclasses.fields(data)}
    with open(fname, "wb") as f:
        np.savez(f, t=t, data=d, params=np.asarray(_host(params), dtype=object)
                 if not isinstance(params, np.ndarray) else params, opt_state=np.asarray(_host(opt_state), dtype=object))
    return fname


def restore(restore_filename: str, batch_size: Optional[int] = None):
    """checkpoint.py:63-70: (t + 1, data, params, opt_state)."""
    del batch_size
    logging.info("Loading checkpoint %s", restore_filename)
    with open(restore_filename, "rb") as f:
        ck = np.load(f, allow_pickle=True)
        t = ck["t"].tolist() + 1
        data = AINetData(**ck["data"].item())
        params = ck["params"].tolist()
        opt_state = ck["opt_state"].tolist()
    return t, data, params, opt_state
