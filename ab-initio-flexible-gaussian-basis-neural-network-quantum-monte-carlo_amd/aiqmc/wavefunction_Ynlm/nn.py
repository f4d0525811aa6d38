"""AIQMC wavefunction factory (drop-in for AIQMCrelease3/wavefunction_Ynlm/nn.py).

``make_ai_net`` has the reference signature (nn.py:511-526) and returns a
``Network(init, apply, orbitals)``.  ``apply(params, pos, spins, atoms,
charges) -> (phase, log|psi|)`` evaluates on the GPU through the HIP kernel
``k_walker_rev`` (libaiqmc_hip.so); unlike the reference it accepts a batch
``pos[..., 3N]`` directly (the reference callers vmap it).  ``orbitals(params, pos, ...)``
returns the reference's ``[M]`` with the complex orbital matrix M (aiqmc_orbitals).

Parameters are the reference pytree (nested dict/list of arrays, nn.py:203-278,
370-407); they are flattened in JAX ``tree_flatten`` order for the C-ABI.
Reference behaviours kept: ``spins`` is ignored by apply (the spin tables are
closures), ``determinants`` is ignored (one full determinant, Q10), the import
side effects of nn.py:557-599 are NOT reproduced (Q12).
"""
from __future__ import annotations

import dataclasses
import hashlib
import math
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch

from .. import _lib

DEFAULT_HIDDEN_DIMS = ((4, 4), (4, 4), (4, 4))
DEFAULT_HIDDEN_DIMS_YNLM = (6, 6, 6)


@dataclasses.dataclass
class AINetData:
    """nn.py:20-25.  positions [B,3N]; spins/atoms/charges per walker or shared."""
    positions: Any
    spins: Any
    atoms: Any
    charges: Any

    def __iter__(self):
        return iter(dataclasses.asdict(self).items())

    def keys(self):
        return [f.name for f in dataclasses.fields(self)]

    def __getitem__(self, k):
        return getattr(self, k)


@dataclasses.dataclass
class Network:
    init: Any
    apply: Any
    orbitals: Any


def tree_flatten(tree):
    """JAX tree_flatten leaf order: dict keys sorted, lists in order."""
    if isinstance(tree, dict):
        out = []
        for k in sorted(tree.keys()):
            out.extend(tree_flatten(tree[k]))
        return out
    if isinstance(tree, (list, tuple)):
        out = []
        for v in tree:
            out.extend(tree_flatten(v))
        return out
    if isinstance(tree, torch.Tensor):
        return [tree.detach().to("cpu", torch.float64).numpy()]
    return [np.asarray(tree, dtype=np.float64)]


def tree_leaves(tree):
    """The leaves themselves (tensors / arrays / scalars), in tree_flatten order."""
    if isinstance(tree, dict):
        return [x for k in sorted(tree.keys()) for x in tree_leaves(tree[k])]
    if isinstance(tree, (list, tuple)):
        return [x for v in tree for x in tree_leaves(v)]
    return [tree]


def _flatten_leaves(leaves) -> np.ndarray:
    """Concatenated float64 copy of the leaves; tensor leaves on one device are gathered there and
    copied to the host once (a device->host copy per leaf synchronises once per leaf)."""
    if not leaves:
        return np.zeros(0)
    if all(isinstance(l, torch.Tensor) for l in leaves) and len({l.device for l in leaves}) == 1:
        return torch.cat([l.detach().reshape(-1).to(torch.float64) for l in leaves]).cpu().numpy()
    return np.concatenate([l.reshape(-1) for l in tree_flatten(leaves)])


def flatten_params(params) -> np.ndarray:
    return _flatten_leaves(tree_leaves(params))


def _device_flat(leaves):
    """The float64 device vector whose consecutive pieces the leaves are, in tree order (the trees
    an optimiser step returns: views of one vector), or None.  Checked per leaf from tensor
    metadata only (base, offset, size) -- no device op; a per-leaf gather costs ~3 dispatcher calls
    a leaf, which for the ~60 leaves of a tree is most of a small training step's host time."""
    base = getattr(leaves[0], "_base", None) if leaves else None
    if base is None or base.dtype != torch.float64 or not base.is_contiguous() or base.dim() != 1:
        return None
    off = 0
    for l in leaves:
        if not isinstance(l, torch.Tensor) or l._base is not base or l.storage_offset() != off or not l.is_contiguous():
            return None
        off += l.numel()
    return base if off == base.numel() else None


def flatten_params_device(params, device) -> torch.Tensor:
    """The canonical float64 vector on `device`: device leaves are concatenated there (no host
    round trip; the vector itself when the leaves are its views); host leaves are flattened and
    copied once."""
    leaves = tree_leaves(params)
    if leaves and all(isinstance(l, torch.Tensor) and l.device == torch.device(device) for l in leaves):
        flat = _device_flat(leaves)
        if flat is not None:
            return flat
        return torch.cat([l.detach().reshape(-1).to(torch.float64) for l in leaves])
    return torch.as_tensor(_flatten_leaves(leaves), dtype=torch.float64, device=device)


def _leaf_key(leaves):
    """Identity + in-place version of every tensor leaf (no device sync); None when a leaf is not a
    tensor (its value must then be compared)."""
    if not all(isinstance(l, torch.Tensor) for l in leaves):
        return None
    return [(l, l._version, l.data_ptr()) for l in leaves]


def _same_leaves(key, leaves) -> bool:
    return key is not None and len(key) == len(leaves) and all(
        t is l and v == l._version and p == l.data_ptr() for (t, v, p), l in zip(key, leaves))


def _first(x):
    """Accept jnp.nonzero-style 1-tuples or plain arrays."""
    if isinstance(x, tuple) and len(x) == 1:
        x = x[0]
    return np.asarray(x, dtype=np.int32).reshape(-1)


def _atoms_charges(atoms, charges):
    a = atoms.detach().cpu().numpy() if isinstance(atoms, torch.Tensor) else np.asarray(atoms)
    c = charges.detach().cpu().numpy() if isinstance(charges, torch.Tensor) else np.asarray(charges)
    a = np.asarray(a, dtype=np.float64)
    c = np.asarray(c, dtype=np.float64)
    if a.ndim == 3:          # batch-tiled atoms (driver layout, main_all_electrons_adam_muti_GPU.py:87)
        a = a.reshape(-1, a.shape[-2], a.shape[-1])[0]
    if c.ndim == 2:
        c = c.reshape(-1, c.shape[-1])[0]
    return a, c


class AINet:
    """Holds the closures of make_ai_net and the per-(device, dtype, atoms) HIP contexts."""

    def __init__(self, nspins, charges, parallel_indices, antiparallel_indices, spin_up_indices,
                 spin_down_indices, n_parallel, n_antiparallel, ndim, natoms, nelectrons):
        if ndim != 3:
            raise NotImplementedError("ndim must be 3")
        self.nspins = (int(nspins[0]), int(nspins[1]))
        self.charges = np.asarray(charges.detach().cpu() if isinstance(charges, torch.Tensor) else charges,
                                  dtype=np.float64)
        self.par = np.asarray(parallel_indices, dtype=np.int32).reshape(2, -1)
        self.anti = np.asarray(antiparallel_indices, dtype=np.int32).reshape(2, -1)
        if self.par.shape[1] != n_parallel or self.anti.shape[1] != n_antiparallel:
            raise ValueError("n_parallel / n_antiparallel do not match the index tables")
        self.up = _first(spin_up_indices)
        self.dn = _first(spin_down_indices)
        self.natoms = int(natoms)
        self.nelectrons = int(nelectrons)
        self._ctx: Dict[Tuple, _lib.Context] = {}
        self._loaded: Dict[int, tuple] = {}   # id(ctx) -> (leaf key, digest) of the last upload

    # -- init (nn.py:203-278, 370-407; network_blocks.py:63-102) --------------
    def init(self, key) -> Dict[str, Any]:
        rng = key if isinstance(key, np.random.Generator) else np.random.default_rng(int(key))
        N, A = self.nelectrons, self.natoms
        nch = len([s for s in self.nspins if s > 0])

        def lin(i, o, bias=True):
            p = {"w": rng.standard_normal((i, o)) / math.sqrt(float(i))}
            if bias:
                p["b"] = rng.standard_normal((o,))
            return p

        d1, d2, dy = 4 * A, 4, 4 * A + 2
        streams, streams_y = [], []
        for l in range(3):
            din = (nch + 1) * d1 + nch * d2
            layer = {"convolutional": {"w": rng.standard_normal((N, din)) / math.sqrt(float(N)),
                                       "b": rng.standard_normal((N, din // 4))},
                     "single": lin(din // 4, 4)}
            if l < 2:
                layer["double"] = lin(d2, 4)
            streams.append(layer)
            streams_y.append({"single_Ynlm": lin(dy, 6)})
            d1, d2, dy = 4, 4, 6
        return {
            "layers": {"input": {}, "streams": streams, "streams_y": streams_y},
            "orbitals": [lin(d1, 2 * N) for _ in range(nch)],
            "y": [{"w": rng.standard_normal((dy, N)) / math.sqrt(float(dy))}],
            "jastrow_ee": {"ee_par": np.ones(self.par.shape[1]), "ee_anti": np.ones(self.anti.shape[1])},
            "jastrow_ae": {"ae": np.ones((N, A))},
            "envelope": [{"pi": np.ones((A, 3)), "sigma": np.ones((A, 3)), "alpha": np.ones(1),
                          "beta": np.ones(A), "xi": np.ones(1), "eplion": np.ones((A, 3)),
                          "mu": np.ones(A), "nu": np.ones(A)} for _ in range(N)],
        }

    # -- HIP context management ---------------------------------------------
    def context(self, atoms, dtype=torch.float32, device: Optional[int] = None) -> _lib.Context:
        a, _ = _atoms_charges(atoms, self.charges)
        if device is None:
            device = torch.cuda.current_device()
        key = (int(device), dtype, a.tobytes())
        ctx = self._ctx.get(key)
        if ctx is None:
            ctx = _lib.Context(self.nelectrons, self.natoms, self.nspins, a, self.charges, self.up, self.dn,
                               self.par, self.anti, dtype=dtype, device=int(device))
            self._ctx[key] = ctx
        return ctx

    def bind(self, params, atoms, dtype=torch.float32, device: Optional[int] = None,
             force: bool = False) -> _lib.Context:
        """Context with `params` uploaded (re-uploads only when the values changed).

        The same tensor leaves at the same in-place versions and storage pointers as the last
        upload are taken as unchanged without looking at their values (no device->host copy, no
        sync: the drop-in drivers call apply / local_energy / mc_step several times per step with
        one params tree); otherwise the leaves are gathered with one copy and compared by digest.

        Contract: a parameter leaf changed in place must bump its autograd version (every torch
        in-place op does: ``w.add_(..)``, ``w.copy_(..)``, ``w[...] = ..``).  Writes that bypass it
        -- through ``w.data``, a NumPy or DLPack view, or a raw device pointer -- are NOT seen;
        after such a write pass ``force=True`` (or a new tensor).  The repo's optimizers return
        new tensors, so this concerns only outside writers."""
        ctx = self.context(atoms, dtype, device)
        leaves = tree_leaves(params)
        k = id(ctx)
        prev = self._loaded.get(k)
        if not force and prev is not None and _same_leaves(prev[0], leaves):
            return ctx
        if leaves and all(isinstance(l, torch.Tensor) and l.is_cuda and l.device == ctx.device for l in leaves):
            # device leaves (an optimiser step that stayed on the GPU): gathered and repacked on
            # the device, stream-ordered -- no host copy, no digest, no sync
            flat_d = _device_flat(leaves)
            if flat_d is None:
                flat_d = torch.cat([l.detach().reshape(-1).to(torch.float64) for l in leaves])
            ctx.set_params_device(flat_d)
            self._loaded[k] = (_leaf_key(leaves), None)
            return ctx
        flat = _flatten_leaves(leaves)
        digest = hashlib.sha1(flat.tobytes()).hexdigest()
        if force or prev is None or prev[1] != digest:
            ctx.set_params(flat)
        self._loaded[k] = (_leaf_key(leaves), digest)
        return ctx

    # -- apply (nn.py:545-551) --------------------------------------------------
    def apply(self, params, pos, spins=None, atoms=None, charges=None):
        del spins, charges   # closures, as in the reference
        pos_t = pos if isinstance(pos, torch.Tensor) else torch.as_tensor(np.asarray(pos))
        dtype = pos_t.dtype if pos_t.dtype in (torch.float32, torch.float64) else torch.float32
        ctx = self.bind(params, atoms, dtype)
        logabs, phase = ctx.logpsi(pos_t)
        shape = pos_t.shape[:-1]
        return phase.reshape(shape), logabs.reshape(shape)

    def orbitals(self, params, pos, spins=None, atoms=None, charges=None):
        """make_orbitals.apply (nn.py:409-506): ``[M]`` with M the complex [..., N, N] matrix
        Phi * Yt * exp(J_ee/N) exp(J_ae/N) whose slogdet apply() returns (a one-element list, as
        the reference's ``total_orbitals_jastrow``; ``determinants`` is ignored, Q10)."""
        del spins, charges
        pos_t = pos if isinstance(pos, torch.Tensor) else torch.as_tensor(np.asarray(pos))
        dtype = pos_t.dtype if pos_t.dtype in (torch.float32, torch.float64) else torch.float32
        ctx = self.bind(params, atoms, dtype)
        m = ctx.orbitals(pos_t)
        return [m.reshape(*pos_t.shape[:-1], self.nelectrons, self.nelectrons)]


def make_ai_net(nspins, charges, parallel_indices, antiparallel_indices, spin_up_indices, spin_down_indices,
                n_parallel: int, n_antiparallel: int, ndim: int, natoms: int, nelectrons: int,
                determinants: int = 1, bias_orbitals: bool = True, rescale_inputs: bool = False,
                hidden_dims=DEFAULT_HIDDEN_DIMS, hidden_dims_Ynlm=DEFAULT_HIDDEN_DIMS_YNLM) -> Network:
    """nn.py:511-553.  ``determinants`` is ignored exactly as in the reference (Q10), and so is
    ``bias_orbitals``: the reference accepts it (nn.py:523) but never hands it to make_orbitals
    (nn.py:531-539), whose orbital layer always carries its bias."""
    del determinants, bias_orbitals
    if rescale_inputs:
        raise NotImplementedError(
            "rescale_inputs=True: the reference's rescaled e-e features are ee*log(1+r_ee)/r_ee with "
            "r_ee masked to 0 on the diagonal (nn.py:115,130-131), i.e. 0/0 = NaN, and the g_two means "
            "(nn.py:151) spread it to every electron, so its log|psi| is NaN for every configuration "
            "(tests/test_oracle_rescale_inputs.py); the drop-in refuses the option instead")
    if tuple(tuple(h) for h in hidden_dims) != DEFAULT_HIDDEN_DIMS or \
            tuple(hidden_dims_Ynlm) != DEFAULT_HIDDEN_DIMS_YNLM:
        raise NotImplementedError("only the default hidden dims are built")
    net = AINet(nspins, charges, parallel_indices, antiparallel_indices, spin_up_indices, spin_down_indices,
                n_parallel, n_antiparallel, ndim, natoms, nelectrons)
    apply = net.apply
    apply_fn = lambda *a, **k: apply(*a, **k)
    apply_fn._aiqmc_network = net
    return Network(init=net.init, apply=apply_fn, orbitals=net.orbitals)


def make_log_network(signed_network):
    """The complex log the pp drivers build from the signed network
    (``log_network`` in DMC/main_dmc.py:91-93, main_pp_adam_muti_GPU.py:119-121):
    log|psi| + i phase, tagged with the aiqmc network so that the pp / T-move drop-ins
    can dispatch to the kernels."""
    net = getattr(signed_network, "_aiqmc_network", None)
    if net is None:
        raise TypeError("make_log_network: signed_network must be an aiqmc make_ai_net apply")

    def log_network(*args, **kwargs):
        phase, mag = signed_network(*args, **kwargs)
        return mag + 1j * phase

    log_network._aiqmc_network = net
    return log_network
