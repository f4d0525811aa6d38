"""ctypes binding of libaiqmc_hip.so (the C-ABI declared in include/aiqmc.h).

The product path has no CPU fallback: if the shared library is missing or a
call fails, this module raises.  torch is imported before the library is
loaded so that the process uses ONE HIP runtime (torch's libamdhip64.so.7
satisfies the library's NEEDED entry by SONAME).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np
import torch  # noqa: F401  (must precede loading the HIP library)

AIQMC_F32 = 0
AIQMC_F64 = 1
AIQMC_RNG_HOST = 0
AIQMC_RNG_PHILOX = 1

# AIQMC_LIB_VARIANT=phaseprof selects the diagnostics build (make -C csrc phaseprof)
_VARIANT = os.environ.get("AIQMC_LIB_VARIANT", "")
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "libaiqmc_hip.so" if not _VARIANT else f"libaiqmc_hip_{_VARIANT}.so")

EXPORTED_SYMBOLS = (
    "aiqmc_create", "aiqmc_destroy", "aiqmc_param_count", "aiqmc_set_params", "aiqmc_set_params_device",
    "aiqmc_logpsi", "aiqmc_logpsi_grad", "aiqmc_local_energy", "aiqmc_local_energy_complex", "aiqmc_mc_step",
    "aiqmc_workspace_bytes", "aiqmc_last_error", "aiqmc_supported_shapes",
    "aiqmc_profile_enable", "aiqmc_profile_read", "aiqmc_debug_logpsi_grad_forward",
    "aiqmc_debug_set_proposal_reuse", "aiqmc_debug_phase_cycles", "aiqmc_debug_local_energy_forward",
    "aiqmc_set_ecp", "aiqmc_local_energy_ecp", "aiqmc_local_energy_ecp_complex", "aiqmc_logpsi_param_grad",
    "aiqmc_dmc_drift_diffusion", "aiqmc_dmc_weights", "aiqmc_dmc_branch", "aiqmc_dmc_tmoves", "aiqmc_phase_param_grad",
    "aiqmc_dmc_weights_ex", "aiqmc_dmc_cut_minima", "aiqmc_orbitals", "aiqmc_debug_set_ablate", "aiqmc_debug_set_fuse_accept", "aiqmc_debug_set_walker_pivots", "aiqmc_debug_set_packed_walkers", "aiqmc_debug_set_quad_pivoted", "aiqmc_debug_set_lap_waves",
    "aiqmc_debug_set_fuse_reduce", "aiqmc_energy_stats", "aiqmc_energy_stats_final",
    "aiqmc_debug_limdrift_factor", "aiqmc_debug_launch_lds", "aiqmc_loss_weights",
    "aiqmc_param_grad_weighted", "aiqmc_loss_level", "aiqmc_loss_pack", "aiqmc_loss_final",
)

PROF_MC_PROPOSAL = 0   # proposal value+gradient launches of aiqmc_mc_step
PROF_MC_WALKER = 1     # walker gradient launches of aiqmc_mc_step
PROF_LOCAL_ENERGY = 2  # aiqmc_local_energy launches
PROF_ECP_QUAD = 3      # value-only launches over the ECP quadrature configurations
ECP_NQ = 50            # quadrature points per (electron, atom) (pseudopotential.py:181-225)


class AiqmcCfg(ctypes.Structure):
    _fields_ = [
        ("nelectrons", ctypes.c_int32),
        ("natoms", ctypes.c_int32),
        ("nspins", ctypes.c_int32 * 2),
        ("dtype", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("atoms", ctypes.POINTER(ctypes.c_double)),
        ("charges", ctypes.POINTER(ctypes.c_double)),
        ("spin_up_indices", ctypes.POINTER(ctypes.c_int32)),
        ("spin_down_indices", ctypes.POINTER(ctypes.c_int32)),
        ("parallel_indices", ctypes.POINTER(ctypes.c_int32)),
        ("n_parallel", ctypes.c_int32),
        ("antiparallel_indices", ctypes.POINTER(ctypes.c_int32)),
        ("n_antiparallel", ctypes.c_int32),
        ("hidden_dims", (ctypes.c_int32 * 2) * 3),
        ("hidden_dims_ynlm", ctypes.c_int32 * 3),
    ]


class AiqmcEcp(ctypes.Structure):
    _fields_ = [
        ("list_l", ctypes.c_int32),
        ("n_local", ctypes.c_int32),
        ("n_nonlocal", ctypes.c_int32),
        ("rn_local", ctypes.POINTER(ctypes.c_double)),
        ("local_coes", ctypes.POINTER(ctypes.c_double)),
        ("local_exps", ctypes.POINTER(ctypes.c_double)),
        ("rn_non_local", ctypes.POINTER(ctypes.c_double)),
        ("non_local_coes", ctypes.POINTER(ctypes.c_double)),
        ("non_local_exps", ctypes.POINTER(ctypes.c_double)),
    ]


_lib: Optional[ctypes.CDLL] = None


def library_sha16(path: Optional[str] = None) -> Optional[str]:
    """First 16 hex digits of the SHA-256 of the shared library file (default: the one this
    module loads).  PMC summaries under profiles/ carry it, and bench.py reports their counters
    only when it matches the library it is running (stale counters are set to null)."""
    import hashlib
    f = path or LIB_PATH
    if not os.path.exists(f):
        return None
    h = hashlib.sha256()
    with open(f, "rb") as fh:
        for chunk in iter(lambda: fh.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()[:16]


def load() -> ctypes.CDLL:
    """Load the HIP library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: build it with `make -C <pkg>/csrc` or __graft_entry__.build(); "
            "the AIQMC hot path has no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    lib.aiqmc_create.argtypes = [ctypes.POINTER(AiqmcCfg), ctypes.POINTER(vp)]
    lib.aiqmc_destroy.argtypes = [vp]
    lib.aiqmc_param_count.argtypes = [vp]
    lib.aiqmc_param_count.restype = i64
    lib.aiqmc_workspace_bytes.argtypes = [vp]
    lib.aiqmc_workspace_bytes.restype = i64
    lib.aiqmc_set_params.argtypes = [vp, ctypes.POINTER(ctypes.c_double), i64, vp]
    lib.aiqmc_set_params_device.argtypes = [vp, vp, i64, vp]
    lib.aiqmc_logpsi.argtypes = [vp, vp, i32, vp, vp, vp]
    lib.aiqmc_logpsi_grad.argtypes = [vp, vp, i32, vp, vp, vp]
    lib.aiqmc_orbitals.argtypes = [vp, vp, i32, vp, vp, vp, vp]
    lib.aiqmc_local_energy.argtypes = [vp, vp, i32, vp, vp, vp, vp]
    lib.aiqmc_local_energy_complex.argtypes = [vp, vp, i32, vp, vp, vp]
    lib.aiqmc_mc_step.argtypes = [vp, vp, i32, i32, ctypes.c_double, i32, vp, vp, vp,
                                  ctypes.c_uint64, ctypes.c_uint64, vp, vp]
    lib.aiqmc_debug_logpsi_grad_forward.argtypes = [vp, vp, i32, vp, vp, vp]
    lib.aiqmc_debug_logpsi_grad_forward.restype = ctypes.c_int
    lib.aiqmc_debug_local_energy_forward.argtypes = [vp, vp, i32, vp, vp, vp, vp]
    lib.aiqmc_debug_local_energy_forward.restype = ctypes.c_int
    lib.aiqmc_debug_set_ablate.argtypes = [vp, i32]
    lib.aiqmc_debug_set_ablate.restype = ctypes.c_int
    lib.aiqmc_debug_set_fuse_accept.argtypes = [vp, i32]
    lib.aiqmc_debug_set_fuse_accept.restype = ctypes.c_int
    lib.aiqmc_loss_weights.argtypes = [vp, vp, i32, i64, ctypes.c_double, i32, ctypes.c_double, vp, vp, vp, vp, vp,
                                       vp]
    lib.aiqmc_loss_weights.restype = ctypes.c_int
    lib.aiqmc_debug_launch_lds.argtypes = [i32, i32, i32, i32, ctypes.POINTER(i32), ctypes.POINTER(i32)]
    lib.aiqmc_debug_launch_lds.restype = ctypes.c_int
    lib.aiqmc_debug_set_walker_pivots.argtypes = [vp, i32]
    lib.aiqmc_debug_set_walker_pivots.restype = ctypes.c_int
    lib.aiqmc_debug_set_packed_walkers.argtypes = [vp, i32]
    lib.aiqmc_debug_set_packed_walkers.restype = ctypes.c_int
    lib.aiqmc_debug_set_quad_pivoted.argtypes = [vp, i32]
    lib.aiqmc_debug_set_quad_pivoted.restype = ctypes.c_int
    lib.aiqmc_debug_set_fuse_reduce.argtypes = [vp, i32]
    lib.aiqmc_debug_set_fuse_reduce.restype = ctypes.c_int
    lib.aiqmc_debug_limdrift_factor.argtypes = [vp, vp, i32, ctypes.c_double, i32,
                                                ctypes.POINTER(ctypes.c_double), vp]
    lib.aiqmc_debug_limdrift_factor.restype = ctypes.c_int
    lib.aiqmc_debug_set_lap_waves.argtypes = [vp, i32]
    lib.aiqmc_debug_set_lap_waves.restype = ctypes.c_int
    lib.aiqmc_debug_set_proposal_reuse.argtypes = [vp, i32]
    lib.aiqmc_debug_set_proposal_reuse.restype = ctypes.c_int
    lib.aiqmc_debug_phase_cycles.argtypes = [vp, vp]
    lib.aiqmc_debug_phase_cycles.restype = ctypes.c_int
    lib.aiqmc_logpsi_param_grad.argtypes = [vp, vp, i32, vp, vp, vp, vp]
    lib.aiqmc_phase_param_grad.argtypes = [vp, vp, i32, vp, vp, vp, vp]
    dbl, u64 = ctypes.c_double, ctypes.c_uint64
    lib.aiqmc_dmc_drift_diffusion.argtypes = [vp, vp, i32, dbl, i32, vp, vp, vp, u64, u64, vp, vp, vp, vp]
    lib.aiqmc_dmc_weights.argtypes = [vp, i32, vp, vp, vp, vp, vp, dbl, dbl, dbl, dbl, vp, vp]
    lib.aiqmc_dmc_weights_ex.argtypes = [vp, i32, vp, vp, vp, vp, vp, dbl, vp, vp, dbl, dbl, dbl, vp, vp, vp]
    lib.aiqmc_dmc_cut_minima.argtypes = [vp, i32, vp, vp, vp, dbl, dbl, vp, vp]
    lib.aiqmc_dmc_branch.argtypes = [vp, i32, vp, dbl, vp, vp, vp]
    lib.aiqmc_dmc_tmoves.argtypes = [vp, vp, i32, dbl, i32, vp, vp, vp, u64, u64, vp, vp]
    lib.aiqmc_set_ecp.argtypes = [vp, ctypes.POINTER(AiqmcEcp)]
    lib.aiqmc_local_energy_ecp.argtypes = [vp, vp, i32, i32, vp, ctypes.c_uint64, ctypes.c_uint64, vp, vp, vp,
                                           vp, vp]
    lib.aiqmc_local_energy_ecp_complex.argtypes = [vp, vp, i32, i32, vp, ctypes.c_uint64, ctypes.c_uint64, vp, vp,
                                                   vp]
    lib.aiqmc_profile_enable.argtypes = [vp, i32]
    lib.aiqmc_profile_read.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i64)]
    lib.aiqmc_energy_stats.argtypes = [vp, i32, i64, vp, i32, vp]
    lib.aiqmc_energy_stats_final.argtypes = [vp, vp]
    lib.aiqmc_param_grad_weighted.argtypes = [vp, vp, i32, i32, vp, i32, vp, vp, vp]
    lib.aiqmc_loss_level.argtypes = [i32, vp, vp, i32, i64, vp, vp, dbl, dbl, i32, vp, vp, vp, vp, vp, vp]
    lib.aiqmc_loss_pack.argtypes = [vp, vp, vp, i32, i32, vp, vp]
    lib.aiqmc_loss_final.argtypes = [vp, vp, i32, i32, i32, i32, i32, vp, vp, vp]
    lib.aiqmc_last_error.restype = ctypes.c_char_p
    lib.aiqmc_supported_shapes.restype = ctypes.c_char_p
    for name in ("aiqmc_create", "aiqmc_destroy", "aiqmc_set_params", "aiqmc_set_params_device", "aiqmc_logpsi",
                 "aiqmc_logpsi_grad", "aiqmc_local_energy", "aiqmc_local_energy_complex", "aiqmc_mc_step", "aiqmc_profile_enable",
                 "aiqmc_profile_read", "aiqmc_set_ecp", "aiqmc_local_energy_ecp", "aiqmc_local_energy_ecp_complex",
                 "aiqmc_logpsi_param_grad",
                 "aiqmc_dmc_drift_diffusion", "aiqmc_dmc_weights", "aiqmc_dmc_branch", "aiqmc_dmc_tmoves",
                 "aiqmc_phase_param_grad", "aiqmc_dmc_weights_ex", "aiqmc_dmc_cut_minima", "aiqmc_orbitals",
                 "aiqmc_energy_stats", "aiqmc_energy_stats_final", "aiqmc_param_grad_weighted",
                 "aiqmc_loss_level", "aiqmc_loss_pack", "aiqmc_loss_final"):
        getattr(lib, name).restype = ctypes.c_int
    _lib = lib
    return lib


def last_error() -> str:
    return load().aiqmc_last_error().decode()


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {last_error()}")


LDS_KINDS = ("proposal", "walker", "adjoint", "lap", "pgrad", "fwdlap")   # AIQMC_LDS_* order


def launch_lds(nelectrons: int, natoms: int, dtype=torch.float32) -> dict:
    """Dynamic LDS bytes and waves per workgroup of the launches of one shape (host only)."""
    lib = load()
    out = {}
    for k, name in enumerate(LDS_KINDS):
        b, w = ctypes.c_int32(0), ctypes.c_int32(0)
        check(lib.aiqmc_debug_launch_lds(int(nelectrons), int(natoms), AIQMC_F32 if dtype == torch.float32 else AIQMC_F64,
                                         k, ctypes.byref(b), ctypes.byref(w)), "aiqmc_debug_launch_lds")
        out[name] = {"dyn_lds_bytes_per_wg": b.value, "waves_per_wg": w.value}
    return out


def supported_shapes():
    s = load().aiqmc_supported_shapes().decode()
    return [tuple(int(v) for v in p.split(":")) for p in s.split(",") if p]


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def energy_stats(e_l: torch.Tensor, finalize: bool = True) -> torch.Tensor:
    """aiqmc_energy_stats on a device tensor of local energies (float32/float64): a float64 device
    tensor [sum |e - m|^2, n m, n m^2, n, mean, variance] (the last two only with finalize)."""
    if not e_l.is_cuda or e_l.dtype not in (torch.float32, torch.float64):
        raise ValueError("energy_stats: a float32/float64 device tensor is required")
    e = e_l.contiguous().reshape(-1)
    out = torch.empty(6, dtype=torch.float64, device=e.device)
    dt = AIQMC_F32 if e.dtype == torch.float32 else AIQMC_F64
    check(load().aiqmc_energy_stats(_ptr(e), dt, e.numel(), _ptr(out), 1 if finalize else 0, _stream(e.device)),
          "aiqmc_energy_stats")
    return out


def loss_weights(e_l: torch.Tensor, clip_scale: float, center_at_clipped: bool, wscale: float,
                 want_imag: bool):
    """aiqmc_loss_weights (one rank): for device local energies (real, or complex: re/im), the
    energy-gradient weights w_re = wscale Re(diff), w_im = wscale Im(diff + aux) (None unless
    want_imag), aux.clipped_energy (same dtype as e_l) and float64 device stats
    [Re mean, Im mean, variance, Re centre, Im centre]."""
    cplx = torch.is_complex(e_l)
    er = (e_l.real if cplx else e_l).contiguous().reshape(-1)
    if not er.is_cuda or er.dtype not in (torch.float32, torch.float64):
        raise ValueError("loss_weights: float32/float64 (or complex64/128) device energies are required")
    ei = e_l.imag.contiguous().reshape(-1) if cplx else None
    n = er.numel()
    wr = torch.empty_like(er)
    wi = torch.empty_like(er) if want_imag else None
    cr = torch.empty_like(er)
    ci = torch.empty_like(er) if cplx else None
    st = torch.empty(5, dtype=torch.float64, device=er.device)
    dt = AIQMC_F32 if er.dtype == torch.float32 else AIQMC_F64
    check(load().aiqmc_loss_weights(_ptr(er), _ptr(ei), dt, n, float(clip_scale), 1 if center_at_clipped else 0,
                                    float(wscale), _ptr(wr), _ptr(wi), _ptr(cr), _ptr(ci), _ptr(st),
                                    _stream(er.device)), "aiqmc_loss_weights")
    clipped = torch.complex(cr, ci) if cplx else cr
    return wr, wi, clipped.reshape(e_l.shape), st


def _dt(t: torch.Tensor) -> int:
    return AIQMC_F32 if t.dtype == torch.float32 else AIQMC_F64


def loss_level(level: int, er: torch.Tensor, ei: Optional[torch.Tensor], L1=None, L2=None,
               clip_scale: float = 0.0, wscale: float = 1.0, g0: bool = False, want_phase: bool = False):
    """aiqmc_loss_level on this rank's device energies (er, ei: contiguous 1-D, float32/float64).
    level 1 -> L1 [6] float64; level 2 -> L2 [2]; level 3 -> (w [1 or 2, n], wp [n] or None,
    clipped_re, clipped_im or None, head [2] float64 = sums of the clipped energies)."""
    n = er.numel()
    dev = er.device
    lib = load()
    st = _stream(dev)
    if level in (1, 2):
        out = torch.empty(6 if level == 1 else 2, dtype=torch.float64, device=dev)
        check(lib.aiqmc_loss_level(level, _ptr(er), _ptr(ei), _dt(er), n, _ptr(L1), None, 0.0, 0.0, 0, None, None,
                                   None, None, _ptr(out), st), "aiqmc_loss_level")
        return out
    w = torch.empty(2 if g0 else 1, n, dtype=er.dtype, device=dev)
    wp = torch.empty_like(er) if want_phase else None
    cr = torch.empty_like(er)
    ci = torch.empty_like(er) if ei is not None else None
    head = torch.empty(2, dtype=torch.float64, device=dev)
    check(lib.aiqmc_loss_level(3, _ptr(er), _ptr(ei), _dt(er), n, _ptr(L1), _ptr(L2), float(clip_scale),
                               float(wscale), 1 if g0 else 0, _ptr(w), _ptr(wp), _ptr(cr), _ptr(ci), _ptr(head), st),
          "aiqmc_loss_level")
    return w, wp, cr, ci, head


def loss_pack(g: torch.Tensor, gp: Optional[torch.Tensor], g0: Optional[torch.Tensor], head: torch.Tensor):
    """L3 = [head (2), g + gp (P), g0 (P, if given)] as one float64 device vector."""
    P = g.numel()
    L3 = torch.empty(2 + P * (2 if g0 is not None else 1), dtype=torch.float64, device=g.device)
    L3[:2].copy_(head)
    check(load().aiqmc_loss_pack(_ptr(g), _ptr(gp), _ptr(g0), _dt(g), P, _ptr(L3), _stream(g.device)),
          "aiqmc_loss_pack")
    return L3


def loss_final(L1: torch.Tensor, L3: torch.Tensor, P: int, g0: bool, center_at_clipped: bool, world: int,
               dtype: torch.dtype):
    """(grad [P] of dtype, stats [6] float64) from the summed level vectors."""
    grad = torch.empty(P, dtype=dtype, device=L1.device)
    stats = torch.empty(6, dtype=torch.float64, device=L1.device)
    check(load().aiqmc_loss_final(_ptr(L1), _ptr(L3), P, 1 if g0 else 0, 1 if center_at_clipped else 0, int(world),
                                  AIQMC_F32 if dtype == torch.float32 else AIQMC_F64, _ptr(grad), _ptr(stats),
                                  _stream(L1.device)), "aiqmc_loss_final")
    return grad, stats


def energy_stats_final(out: torch.Tensor) -> torch.Tensor:
    """aiqmc_energy_stats_final: out[4..5] = [mean, variance] from a summed out[0..3], in place."""
    check(load().aiqmc_energy_stats_final(_ptr(out), _stream(out.device)), "aiqmc_energy_stats_final")
    return out


class Context:
    """One aiqmc_ctx: a system/network configuration bound to one GPU and dtype."""

    def __init__(self, nelectrons: int, natoms: int, nspins: Sequence[int], atoms, charges,
                 spin_up_indices, spin_down_indices, parallel_indices, antiparallel_indices,
                 dtype: torch.dtype = torch.float32, device: int = 0):
        lib = load()
        if dtype not in (torch.float32, torch.float64):
            raise ValueError("dtype must be torch.float32 or torch.float64")
        self.dtype = dtype
        self.device = torch.device("cuda", device)
        self.N = int(nelectrons)
        self.A = int(natoms)
        self._keep = []

        def dbl(a):
            a = np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1))
            self._keep.append(a)
            return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))

        def i32(a):
            a = np.ascontiguousarray(np.asarray(a, dtype=np.int32).reshape(-1))
            self._keep.append(a)
            return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))

        par = np.asarray(parallel_indices, dtype=np.int32).reshape(2, -1)
        anti = np.asarray(antiparallel_indices, dtype=np.int32).reshape(2, -1)
        cfg = AiqmcCfg()
        cfg.nelectrons = self.N
        cfg.natoms = self.A
        cfg.nspins[0], cfg.nspins[1] = int(nspins[0]), int(nspins[1])
        cfg.dtype = AIQMC_F32 if dtype == torch.float32 else AIQMC_F64
        cfg.device = int(device)
        cfg.atoms = dbl(atoms)
        cfg.charges = dbl(charges)
        cfg.spin_up_indices = i32(spin_up_indices)
        cfg.spin_down_indices = i32(spin_down_indices)
        cfg.parallel_indices = i32(par)
        cfg.n_parallel = par.shape[1]
        cfg.antiparallel_indices = i32(anti)
        cfg.n_antiparallel = anti.shape[1]
        for l in range(3):
            cfg.hidden_dims[l][0] = 4
            cfg.hidden_dims[l][1] = 4
            cfg.hidden_dims_ynlm[l] = 6
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib.aiqmc_create(ctypes.byref(cfg), ctypes.byref(h)), "aiqmc_create")
        self._h = h
        self._lib = lib
        self.nparams = int(lib.aiqmc_param_count(h))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                self._lib.aiqmc_destroy(h)
            except Exception:
                pass
            self._h = None

    # -- kernel timing (HIP events on the launch stream) -------------------
    def profile(self, on: bool = True):
        check(self._lib.aiqmc_profile_enable(self._h, 1 if on else 0), "aiqmc_profile_enable")

    def profile_read(self, slot: int):
        """(summed kernel ms, launches) recorded in `slot` since the last read."""
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        check(self._lib.aiqmc_profile_read(self._h, int(slot), ctypes.byref(ms), ctypes.byref(n)),
              "aiqmc_profile_read")
        return ms.value, n.value

    def workspace_bytes(self) -> int:
        return int(self._lib.aiqmc_workspace_bytes(self._h))

    # -- helpers ---------------------------------------------------------
    def _pos(self, pos: torch.Tensor) -> torch.Tensor:
        if not isinstance(pos, torch.Tensor):
            pos = torch.as_tensor(np.asarray(pos))
        pos = pos.to(device=self.device, dtype=self.dtype).contiguous()
        if pos.shape[-1] != 3 * self.N:
            raise ValueError(f"positions must have trailing dim 3N={3 * self.N}, got {tuple(pos.shape)}")
        return pos.reshape(-1, 3 * self.N)

    def set_params(self, flat: np.ndarray):
        flat = np.ascontiguousarray(np.asarray(flat, dtype=np.float64).reshape(-1))
        if flat.size != self.nparams:
            raise ValueError(f"expected {self.nparams} parameters, got {flat.size}")
        with torch.cuda.device(self.device):
            check(self._lib.aiqmc_set_params(self._h, flat.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                             flat.size, _stream(self.device)), "aiqmc_set_params")

    def set_params_device(self, flat: torch.Tensor):
        """Canonical parameters already on this context's device (float64, tree_flatten order):
        repacked into the kernel layout on the device, stream-ordered (no host copy, no sync)."""
        if not (isinstance(flat, torch.Tensor) and flat.is_cuda and flat.dtype == torch.float64
                and flat.is_contiguous() and flat.device == self.device):
            raise ValueError("set_params_device needs a contiguous float64 tensor on the context's device")
        if flat.numel() != self.nparams:
            raise ValueError(f"expected {self.nparams} parameters, got {flat.numel()}")
        with torch.cuda.device(self.device):
            check(self._lib.aiqmc_set_params_device(self._h, _ptr(flat), flat.numel(), _stream(self.device)),
                  "aiqmc_set_params_device")
        self._flat_keep = flat   # the repack reads it later on the stream: keep it alive until then

    def logpsi(self, pos: torch.Tensor, with_phase: bool = True):
        p = self._pos(pos)
        B = p.shape[0]
        logabs = torch.empty(B, dtype=self.dtype, device=self.device)
        phase = torch.empty(B, dtype=self.dtype, device=self.device) if with_phase else None
        check(self._lib.aiqmc_logpsi(self._h, _ptr(p), B, _ptr(logabs), _ptr(phase), _stream(self.device)),
              "aiqmc_logpsi")
        return logabs, phase

    def orbitals(self, pos: torch.Tensor):
        """The complex orbital matrix [B, N, N] (make_orbitals.apply, nn.py:409-506)."""
        p = self._pos(pos)
        B = p.shape[0]
        out = torch.empty(B, self.N, self.N, 2, dtype=self.dtype, device=self.device)
        check(self._lib.aiqmc_orbitals(self._h, _ptr(p), B, _ptr(out), None, None, _stream(self.device)),
              "aiqmc_orbitals")
        return torch.view_as_complex(out)

    def logpsi_grad(self, pos: torch.Tensor):
        p = self._pos(pos)
        B = p.shape[0]
        logabs = torch.empty(B, dtype=self.dtype, device=self.device)
        grad = torch.empty_like(p)
        check(self._lib.aiqmc_logpsi_grad(self._h, _ptr(p), B, _ptr(logabs), _ptr(grad), _stream(self.device)),
              "aiqmc_logpsi_grad")
        return logabs, grad

    def logpsi_grad_forward_mode(self, pos: torch.Tensor):
        """Diagnostics: the same quantity through the forward-mode kernel (cross-check)."""
        p = self._pos(pos)
        B = p.shape[0]
        logabs = torch.empty(B, dtype=self.dtype, device=self.device)
        grad = torch.empty_like(p)
        check(self._lib.aiqmc_debug_logpsi_grad_forward(self._h, _ptr(p), B, _ptr(logabs), _ptr(grad),
                                                        _stream(self.device)), "aiqmc_debug_logpsi_grad_forward")
        return logabs, grad

    def set_lap_waves(self, waves: int):
        """Waves per walker of the local energy's first-derivative pass (0 = by batch size)."""
        check(self._lib.aiqmc_debug_set_lap_waves(self._h, int(waves)), "aiqmc_debug_set_lap_waves")

    def set_fuse_accept(self, on: bool):
        """Diagnostics: fused (default) or separate per-sweep acceptance launch in mc_step."""
        check(self._lib.aiqmc_debug_set_fuse_accept(self._h, int(bool(on))), "aiqmc_debug_set_fuse_accept")

    def set_walker_pivots(self, reuse: bool):
        """Diagnostics: walker launches after an mc_step's first sweep re-use the previous sweep's
        Gauss-Jordan pivot order (default) or run partial pivoting every sweep."""
        check(self._lib.aiqmc_debug_set_walker_pivots(self._h, int(bool(reuse))), "aiqmc_debug_set_walker_pivots")

    def set_packed_walkers(self, on: bool):
        """Diagnostics: walker launches of N <= 8 several per wave (default) or one wave each."""
        check(self._lib.aiqmc_debug_set_packed_walkers(self._h, int(bool(on))), "aiqmc_debug_set_packed_walkers")

    def set_quad_pivoted(self, on: bool):
        """Diagnostics: the N <= 8 ECP quadrature launch factors every configuration with partial
        pivoting (on) instead of the walker's recorded order with a per-configuration fallback."""
        check(self._lib.aiqmc_debug_set_quad_pivoted(self._h, int(bool(on))), "aiqmc_debug_set_quad_pivoted")

    def set_fuse_reduce(self, mode):
        """Diagnostics: fp32 mc_step limdrift sums fused into the walker / proposal launches as
        exact integer accumulations: 1 (default) and 2 always,
        0 never (reduction launches summing the same integers: the same bits), 3 never with the
        fp64 tree-sum launch (k_taueff).  True/False map to 2/0."""
        m = 2 if mode is True else (0 if mode is False else int(mode))
        check(self._lib.aiqmc_debug_set_fuse_reduce(self._h, m), "aiqmc_debug_set_fuse_reduce")

    def limdrift_factor(self, sumsq: torch.Tensor, tstep: float, mode: int) -> float:
        """Diagnostics: the fp32 limdrift factor of the per-configuration |grad|^2 values `sumsq`
        (float32 on this context's device) through mc_step's reductions: 0 = fused integer
        accumulators, 1 = k_taueff_part partials, 2 = the fp64 tree sum (k_taueff)."""
        if sumsq.dtype != torch.float32 or sumsq.device != self.device or sumsq.dim() != 1:
            raise TypeError("sumsq must be a 1-D float32 tensor on the context's device")
        x = sumsq.contiguous()
        out = ctypes.c_double(0.0)
        check(self._lib.aiqmc_debug_limdrift_factor(self._h, _ptr(x), int(x.numel()), float(tstep), int(mode),
                                                    ctypes.byref(out), _stream(self.device)),
              "aiqmc_debug_limdrift_factor")
        return out.value

    def set_ablate(self, mask: int):
        """Development builds (-DAQ_ABLATE) only: skip proposal phases to time them."""
        check(self._lib.aiqmc_debug_set_ablate(self._h, int(mask)), "aiqmc_debug_set_ablate")

    def set_proposal_reuse(self, on: bool):
        """Diagnostics: proposals from the walker cache (default) or recomputed from scratch."""
        check(self._lib.aiqmc_debug_set_proposal_reuse(self._h, 1 if on else 0), "aiqmc_debug_set_proposal_reuse")

    def phase_cycles(self):
        """Diagnostics (AQ_PHASE_PROF builds): per-phase cycle sums [32], then cleared."""
        import numpy as np
        out = np.zeros(32, dtype=np.uint64)
        check(self._lib.aiqmc_debug_phase_cycles(self._h, out.ctypes.data), "aiqmc_debug_phase_cycles")
        return out

    def local_energy(self, pos: torch.Tensor, want_logabs: bool = False, want_grad: bool = False,
                     out: Optional[torch.Tensor] = None):
        p = self._pos(pos)
        B = p.shape[0]
        el = out if out is not None else torch.empty(B, dtype=self.dtype, device=self.device)
        logabs = torch.empty(B, dtype=self.dtype, device=self.device) if want_logabs else None
        grad = torch.empty_like(p) if want_grad else None
        check(self._lib.aiqmc_local_energy(self._h, _ptr(p), B, _ptr(el), _ptr(logabs), _ptr(grad),
                                           _stream(self.device)), "aiqmc_local_energy")
        return el, logabs, grad

    def local_energy_complex(self, pos: torch.Tensor) -> torch.Tensor:
        """complex_output=True local energy (hamiltonian.py:110-130): V - 1/2 [lap log|psi| + i lap theta
        + |grad log|psi||^2 - |grad theta|^2 + 2 i grad log|psi| . grad theta], theta = arg psi; a
        complex tensor [B] (complex64 for a float32 context)."""
        p = self._pos(pos)
        B = p.shape[0]
        re = torch.empty(B, dtype=self.dtype, device=self.device)
        im = torch.empty(B, dtype=self.dtype, device=self.device)
        check(self._lib.aiqmc_local_energy_complex(self._h, _ptr(p), B, _ptr(re), _ptr(im), _stream(self.device)),
              "aiqmc_local_energy_complex")
        return torch.complex(re, im)

    def local_energy_forward_mode(self, pos: torch.Tensor, want_logabs: bool = False, want_grad: bool = False):
        """Diagnostics: the same quantity through the single-launch forward-Laplacian kernel."""
        p = self._pos(pos)
        B = p.shape[0]
        el = torch.empty(B, dtype=self.dtype, device=self.device)
        logabs = torch.empty(B, dtype=self.dtype, device=self.device) if want_logabs else None
        grad = torch.empty_like(p) if want_grad else None
        check(self._lib.aiqmc_debug_local_energy_forward(self._h, _ptr(p), B, _ptr(el), _ptr(logabs), _ptr(grad),
                                                         _stream(self.device)), "aiqmc_debug_local_energy_forward")
        return el, logabs, grad

    def logpsi_param_grad(self, pos: torch.Tensor, weights: Optional[torch.Tensor] = None,
                          want_logabs: bool = False):
        """d log|psi| / d theta in canonical (tree_flatten) order: [B, P] per walker, or [P] =
        sum_b weights[b] d log|psi_b| / d theta when weights [B] are given."""
        p = self._pos(pos)
        B = p.shape[0]
        w = None
        if weights is not None:
            w = weights.to(self.device, self.dtype).contiguous()
            if w.numel() != B:
                raise ValueError("weights must have one entry per walker")
            out = torch.empty(self.nparams, dtype=self.dtype, device=self.device)
        else:
            out = torch.empty(B, self.nparams, dtype=self.dtype, device=self.device)
        la = torch.empty(B, dtype=self.dtype, device=self.device) if want_logabs else None
        check(self._lib.aiqmc_logpsi_param_grad(self._h, _ptr(p), B, _ptr(w), _ptr(out), _ptr(la),
                                                _stream(self.device)), "aiqmc_logpsi_param_grad")
        return (out, la) if want_logabs else out

    def param_grad_weighted(self, pos: torch.Tensor, weights: torch.Tensor, phase: bool = False) -> torch.Tensor:
        """[K, P] = weights [K, B] times d f / d theta (f = log|psi|, or the phase), one gradient pass."""
        p = self._pos(pos)
        B = p.shape[0]
        w = weights.to(self.device, self.dtype).contiguous()
        if w.dim() != 2 or w.shape[1] != B:
            raise ValueError("weights must be [K, B]")
        out = torch.empty(w.shape[0], self.nparams, dtype=self.dtype, device=self.device)
        check(self._lib.aiqmc_param_grad_weighted(self._h, _ptr(p), B, 1 if phase else 0, _ptr(w), w.shape[0],
                                                  _ptr(out), None, _stream(self.device)), "aiqmc_param_grad_weighted")
        return out

    def phase_param_grad(self, pos: torch.Tensor, weights: Optional[torch.Tensor] = None,
                         want_phase: bool = False):
        """d phase / d theta (phase = arg det A), same conventions as logpsi_param_grad."""
        p = self._pos(pos)
        B = p.shape[0]
        w = None
        if weights is not None:
            w = weights.to(self.device, self.dtype).contiguous()
            if w.numel() != B:
                raise ValueError("weights must have one entry per walker")
            out = torch.empty(self.nparams, dtype=self.dtype, device=self.device)
        else:
            out = torch.empty(B, self.nparams, dtype=self.dtype, device=self.device)
        ph = torch.empty(B, dtype=self.dtype, device=self.device) if want_phase else None
        check(self._lib.aiqmc_phase_param_grad(self._h, _ptr(p), B, _ptr(w), _ptr(out), _ptr(ph),
                                               _stream(self.device)), "aiqmc_phase_param_grad")
        return (out, ph) if want_phase else out

    # -- DMC (DMC/drift_diffusion.py, S_matrix.py, dmc.py, branch.py) -------------
    def dmc_drift_diffusion(self, pos: torch.Tensor, tstep: float, gauss1=None, gauss2=None, u=None, seed: int = 0,
                            offset: int = 0):
        """In-place drift-diffusion step; returns (grad_eff_old, grad_new_eff, tdamp[3] float64)."""
        if not (pos.is_cuda and pos.dtype == self.dtype and pos.is_contiguous()):
            raise ValueError("dmc_drift_diffusion needs a contiguous device tensor of the context dtype")
        B = pos.numel() // (3 * self.N)
        if B * 3 * self.N != pos.numel():
            raise ValueError(f"positions must hold whole walkers of 3N={3 * self.N} coordinates")
        host = gauss1 is not None
        if host != (gauss2 is not None) or host != (u is not None):
            raise ValueError("gauss1, gauss2 and u are injected together or not at all")
        g1 = self._dev(gauss1, B * 3 * self.N) if host else None      # [1, B, 3N]
        g2 = self._dev(gauss2, B * self.N * 3) if host else None      # [1, B, N, 3] (diagonal blocks)
        uu = self._dev(u, B * self.N) if host else None               # [1, B, N]
        go = torch.empty(B, 3 * self.N, dtype=self.dtype, device=self.device)
        gn = torch.empty_like(go)
        td = torch.zeros(3, dtype=torch.float64, device=self.device)
        check(self._lib.aiqmc_dmc_drift_diffusion(self._h, _ptr(pos), B, float(tstep),
                                                  AIQMC_RNG_HOST if host else AIQMC_RNG_PHILOX, _ptr(g1), _ptr(g2),
                                                  _ptr(uu), ctypes.c_uint64(seed), ctypes.c_uint64(offset), _ptr(go),
                                                  _ptr(gn), _ptr(td), _stream(self.device)), "aiqmc_dmc_drift_diffusion")
        return go, gn, td

    def _real_dev(self, t, n: int, what: str) -> torch.Tensor:
        t = torch.as_tensor(t)
        t = t.real if torch.is_complex(t) else t
        t = t.to(self.device, self.dtype).contiguous()
        if t.numel() != n:
            raise ValueError(f"{what}: expected {n} values, got {t.numel()}")
        return t

    def _grad_arg(self, g: torch.Tensor, B: int, what: str) -> torch.Tensor:
        if not (isinstance(g, torch.Tensor) and g.is_cuda and g.dtype == self.dtype):
            raise ValueError(f"{what} must be a device tensor of the context dtype {self.dtype}")
        if g.numel() != B * 3 * self.N:
            raise ValueError(f"{what}: expected {B * 3 * self.N} values, got {g.numel()}")
        return g.contiguous()

    def dmc_weights(self, weights: torch.Tensor, eloc_old, eloc_new, grad_eff_old, grad_new_eff, tdamp, tstep: float,
                    e_trial, e_est, branchcut: float, cut_minima: Optional[torch.Tensor] = None):
        """weights *= exp(tau tdamp (S_new + S_old) / 2), in place (S_matrix.py:4-24, dmc.py:88-92).
        e_trial / e_est: scalars, or per-walker [B] values (the driver's first block);
        cut_minima: optional device float64[2] global e_cut minima (multi-GPU, dmc_cut_minima)."""
        B = weights.numel()
        if not (weights.is_cuda and weights.dtype == self.dtype and weights.is_contiguous()):
            raise ValueError("weights must be a contiguous device tensor of the context dtype (updated in place)")
        eo = self._real_dev(eloc_old, B, "eloc_old")
        en = self._real_dev(eloc_new, B, "eloc_new")
        go = self._grad_arg(grad_eff_old, B, "grad_eff_old")
        gn = self._grad_arg(grad_new_eff, B, "grad_new_eff")
        if not (isinstance(tdamp, torch.Tensor) and tdamp.is_cuda and tdamp.dtype == torch.float64 and tdamp.numel() == 3):
            raise ValueError("tdamp must be the device float64[3] of dmc_drift_diffusion")
        et_b = ee_b = None
        if torch.is_tensor(e_trial) and e_trial.numel() > 1:
            et_b = self._real_dev(e_trial, B, "e_trial")
            e_trial = 0.0
        if torch.is_tensor(e_est) and e_est.numel() > 1:
            ee_b = self._real_dev(e_est, B, "e_est")
            e_est = 0.0
        e_trial = complex(e_trial).real if not torch.is_tensor(e_trial) else complex(e_trial.item()).real
        e_est = complex(e_est).real if not torch.is_tensor(e_est) else complex(e_est.item()).real
        cm = None
        if cut_minima is not None:
            if not (cut_minima.is_cuda and cut_minima.dtype == torch.float64 and cut_minima.numel() == 2):
                raise ValueError("cut_minima must be a device float64[2]")
            cm = cut_minima.contiguous()
        check(self._lib.aiqmc_dmc_weights_ex(self._h, B, _ptr(eo), _ptr(en), _ptr(go), _ptr(gn), _ptr(tdamp),
                                             float(tstep), _ptr(et_b), _ptr(ee_b), float(e_trial), float(e_est),
                                             float(branchcut), _ptr(cm), _ptr(weights), _stream(self.device)),
              "aiqmc_dmc_weights_ex")
        return weights

    def dmc_cut_minima(self, eloc_old, eloc_new, e_est, branchcut: float) -> torch.Tensor:
        """This batch's e_cut minima [2] (float64, device) for eloc_old / eloc_new (S_matrix.py:21-22);
        a multi-GPU driver all-reduces them with MIN (the reference's jnp.min spans all devices)."""
        eo = torch.as_tensor(eloc_old)
        B = eo.numel()
        eo = self._real_dev(eo, B, "eloc_old")
        en = self._real_dev(eloc_new, B, "eloc_new")
        ee_b = None
        if torch.is_tensor(e_est) and e_est.numel() > 1:
            ee_b = self._real_dev(e_est, B, "e_est")
            e_est = 0.0
        e_est = complex(e_est).real if not torch.is_tensor(e_est) else complex(e_est.item()).real
        out = torch.empty(2, dtype=torch.float64, device=self.device)
        check(self._lib.aiqmc_dmc_cut_minima(self._h, B, _ptr(eo), _ptr(en), _ptr(ee_b), float(e_est),
                                             float(branchcut), _ptr(out), _stream(self.device)), "aiqmc_dmc_cut_minima")
        return out

    def dmc_branch(self, weights: torch.Tensor, u: float):
        """Stochastic comb (branch.py:10-33): (new uniform weight [1], newinds [B] int32)."""
        B = weights.numel()
        w = weights.to(self.device, self.dtype).contiguous()
        idx = torch.empty(B, dtype=torch.int32, device=self.device)
        wo = torch.empty(1, dtype=self.dtype, device=self.device)
        check(self._lib.aiqmc_dmc_branch(self._h, B, _ptr(w), float(u), _ptr(idx), _ptr(wo), _stream(self.device)),
              "aiqmc_dmc_branch")
        return wo, idx

    def dmc_tmoves(self, pos: torch.Tensor, tstep: float, rot=None, u_sel=None, u_acc=None, seed: int = 0,
                   offset: int = 0):
        """In-place T-moves (DMC/Tmoves.py:32-225) on `pos`; returns the acceptance [B, N].
        rot [B,3,3], u_sel [B], u_acc [B,N]: injected draws (parity mode); all None: Philox."""
        if not (pos.is_cuda and pos.dtype == self.dtype and pos.is_contiguous()):
            raise ValueError("dmc_tmoves needs a contiguous device tensor of the context dtype (updated in place)")
        B = pos.numel() // (3 * self.N)
        host = rot is not None
        if host != (u_sel is not None) or host != (u_acc is not None):
            raise ValueError("rot, u_sel and u_acc are injected together or not at all")
        dev = lambda t, n: None if t is None else self._dev(t, n)
        r, us, ua = dev(rot, 9 * B), dev(u_sel, B), dev(u_acc, B * self.N)
        acc = torch.empty(B, self.N, dtype=self.dtype, device=self.device)
        check(self._lib.aiqmc_dmc_tmoves(self._h, _ptr(pos), B, float(tstep), AIQMC_RNG_HOST if host else
                                         AIQMC_RNG_PHILOX, _ptr(r), _ptr(us), _ptr(ua), ctypes.c_uint64(seed),
                                         ctypes.c_uint64(offset), _ptr(acc), _stream(self.device)),
              "aiqmc_dmc_tmoves")
        return acc

    def _dev(self, t, n: int) -> torch.Tensor:
        t = torch.as_tensor(t).to(self.device, self.dtype).contiguous()
        if t.numel() != n:
            raise ValueError(f"expected {n} values, got {t.numel()}")
        return t

    def set_ecp(self, rn_local, local_coes, local_exps, rn_non_local, non_local_coes, non_local_exps,
                list_l: int):
        """Pseudopotential tables in the reference drivers' shapes (single_atom_C.py:13-23):
        rn_local/local_coes/local_exps [A][KL], rn_non_local/... [A][list_l+1][KN]."""
        A = self.A
        loc = [np.ascontiguousarray(np.asarray(a, np.float64).reshape(A, -1)) for a in
               (rn_local, local_coes, local_exps)]
        nl = [np.ascontiguousarray(np.asarray(a, np.float64).reshape(A, int(list_l) + 1, -1)) for a in
              (rn_non_local, non_local_coes, non_local_exps)]
        if len({a.shape for a in loc}) != 1 or len({a.shape for a in nl}) != 1:
            raise ValueError("ECP tables of one kind must share their shape")
        self._ecp_keep = loc + nl
        e = AiqmcEcp()
        e.list_l = int(list_l)
        e.n_local = loc[0].shape[1]
        e.n_nonlocal = nl[0].shape[2]
        dp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        e.rn_local, e.local_coes, e.local_exps = (dp(a) for a in loc)
        e.rn_non_local, e.non_local_coes, e.non_local_exps = (dp(a) for a in nl)
        with torch.cuda.device(self.device):
            check(self._lib.aiqmc_set_ecp(self._h, ctypes.byref(e)), "aiqmc_set_ecp")

    def local_energy_ecp(self, pos: torch.Tensor, rot: Optional[torch.Tensor] = None, seed: int = 0,
                         offset: int = 0, want_quadrature: bool = False, complex_output: bool = False):
        """Complex pseudopotential local energy [B] (pphamiltonian.py:177-188).  rot [B,3,3]:
        injected rotations (parity mode); None: Philox Haar draws from (seed, offset).
        complex_output: with the kinetic energy's phase terms (pphamiltonian.py:84-104)."""
        p = self._pos(pos)
        B = p.shape[0]
        er = torch.empty(B, dtype=self.dtype, device=self.device)
        ei = torch.empty(B, dtype=self.dtype, device=self.device)
        r = None
        if rot is not None:
            r = rot.to(self.device, self.dtype).contiguous()
            if r.numel() != 9 * B:
                raise ValueError("rot must be [B,3,3]")
        nq = B * self.N * self.A * ECP_NQ
        lq = torch.empty(nq, dtype=self.dtype, device=self.device) if want_quadrature else None
        pq = torch.empty(nq, dtype=self.dtype, device=self.device) if want_quadrature else None
        mode = AIQMC_RNG_HOST if r is not None else AIQMC_RNG_PHILOX
        if complex_output:
            if want_quadrature:
                raise ValueError("want_quadrature is not available with complex_output")
            check(self._lib.aiqmc_local_energy_ecp_complex(self._h, _ptr(p), B, mode, _ptr(r), ctypes.c_uint64(seed),
                                                           ctypes.c_uint64(offset), _ptr(er), _ptr(ei),
                                                           _stream(self.device)), "aiqmc_local_energy_ecp_complex")
        else:
            check(self._lib.aiqmc_local_energy_ecp(self._h, _ptr(p), B, mode, _ptr(r), ctypes.c_uint64(seed),
                                                   ctypes.c_uint64(offset), _ptr(er), _ptr(ei), _ptr(lq), _ptr(pq),
                                                   _stream(self.device)), "aiqmc_local_energy_ecp")
        e = torch.complex(er, ei)
        if want_quadrature:
            return e, lq.reshape(B, self.N, self.A, ECP_NQ), pq.reshape(B, self.N, self.A, ECP_NQ)
        return e

    def mc_step(self, pos: torch.Tensor, nsteps: int, tstep: float, gauss1=None, gauss2=None, u=None,
                seed: int = 0, offset: int = 0, count_accepts: bool = False):
        """In-place Metropolis on `pos` (must be a contiguous device tensor of ctx dtype)."""
        if not (pos.is_cuda and pos.dtype == self.dtype and pos.is_contiguous()):
            raise ValueError("mc_step needs a contiguous device tensor of the context dtype (updated in place)")
        B = pos.numel() // (3 * self.N)
        host = gauss1 is not None
        acc = torch.zeros(B, dtype=torch.int32, device=self.device) if count_accepts else None
        if host:
            g1 = gauss1.to(self.device, self.dtype).contiguous()
            g2 = gauss2.to(self.device, self.dtype).contiguous()
            uu = u.to(self.device, self.dtype).contiguous()
            if g1.numel() != nsteps * B * 3 * self.N or g2.numel() != nsteps * B * self.N * 3 or \
                    uu.numel() != nsteps * B * self.N:
                raise ValueError("host draws have the wrong size")
        else:
            g1 = g2 = uu = None
        check(self._lib.aiqmc_mc_step(self._h, _ptr(pos), B, int(nsteps), float(tstep),
                                      AIQMC_RNG_HOST if host else AIQMC_RNG_PHILOX,
                                      _ptr(g1), _ptr(g2), _ptr(uu), ctypes.c_uint64(seed),
                                      ctypes.c_uint64(offset), _ptr(acc), _stream(self.device)),
              "aiqmc_mc_step")
        return acc
