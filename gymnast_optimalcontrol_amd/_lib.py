"""ctypes binding of the C-ABI in include/gymnast_acrobot.h (libgymnast_acrobot.so).

The HIP library is the only compute path of this package.  If it is missing, or no HIP
device is visible, every compute entry point raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  -- load torch's HIP runtime first so the library binds to the same one

from . import _build

# GYM_LIB_PATH selects another build of the same library (measurement / diagnostic variants)
LIB_PATH = os.environ.get("GYM_LIB_PATH") or _build.LIB_PATH

# exported symbols, in include/gymnast_acrobot.h order (tests check every one is present)
EXPORTS = (
    "gym_abi_version", "gym_build_id", "gym_model_from_params",
    "gym_continuous_dynamics", "gym_rk4_step", "gym_jacobians", "gym_stage_cost_derivs",
    "gym_pack_lanes", "gym_unpack_lanes", "gym_unpack_gains",
    "gym_rollout_open_loop", "gym_closed_loop", "gym_total_cost", "gym_backward_sweep", "gym_linearize",
    "gym_riccati_general",
    "gym_newton_init", "gym_newton_iteration", "gym_newton_pipeline_split", "gym_newton_phase", "gym_newton_phase_kind",
    "gym_newton_run",
    "gym_newton_tail", "gym_newton_tail_scratch", "gym_newton_cand_scratch", "gym_newton_tail_lds",
    "gym_newton_finalize", "gym_newton_fill_states", "gym_placement_probe", "gym_newton_sigma",
    "gym_gamma_sweep", "gym_newton_gamma_sweep",
    "gym_tv_lqr_gains", "gym_dare_fixed_point", "gym_mpc_gains", "gym_lq_forward", "gym_track_rollout", "gym_track_rollout_ex",
    "gym_timing_create", "gym_timing_destroy", "gym_timing_collect",
)
KERNEL_KINDS = ("backward", "trial", "candidates", "retry", "stats", "phase_odd", "phase_even", "sigma", "run",
                "tail")

ABI_VERSION = 17        # GYM_ABI_VERSION of the header this binding mirrors
MAX_BP = 1 << 26         # GYM_MAX_BP
FLAG_U0_ZERO = 1         # GYM_FLAG_U0_ZERO
FLAG_X_CKPT = 2          # GYM_FLAG_X_CKPT
FLAG_RUN_SINGLE = 4      # GYM_FLAG_RUN_SINGLE
FLAG_REF_LANE = 8        # GYM_FLAG_REF_LANE
FLAG_SIGMA_STREAM = 16   # GYM_FLAG_SIGMA_STREAM
TRACK_SINGLE = 1         # GYM_TRACK_SINGLE
CKPT_INTERVAL = 4        # GYM_CKPT_INTERVAL

ACTIVE, CONVERGED, LS_FAILED, MAX_ITERS, PAD = 0, 1, 2, 3, 4
STATUS_NAMES = {ACTIVE: "active", CONVERGED: "converged", LS_FAILED: "ls_failed", MAX_ITERS: "max_iters", PAD: "pad"}


class GymModel(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("a", "b", "d", "g1", "g2", "f1", "f2", "dt")]


class GymWeights(C.Structure):
    _fields_ = [("Q", C.c_double * 4), ("R", C.c_double * 2), ("QT", C.c_double * 4)]


class GymArmijo(C.Structure):
    _fields_ = [("tol", C.c_double), ("beta", C.c_double), ("c", C.c_double), ("gamma0", C.c_double),
                ("max_ls", C.c_int32), ("record_history", C.c_int32)]


_P = C.c_void_p


TIMING_POOL = 512        # GYM_TIMING_POOL


class GymTiming(C.Structure):
    _fields_ = [("ev", _P * 20), ("ms", C.c_double * 10), ("launches", C.c_int64 * 10), ("pending", C.c_int32),
                ("pool_used", C.c_int32), ("pool_ev", _P * (2 * TIMING_POOL)), ("pool_kind", C.c_int32 * TIMING_POOL)]


class GymBatch(C.Structure):
    _fields_ = [("B", C.c_int64), ("Bp", C.c_int64), ("N", C.c_int32), ("hist_len", C.c_int32),
                ("flags", C.c_int32), ("pad", C.c_int32), ("x", _P * 2), ("u", _P * 2), ("K1", _P), ("cs", _P), ("x_ref", _P), ("u_ref", _P),
                ("cost", _P), ("dJ", _P), ("smax", _P), ("gamma", _P), ("status", _P), ("n_iter", _P),
                ("res_buf", _P), ("n_roll", _P), ("retry_list", _P), ("counters", _P), ("cand_ok", _P),
                ("partials", _P), ("stats", _P), ("hist_cost", _P), ("hist_smax", _P), ("lane_map", _P),
                ("timing", C.POINTER(GymTiming)), ("cand_scratch", _P), ("cand_slots", C.c_int64)]


_I64, _I32, _D = C.c_int64, C.c_int32, C.c_double
_MP, _WP, _AP, _BP = C.POINTER(GymModel), C.POINTER(GymWeights), C.POINTER(GymArmijo), C.POINTER(GymBatch)
_SIGS = {
    "gym_abi_version": [],
    "gym_model_from_params": [_P, _D, _MP],
    "gym_continuous_dynamics": [_MP, _P, _P, _P, _I64, _P],
    "gym_rk4_step": [_MP, _P, _P, _P, _I64, _P],
    "gym_jacobians": [_MP, _P, _P, _P, _P, _I64, _P],
    "gym_stage_cost_derivs": [_P, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _I64, _P],
    "gym_pack_lanes": [_P, _P, _I64, _I64, _I32, _I32, _I32, _P],
    "gym_unpack_lanes": [_P, _P, _P, _P, _I64, _I64, _I32, _I32, _I32, _P],
    "gym_unpack_gains": [_P, _P, _I64, _I64, _I32, _P],
    "gym_rollout_open_loop": [_MP, _WP, _P, _P, _P, _P, _P, _P, _I64, _I64, _I32, _P],
    "gym_closed_loop": [_MP, _WP, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I32, _P],
    "gym_total_cost": [_P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I32, _P],
    "gym_backward_sweep": [_MP, _WP, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I32, _P],
    "gym_linearize": [_MP, _WP, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I32, _P],
    "gym_riccati_general": [_P] * 12 + [_I64, _I64, _I32, _P],
    "gym_newton_init": [_MP, _WP, _P, _BP, _P],
    "gym_newton_iteration": [_MP, _WP, _AP, _BP, _I32, _P],
    "gym_newton_pipeline_split": [_BP, C.POINTER(C.c_int64)],
    "gym_newton_phase_kind": [_BP, C.POINTER(C.c_int32)],
    "gym_newton_phase": [_MP, _WP, _AP, _BP, _I32, _I32, _P],
    "gym_newton_run": [_MP, _WP, _AP, _BP, _I32, _I32, _P],
    "gym_newton_tail": [_MP, _WP, _AP, _BP, _P, _I32, _P, _I64, _I32, _I32, _P],
    "gym_newton_tail_scratch": [_I32, _I32, _I32, C.POINTER(C.c_int64)],
    "gym_newton_cand_scratch": [_I32, _I64, C.POINTER(C.c_int64)],
    "gym_newton_tail_lds": [_I32, C.POINTER(C.c_int64), C.POINTER(C.c_int64)],
    "gym_newton_finalize": [_MP, _WP, _BP, _I32, _P, _P, _P, _P, _P],
    "gym_newton_fill_states": [_MP, _BP, _I32, _P],
    "gym_placement_probe": [_BP, _I32, _P],
    "gym_newton_sigma": [_MP, _WP, _BP, _P, _P],
    "gym_gamma_sweep": [_MP, _WP, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _I64, _I64, _I32, _P],
    "gym_newton_gamma_sweep": [_MP, _WP, _AP, _BP, _I32, _P, _I32, _P, _P],
    "gym_tv_lqr_gains": [_P, _P, _I32, _P, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _D, _P, _P],
    "gym_dare_fixed_point": [_P, _P, _P, _P, _I32, _D, _P, _P, _P],
    "gym_mpc_gains": [_MP, _P, _P, _I32, _P, _P, _P, _P, _I32, _I32, _I32, _D, _P, _P, _P, _P],
    "gym_lq_forward": [_P, _P, _I32, _P, _P, _I32, _D, _P, _P, _I32, _P, _P, _P],
    "gym_track_rollout": [_MP, _P, _P, _P, _P, _I64, _I32, _P, _P, _P],
    "gym_track_rollout_ex": [_MP, _P, _P, _P, _P, _I64, _I32, _I32, _P, _P, _P],
    "gym_timing_create": [C.POINTER(GymTiming)],
    "gym_timing_destroy": [C.POINTER(GymTiming)],
    "gym_timing_collect": [C.POINTER(GymTiming)],
}

_libs: dict = {}


def load(path: str = LIB_PATH):
    """Load (once per path) and return the ctypes library.  Raises if the HIP library is not built."""
    if path not in _libs:
        if not os.path.exists(path):
            raise ImportError(
                f"{path} is missing: build the HIP library first (python -m gymnast_optimalcontrol_amd._build "
                "or __graft_entry__.build()); there is no CPU fallback")
        lib = C.CDLL(path)
        lib.gym_abi_version.restype = C.c_int
        if lib.gym_abi_version() != ABI_VERSION:
            raise ImportError(f"{path} implements ABI {lib.gym_abi_version()}, this binding needs {ABI_VERSION}: "
                              "rebuild the HIP library")
        lib.gym_build_id.restype = C.c_char_p
        lib.gym_build_id.argtypes = []
        have, want = lib.gym_build_id().decode(), _build.source_hash()
        if have != want and not os.environ.get("GYM_ALLOW_FOREIGN_BUILD"):
            raise ImportError(f"{path} was built from other sources (build id {have}, tree {want}): stale binary, "
                              "rebuild it (__graft_entry__.build() or python -m gymnast_optimalcontrol_amd._build)")
        for name, args in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = C.c_int
        _libs[path] = lib
    return _libs[path]


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed with HIP error code {rc}")


def require_device(device=None, lib_path: str = LIB_PATH) -> torch.device:
    """The compute path runs on a HIP device only."""
    if not torch.cuda.is_available():
        raise RuntimeError("gymnast_optimalcontrol_amd needs a HIP (ROCm) GPU: no device is visible "
                           "and there is no CPU fallback")
    load(lib_path)
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if dev.type != "cuda":
        raise ValueError(f"device must be a HIP device, got {dev}")
    return dev


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
