"""ctypes binding of libhbx.so (include/hbx.h).

The library is the product: if it is missing or does not load, every entry
point raises -- there is no CPU fallback anywhere in ``hbx``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HBX_LIB", os.path.join(_HERE, "libhbx.so"))

# constants mirrored from include/hbx.h
ABI_VERSION = 14
OK = 0
ERR_INVALID, ERR_HIP, ERR_UNSUPPORTED, ERR_NOMEM = -1, -2, -3, -4
TF_ASM, TF_FRESNEL = 0, 1
FIELD_AMPLITUDE, FIELD_PHASE = 0, 1
REL_NONE, REL_LSQ = 0, 1
ACCEPT_ENV, ACCEPT_DBS = 0, 1
REWARD_PSNR, REWARD_IMPORTANCE = 0, 1
MAX_GROUPS = 4
WALK_MAX_K = 256           # hbx_dbs_walk_psf speculation depth bound
WALK_FUSED_K = (1, 2, 3, 4)   # one launch per batch (two accepts resolved for K = 2..4)
PRECISION_F32, PRECISION_BF16_STORE, PRECISION_F16_STORE = 0, 1, 2   # hbx_plan_set_precision
OBS_STATE, OBS_RECON, OBS_RESOLVE, OBS_SETTLE = 1, 2, 4, 8   # hbx_env_obs_sync
SRC_U8, SRC_F32, SRC_F64 = 0, 1, 2             # hbx_pack_mask / hbx_rel_stats value kinds (ABI v14)
PACK_BINARY, PACK_THRESHOLD = 0, 1
REL_WORKSPACE_DOUBLES = 3072

EXPORTED_SYMBOLS = (
    "hbx_abi_version", "hbx_last_error", "hbx_plan_create", "hbx_plan_destroy",
    "hbx_plan_workspace_bytes", "hbx_plan_pipeline", "hbx_propagate", "hbx_psnr", "hbx_env_reset", "hbx_env_step",
    "hbx_step", "hbx_eval_flips", "hbx_commit_flip", "hbx_plan_set_timing", "hbx_plan_set_timing_sampled", "hbx_plan_read_timing",
    "hbx_env_step_psf", "hbx_field_refresh", "hbx_simulate", "hbx_flip_map",
    "hbx_eval_flips_psf", "hbx_commit_flip_psf", "hbx_dbs_walk_psf",
    "hbx_plan_set_precision", "hbx_plan_precision", "hbx_env_obs_sync",
    "hbx_planes_fill", "hbx_eval_flips_planes", "hbx_commit_flip_planes", "hbx_dbs_walk_planes",
    "hbx_dbs_walk_planes_fill", "hbx_host_alloc", "hbx_host_free", "hbx_pack_mask", "hbx_rel_stats",
)
NUM_PASSES = 5
PASS_NAMES = ("k_rowfwd", "k_col", "k_rowinv", "k_psf_eval", "k_psf_commit")
# hbx_plan_pipeline: the three-pass pipeline is the only one built since ABI v8 (the
# bits -> column and composed-896 variants measured slower and were removed)
PIPE_THREE_PASS = 0
PIPE_PASS_NAMES = {PIPE_THREE_PASS: PASS_NAMES}


class HbxError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where} failed ({code}): {msg}")
        self.code = code


class Optics(C.Structure):
    _fields_ = [
        ("height", C.c_int32), ("width", C.c_int32), ("groups", C.c_int32), ("planes", C.c_int32),
        ("wavelength", C.c_double * MAX_GROUPS),
        ("dx", C.c_double), ("dy", C.c_double), ("z", C.c_double),
        ("tf_kind", C.c_int32), ("field_kind", C.c_int32), ("rel_scale", C.c_int32),
        ("reserved", C.c_int32), ("peak", C.c_double),
    ]


class DbsWalk(C.Structure):
    """hbx_dbs_walk_t (include/hbx.h): device-resident greedy DBS walk state."""
    _fields_ = [
        ("pos", C.c_int64), ("total", C.c_int64), ("accepted", C.c_int64), ("batches", C.c_int64),
        ("prev_psnr", C.c_double), ("init_psnr", C.c_double), ("last_psnr", C.c_double),
        ("stop_diff", C.c_double),
        ("stop_enabled", C.c_int32), ("refresh_every", C.c_int32), ("done", C.c_int32), ("halt", C.c_int32),
        ("stopped_early", C.c_int32), ("commit_ch", C.c_int32), ("commit_pix", C.c_int32),
        ("commit2_ch1", C.c_int32), ("commit_pix2", C.c_int32), ("split_ch1", C.c_int32),
        ("split_pix", C.c_int32), ("fault", C.c_int32),
    ]


class EnvBuffers(C.Structure):
    _fields_ = [
        ("mask", C.c_void_p), ("record", C.c_void_p), ("target", C.c_void_p),
        ("chan_stats", C.c_void_p), ("init_psnr", C.c_void_p), ("prev_psnr", C.c_void_p),
        ("max_psnr_diff", C.c_void_p), ("steps", C.c_void_p), ("flip_count", C.c_void_p),
        ("sustained", C.c_void_p), ("intensity", C.c_void_p), ("error", C.c_void_p),
        ("field", C.c_void_p),
        ("imp_changes", C.c_void_p), ("imp_values", C.c_void_p), ("t_psnr_diff", C.c_void_p),
        ("imp_count", C.c_int32), ("reserved", C.c_int32),
        ("state_bytes", C.c_void_p), ("recon", C.c_void_p), ("recon_pending", C.c_void_p),
        ("plane_inten", C.c_void_p), ("plane_slot", C.c_void_p),   # ABI v9 plane cache
        ("error_host", C.c_void_p),                                 # ABI v11 error mirror
    ]


class EnvParams(C.Structure):
    _fields_ = [
        ("max_steps", C.c_int64), ("t_psnr", C.c_double), ("t_steps", C.c_int64),
        ("t_psnr_diff", C.c_double), ("reward_weight", C.c_double),
        ("accept_rule", C.c_int32), ("reward_kind", C.c_int32),
    ]


_lib = None
_lock = threading.Lock()
VP, I32, I64 = C.c_void_p, C.c_int32, C.c_int64


def _declare(lib):
    lib.hbx_abi_version.restype = C.c_int
    lib.hbx_last_error.restype = C.c_char_p
    lib.hbx_plan_create.argtypes = [C.POINTER(VP), C.POINTER(Optics), I32, I32]
    lib.hbx_plan_destroy.argtypes = [VP]
    lib.hbx_plan_workspace_bytes.argtypes = [VP]
    lib.hbx_plan_workspace_bytes.restype = C.c_size_t
    lib.hbx_plan_pipeline.argtypes = [VP]
    lib.hbx_propagate.argtypes = [VP, VP, VP, I32, VP, VP, VP, VP]
    lib.hbx_psnr.argtypes = [VP, VP, I32, VP, VP]
    lib.hbx_env_reset.argtypes = [VP, C.POINTER(EnvBuffers), I32, VP, I32, VP]
    lib.hbx_env_step.argtypes = [VP, C.POINTER(EnvBuffers), C.POINTER(EnvParams), I32, VP, VP, VP,
                                 VP, VP, VP, VP, VP]
    lib.hbx_step.argtypes = [VP, VP, VP, I32, VP, VP, VP, VP, VP, I32, VP]
    lib.hbx_eval_flips.argtypes = [VP, VP, VP, VP, VP, I32, VP, VP, VP]
    lib.hbx_commit_flip.argtypes = [VP, VP, VP, VP, VP, VP, VP, VP, I32, VP]
    lib.hbx_env_step_psf.argtypes = [VP, C.POINTER(EnvBuffers), C.POINTER(EnvParams), I32, VP, VP, VP,
                                     VP, VP, VP, VP]
    lib.hbx_field_refresh.argtypes = [VP, C.POINTER(EnvBuffers), I32, VP, I32, VP]
    lib.hbx_simulate.argtypes = [VP, VP, I32, VP, VP, VP]
    lib.hbx_flip_map.argtypes = [VP, VP, VP, VP, VP, VP]
    lib.hbx_eval_flips_psf.argtypes = [VP, VP, VP, VP, VP, VP, VP, I32, VP, VP, VP]
    lib.hbx_commit_flip_psf.argtypes = [VP, VP, VP, VP, VP, VP, VP, VP, VP, VP, I32, VP]
    lib.hbx_dbs_walk_psf.argtypes = [VP, VP, VP, VP, VP, VP, VP, I64, VP, VP, VP, I64, I32, I32, VP]
    lib.hbx_plan_set_precision.argtypes = [VP, I32]
    lib.hbx_plan_precision.argtypes = [VP]
    lib.hbx_env_obs_sync.argtypes = [VP, C.POINTER(EnvBuffers), I32, VP, I32, I32, VP]
    lib.hbx_planes_fill.argtypes = [VP, VP, VP, VP, VP, I32, VP, VP, VP]
    lib.hbx_eval_flips_planes.argtypes = [VP, VP, VP, VP, VP, VP, I32, VP, I32, VP, VP, VP]
    lib.hbx_commit_flip_planes.argtypes = [VP, VP, VP, VP, VP, I32, VP, VP, VP, VP, I32, VP]
    lib.hbx_dbs_walk_planes.argtypes = [VP, VP, VP, VP, VP, VP, I32, VP, I64, VP, VP, VP, I64, I32, I32, VP]
    lib.hbx_dbs_walk_planes_fill.argtypes = [VP, VP, VP, VP, VP, VP, I32, VP, I64, VP, VP, VP, I64, I32, I32, VP,
                                             I64, I64, VP]
    lib.hbx_host_alloc.argtypes = [C.c_size_t, C.POINTER(VP), C.POINTER(VP)]
    lib.hbx_host_free.argtypes = [VP]
    lib.hbx_pack_mask.argtypes = [VP, I32, I64, I32, C.c_double, VP, VP, VP]
    lib.hbx_rel_stats.argtypes = [VP, VP, I32, I64, I32, C.c_double, VP, VP, VP]
    lib.hbx_plan_set_timing.argtypes = [VP, I32]
    lib.hbx_plan_set_timing_sampled.argtypes = [VP, I32, I32]
    lib.hbx_plan_read_timing.argtypes = [VP, C.POINTER(C.c_double), C.POINTER(C.c_int64),
                                         C.POINTER(C.c_int64)]
    for name in EXPORTED_SYMBOLS:
        if name not in ("hbx_last_error", "hbx_plan_workspace_bytes"):
            getattr(lib, name).restype = C.c_int


def load():
    """Load libhbx.so once (raises if absent: the HIP path is mandatory)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"libhbx.so not found at {LIB_PATH}; build it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
            lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
            _declare(lib)
            v = lib.hbx_abi_version()
            if v != ABI_VERSION:
                raise ImportError(f"libhbx ABI {v} != expected {ABI_VERSION}")
            _lib = lib
    return _lib


def check(rc: int, where: str):
    if rc != OK:
        msg = load().hbx_last_error().decode(errors="replace")
        raise HbxError(rc, where, msg)

