"""hbx -- MI355X-native binary-hologram environment (HIP kernels behind a C-ABI).

Public surface:
  OpticsConfig, mono_config, rgb_config, Plan     propagation operator (hbx_plan_t)
  HologramVecEnv, BinaryHologramEnv               env.py / env_1024_24.py drop-ins
  dbs.greedy, dbs.probe                           DBS*.py / range.py drivers
  dist                                            one-process-per-GPU sharding helpers
The torchOptics-compatible operator shim lives in the sibling package
``torchOptics`` (optics.Tensor / simulate / relativeLoss, metrics.get_PSNR).
"""
from . import _lib
from ._lib import (ACCEPT_DBS, ACCEPT_ENV, FIELD_AMPLITUDE, FIELD_PHASE, PRECISION_BF16_STORE,
                   PRECISION_F16_STORE, PRECISION_F32, REL_LSQ, REL_NONE, TF_ASM, TF_FRESNEL, HbxError)
from .plan import (OpticsConfig, Plan, crop, crop_bits, crop_config, mono_config, pack_bits, pack_mask, rgb_config,
                   unpack_bits)

__all__ = [
    "OpticsConfig", "Plan", "mono_config", "rgb_config", "pack_bits", "pack_mask", "unpack_bits", "crop", "crop_bits",
    "crop_config", "HbxError",
    "TF_ASM", "TF_FRESNEL", "FIELD_AMPLITUDE", "FIELD_PHASE", "REL_LSQ", "REL_NONE", "ACCEPT_ENV",
    "ACCEPT_DBS", "PRECISION_F32", "PRECISION_BF16_STORE", "PRECISION_F16_STORE", "load_library",
]


def load_library():
    """Load libhbx.so (raises ImportError if it was not built)."""
    return _lib.load()


def __getattr__(name):  # lazy: env / dbs pull torch tensors on a GPU
    if name in ("HologramVecEnv", "BinaryHologramEnv", "EnvState"):
        from . import env
        return getattr(env, name)
    if name in ("dbs", "dist", "env"):
        import importlib
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
