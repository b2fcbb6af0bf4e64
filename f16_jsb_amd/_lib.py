"""ctypes binding of libf16env.so (the HIP product path).

The library is built in-tree (f16_jsb_amd/libf16env.so, see build.py). torch is imported
first so that the process has exactly one HIP runtime (torch's libamdhip64.so.7, which
libf16env.so's NEEDED entry then resolves to). There is no CPU fallback: if the library is
missing, or no GPU is visible, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

from .abi import F16ENV_ABI_VERSION, EnvConfig, RolloutSlot

LIB_PATH = os.environ.get("F16ENV_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libf16env.so")

_lib = None


class F16EnvError(RuntimeError):
    pass


def _set(L, name, argtypes, restype):
    """Declare an entry point; tolerate its absence in an older build (tools/variant_sweep.py
    times earlier libraries side by side -- tests check the product exports every symbol)."""
    f = getattr(L, name, None)
    if f is not None:
        f.argtypes, f.restype = argtypes, restype


def lib():
    """Load libf16env.so (raises F16EnvError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  -- one HIP runtime per process (torch's)

    if not os.path.exists(LIB_PATH):
        raise F16EnvError(
            "libf16env.so not found at %s: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `python -m f16_jsb_amd.build`" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, u64, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_size_t
    L.f16env_config_default.argtypes = [ctypes.POINTER(EnvConfig)]
    L.f16env_config_cfg5.argtypes = [ctypes.POINTER(EnvConfig)]
    L.f16env_create.argtypes = [ctypes.POINTER(EnvConfig), i32, ctypes.POINTER(vp)]
    L.f16env_destroy.argtypes = [vp]
    L.f16env_state_bytes.argtypes = [vp]
    L.f16env_state_bytes.restype = sz
    L.f16env_state_bytes_per_env.restype = i32
    L.f16env_reset.argtypes = [vp, vp, vp, vp, vp, vp]
    L.f16env_step.argtypes = [vp] * 13
    _set(L, "f16env_step_rollout", [vp, vp, ctypes.POINTER(RolloutSlot)] + [vp] * 11, i32)
    i64 = ctypes.c_int64
    _set(L, "f16env_step_window", [vp, vp, vp, vp, vp, i64, i32] + [vp] * 7, i32)
    _set(L, "f16env_reset_window", [vp, vp, vp, vp, vp, vp, i64, i32], i32)
    _set(L, "f16env_window_restart", [vp, vp, vp, vp, i64, i32], i32)
    _set(L, "f16env_step_window_waves_per_simd", [vp], i32)
    _set(L, "f16env_step_mode", [vp], i32)
    _set(L, "f16env_features_strided", [vp, i64, i32, vp, i64, i64, vp], i32)
    _set(L, "f16env_features_window_step", [vp, i64, i32, i32, vp, i64, i64, vp, vp, vp, vp, i32, i32], i32)
    _set(L, "f16env_set_window_order", [vp, i32], i32)
    _set(L, "f16env_window_clear_fresh", [vp, vp], i32)
    _set(L, "f16env_window_bind", [vp, vp, vp, i64, vp, vp, vp, vp, vp], i32)
    _set(L, "f16env_window_step_bound", [vp, vp, vp, i32, i32], i32)
    _set(L, "f16env_window_feature_bind", [vp, vp, vp], i32)
    _set(L, "f16env_step_window_nt", [vp], i32)
    L.f16env_get_state.argtypes = [vp, vp, vp]
    L.f16env_nonfinite_count.argtypes = [vp, vp, ctypes.POINTER(u64)]
    _set(L, "f16env_obs_bounds_count", [vp, vp, ctypes.POINTER(u64)], i32)
    _set(L, "f16env_debug_checks", [vp, vp, ctypes.POINTER(ctypes.c_uint32)], i32)
    L.f16env_rollout_random.argtypes = [vp, vp, u64, u64, i32] + [vp] * 7
    _set(L, "f16env_window_rollout_random", [vp, vp, u64, u64, i32, i32, i32, i32] + [vp] * 5, i32)
    _set(L, "f16env_window_step_rollout", [vp, vp, ctypes.POINTER(RolloutSlot), vp, i32, i32], i32)
    _set(L, "f16env_window_step_ex", [vp, vp, vp, i32, i32, ctypes.c_uint32, u64, u64], i32)
    _set(L, "f16env_window_step_ex_kernel_name", [vp, ctypes.c_uint32], ctypes.c_char_p)
    _set(L, "f16env_window_poses_bind", [vp, vp], i32)
    _set(L, "f16env_window_resets_deferred", [vp], i32)
    _set(L, "f16env_sample_actions_steps", [vp, vp, u64, u64, i32, vp], i32)
    _set(L, "f16env_bootstrap_timeouts", [vp, i64, vp, vp, vp, vp, ctypes.c_double], i32)
    _set(L, "f16env_bootstrap_stash", [vp, i64, i32, vp, i64, i64, vp, vp, i64, vp, vp, vp, i64], i32)
    _set(L, "f16env_bootstrap_apply", [vp, i64, vp, vp, vp, ctypes.c_double], i32)
    _set(L, "f16env_abi_version", [], i32)
    L.f16env_set_state.argtypes = [vp, vp, vp]
    L.f16env_trim.argtypes = [vp, vp, vp, vp, vp]
    L.f16env_sample_actions.argtypes = [vp, vp, u64, u64, vp]
    L.f16env_gae.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, vp, vp, vp, vp, vp, ctypes.c_double,
                             ctypes.c_double, vp, vp]
    L.f16env_features.argtypes = [vp, ctypes.c_int64, vp, vp]
    _set(L, "f16env_poses", [vp, ctypes.c_int64, vp, ctypes.c_int64, vp], i32)
    L.f16env_step_kernel_name.argtypes = [vp]
    L.f16env_step_kernel_name.restype = ctypes.c_char_p
    _set(L, "f16env_profile_times", [vp, ctypes.POINTER(ctypes.c_double), i32], i32)
    L.f16env_step_waves_per_simd.argtypes = [vp]
    L.f16env_step_waves_per_simd.restype = i32
    _set(L, "f16env_step_variant", [vp], i32)
    _set(L, "f16env_profile_begin", [vp, i32], i32)
    _set(L, "f16env_profile_end", [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_int)], i32)
    L.f16env_algorithmic_bytes_per_env_step.argtypes = [i32]
    L.f16env_algorithmic_bytes_per_env_step.restype = ctypes.c_double
    L.f16env_last_error.restype = ctypes.c_char_p
    for name in ("f16env_config_default", "f16env_config_cfg5", "f16env_create", "f16env_destroy", "f16env_reset",
                 "f16env_step", "f16env_get_state", "f16env_set_state", "f16env_trim",
                 "f16env_sample_actions", "f16env_gae", "f16env_features", "f16env_rollout_random"):
        getattr(L, name).restype = i32
    # the header's F16ENV_ABI_VERSION must be the library's (a stale build behind a changed
    # signature would be called with the wrong arguments); libraries from before the version
    # export (ABI 2) load only when named explicitly through F16ENV_LIB (tools comparing builds)
    got = L.f16env_abi_version() if hasattr(L, "f16env_abi_version") else 2
    if got != F16ENV_ABI_VERSION and (got != 2 or not os.environ.get("F16ENV_LIB")):
        raise F16EnvError("%s has ABI version %d, this binding expects %d: rebuild it (python -m f16_jsb_amd.build)"
                          % (LIB_PATH, got, F16ENV_ABI_VERSION))
    _lib = L
    return L


def check(status: int, what: str):
    if status != 0:
        msg = lib().f16env_last_error()
        raise F16EnvError("%s failed (%d): %s" % (what, status, msg.decode() if msg else "?"))


# symbols include/f16env.h declares (tests check the .so exports every one of them)
EXPORTED_SYMBOLS = (
    "f16env_config_default", "f16env_config_cfg5", "f16env_create", "f16env_destroy", "f16env_state_bytes",
    "f16env_state_bytes_per_env", "f16env_reset", "f16env_step", "f16env_step_rollout", "f16env_nonfinite_count", "f16env_obs_bounds_count", "f16env_debug_checks", "f16env_rollout_random",
    "f16env_step_window", "f16env_reset_window", "f16env_window_restart", "f16env_step_window_waves_per_simd",
    "f16env_step_mode", "f16env_features_strided", "f16env_features_window_step", "f16env_set_window_order", "f16env_window_clear_fresh",
    "f16env_window_bind", "f16env_window_step_bound", "f16env_window_feature_bind", "f16env_step_window_nt", "f16env_window_step_rollout",
    "f16env_window_step_ex", "f16env_window_step_ex_kernel_name", "f16env_window_poses_bind",
    "f16env_window_resets_deferred", "f16env_sample_actions_steps",
    "f16env_window_rollout_random", "f16env_bootstrap_timeouts", "f16env_bootstrap_stash", "f16env_bootstrap_apply", "f16env_abi_version",
    "f16env_get_state",
    "f16env_set_state", "f16env_trim", "f16env_sample_actions", "f16env_gae", "f16env_features", "f16env_poses", "f16env_step_kernel_name", "f16env_step_waves_per_simd", "f16env_step_variant", "f16env_profile_begin", "f16env_profile_end", "f16env_profile_times",
    "f16env_algorithmic_bytes_per_env_step", "f16env_last_error",
)
