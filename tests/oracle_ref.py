"""ctypes binding of the CPU oracle (oracle/_build/libf16ref.so).

TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
import this module. The product path (f16_jsb_amd) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from f16_jsb_amd.abi import (F16C_N, F16_IC_N, F16_OBS_DIM, EnvConfig, config_default)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# F16REF_LIB: another build of the oracle, e.g. the ASan/UBSan one (oracle/Makefile `sanitize`)
LIB_PATH = os.environ.get("F16REF_LIB") or os.path.join(ROOT, "oracle", "_build", "libf16ref.so")

_lib = None


def build_oracle(quiet: bool = True) -> str:
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build_oracle()
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, u64, dp = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_double
        L.f16ref_create.restype = vp
        L.f16ref_create.argtypes = [ctypes.POINTER(EnvConfig)]
        L.f16ref_destroy.argtypes = [vp]
        L.f16ref_reset.argtypes = [vp, vp, vp, vp, vp]
        L.f16ref_step.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.f16ref_get_state.argtypes = [vp, vp]
        L.f16ref_set_state.argtypes = [vp, vp]
        L.f16ref_trim.argtypes = [vp, vp, vp, vp]
        L.f16ref_sample_actions.argtypes = [vp, u64, u64, vp]
        L.f16ref_philox4x32.argtypes = [vp, vp, vp]
        L.f16ref_atmosphere.argtypes = [dp, vp]
        L.f16ref_geodetic_to_ecef.argtypes = [dp, dp, dp, vp]
        L.f16ref_geodetic_altitude.argtypes = [vp]
        L.f16ref_geodetic_altitude.restype = dp
        L.f16ref_vcas_kts.argtypes = [dp, dp]
        L.f16ref_vcas_kts.restype = dp
        L.f16ref_aero_table.argtypes = [i32, dp, dp]
        L.f16ref_aero_table.restype = dp
        L.f16ref_n_aero_fns.restype = i32
        L.f16ref_threads.restype = i32
        L.f16ref_set_threads.argtypes = [i32]
        L.f16ref_obs_bounds_count.argtypes = [vp]
        L.f16ref_obs_bounds_count.restype = u64
        L.f16ref_set_threads.restype = i32
        L.f16ref_set_physics_mask.argtypes = [i32]
        L.f16ref_get_physics_mask.restype = i32
        L.f16ref_mass_props.argtypes = [vp, vp]
        for name in ("f16ref_kinematic", "f16ref_pid", "f16ref_aero_scale", "f16ref_seek"):
            getattr(L, name).restype = dp
        L.f16ref_kinematic.argtypes = [dp, dp, vp, vp, i32, dp, i32]
        L.f16ref_pid.argtypes = [dp, vp, vp, dp, dp, dp, dp, dp, i32]
        L.f16ref_aero_scale.argtypes = [dp, dp, dp, dp, dp]
        L.f16ref_seek.argtypes = [dp, dp, dp, dp, dp]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class OracleEnvs:
    """Batch of N envs on the CPU oracle, numpy in/out, same layout as the HIP ABI."""

    def __init__(self, n_envs=1, stack_k=10, **kw):
        self.cfg = config_default(n_envs=n_envs, stack_k=stack_k, **kw)
        self.n = n_envs
        self.k = stack_k
        self._h = lib().f16ref_create(ctypes.byref(self.cfg))

    def close(self):
        if self._h:
            lib().f16ref_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, mask=None, goals=None, ic=None):
        obs = np.zeros((self.n, self.k, F16_OBS_DIM), np.float32)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        g = None if goals is None else np.ascontiguousarray(goals, np.float32)
        c = None if ic is None else np.ascontiguousarray(ic, np.float64)
        lib().f16ref_reset(self._h, _p(m), _p(g), _p(c), _p(obs))
        return obs

    def step(self, act):
        act = np.ascontiguousarray(act, np.float32)
        n, k = self.n, self.k
        obs = np.zeros((n, k, F16_OBS_DIM), np.float32)
        rew = np.zeros(n, np.float32)
        term = np.zeros(n, np.uint8)
        trunc = np.zeros(n, np.uint8)
        tobs = np.zeros((n, k, F16_OBS_DIM), np.float32)
        eret = np.zeros(n, np.float64)
        elen = np.zeros(n, np.int32)
        lib().f16ref_step(self._h, _p(act), _p(obs), _p(rew), _p(term), _p(trunc), _p(tobs),
                          _p(eret), _p(elen))
        return obs, rew, term.astype(bool), trunc.astype(bool), tobs, eret, elen

    def get_state(self):
        s = np.zeros((self.n, F16C_N), np.float64)
        lib().f16ref_get_state(self._h, _p(s))
        return s

    def set_state(self, s):
        s = np.ascontiguousarray(s, np.float64)
        assert s.shape == (self.n, F16C_N)
        lib().f16ref_set_state(self._h, _p(s))

    def trim(self, ic):
        ic = np.ascontiguousarray(ic, np.float64)
        out = np.zeros_like(ic)
        res = np.zeros((self.n, 3), np.float64)
        lib().f16ref_trim(self._h, _p(ic), _p(out), _p(res))
        return out, res

    @property
    def obs_bounds_count(self):
        return int(lib().f16ref_obs_bounds_count(self._h))

    def sample_actions(self, seed, step):
        a = np.zeros((self.n, 4), np.float32)
        lib().f16ref_sample_actions(self._h, seed, step, _p(a))
        return a


def atmosphere(h_ft):
    out = np.zeros(4)
    lib().f16ref_atmosphere(float(h_ft), _p(out))
    return out


def philox(key, ctr):
    k = np.ascontiguousarray(key, np.uint32)
    c = np.ascontiguousarray(ctr, np.uint32)
    o = np.zeros(4, np.uint32)
    lib().f16ref_philox4x32(_p(k), _p(c), _p(o))
    return o


def default_ic():
    return np.array(config_default().ic[:F16_IC_N], np.float64)
