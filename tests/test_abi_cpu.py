"""CPU checks of the drop-in boundary: the C-ABI library builds, loads and exports every
entry point include/f16env.h declares; the Python mirror matches the header; the product
package never reaches into oracle/ (no CPU fallback)."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "f16env.h")


def declared_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(f16env_\w+)\s*\(", src)))


@pytest.fixture(scope="module")
def so_path():
    from f16_jsb_amd.build import build
    return build()


def test_library_exports_every_declared_symbol(so_path):
    out = subprocess.run(["nm", "-D", "--defined-only", so_path], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (f16env_\w+)", out))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing


def test_library_loads_without_gpu(so_path):
    from f16_jsb_amd import _lib
    L = _lib.lib()  # imports torch first, then dlopens libf16env.so
    for name in declared_functions():
        assert hasattr(L, name)
    assert set(_lib.EXPORTED_SYMBOLS) == set(declared_functions())
    # pure functions need no device
    assert L.f16env_step_kernel_name(None) == b""  # no handle, no kernel
    s = L.f16env_state_bytes_per_env()
    assert 200 <= s <= 400
    assert L.f16env_algorithmic_bytes_per_env_step(4) == 16 + 60 * 4 + 60 * 3 + 4 + 2 + 2 * s
    # the windowed step's moved bytes (bench.py's roofline basis): the state read whole, written
    # back without its per-episode column (goal, episode count) except by the lanes it reset
    from f16_jsb_amd.abi import algorithmic_bytes_per_env_step
    assert algorithmic_bytes_per_env_step(4, s, "window") == 16 + 2 * 60 + 4 + 2 + s + (s - 16)
    assert algorithmic_bytes_per_env_step(10, 256, "window") == 638
    assert algorithmic_bytes_per_env_step(4, 256) == 954  # SURVEY 8(d)'s B(4), the contract


def test_config_default_matches_python_mirror(so_path):
    from f16_jsb_amd import _lib
    from f16_jsb_amd.abi import EnvConfig, config_default
    c = EnvConfig()
    assert _lib.lib().f16env_config_default(ctypes.byref(c)) == 0
    p = config_default()
    for f, _ in EnvConfig._fields_:
        a, b = getattr(c, f), getattr(p, f)
        if f in ("ic", "ic_lo", "ic_hi"):
            assert list(a) == list(b), f
        else:
            assert a == b, f


def test_header_enums_match_python_mirror():
    from f16_jsb_amd import abi
    src = open(HDR).read()
    for name, val in re.findall(r"\b(F16C_\w+)\s*=\s*(\d+)", src):
        assert getattr(abi, name) == int(val), name
    ic_names = re.findall(r"^\s+(F16_IC_\w+)\s*[,=]", src, re.M)
    assert [getattr(abi, n) for n in ic_names] == list(range(len(ic_names)))
    for name, val in re.findall(r"#define (F16_FLAG_\w+)\s+(0x[0-9a-fA-F]+)", src):
        assert getattr(abi, name) == int(val, 16), name
    assert f"#define F16ENV_ABI_VERSION {abi.F16ENV_ABI_VERSION}" in src
    assert abi.F16_IC_N == 19 and abi.F16C_N == 75
    assert "#define F16_OBS_DIM 15" in src


def test_create_without_gpu_fails_loudly(so_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd._lib import F16EnvError
    with pytest.raises(F16EnvError):
        F16Envs(4)


def test_null_handle_calls_return_errors(so_path):
    """Every handle-taking entry point of the windowed / features ABI refuses a NULL handle or
    a bad argument with a negative status and a message (no device needed, nothing launched)."""
    from f16_jsb_amd import _lib
    L = _lib.lib()
    assert L.f16env_set_window_order(None, 1) < 0
    assert L.f16env_window_bind(None, None, None, 8, None, None, None, None, None) < 0
    assert L.f16env_window_step_bound(None, None, None, 0, 3) < 0
    assert L.f16env_step_window_nt(None) == -1
    assert L.f16env_step_window_waves_per_simd(None) == 0
    assert L.f16env_step_window(None, None, None, None, None, 8, 3, None, None, None, None, None, None, None) < 0
    assert L.f16env_profile_times(None, None, 4) < 0
    assert L.f16env_window_restart(None, None, None, None, 8, 7) < 0
    assert L.f16env_reset_window(None, None, None, None, None, None, 8, 3) < 0
    # ABI 6
    assert L.f16env_window_resets_deferred(None) < 0
    assert L.f16env_sample_actions_steps(None, None, 1, 0, 4, None) < 0
    # features on a strided block: bad shapes / strides are refused before any launch
    assert L.f16env_features_strided(None, 4, 0, None, 16, 16, None) < 0
    assert L.f16env_features_strided(None, 4, 2, None, -1, 16, None) < 0
    assert L.f16env_features_strided(None, 0, 2, None, 16, 16, None) == 0  # empty: nothing to do
    assert L.f16env_last_error()


def test_product_never_imports_oracle(so_path):
    """No code path of the product reaches the oracle: no Python import of it, no #include
    of oracle/ sources, and libf16env.so does not link it."""
    pkg = os.path.join(ROOT, "f16_jsb_amd")
    for dp, _, files in os.walk(pkg):
        for f in files:
            txt = open(os.path.join(dp, f), errors="ignore").read() if f.endswith((".py", ".hip", ".h")) else ""
            assert not re.search(r"^\s*(import|from)\s+\S*oracle", txt, re.M), f
            assert not re.search(r"#include\s+\S*oracle", txt), f
            assert "f16ref_" not in txt, f
    needed = subprocess.run(["readelf", "-d", so_path], capture_output=True, text=True).stdout
    assert "f16ref" not in needed


def test_spaces_match_reference_bounds():
    from f16_jsb_amd import spaces
    obs = spaces.observation_space(10)
    assert obs.shape == (10, 15) and obs.dtype == np.float32
    assert obs.low[0, 3] == 0 and obs.high[0, 4] == np.float32(np.pi + 1e-5)
    assert obs.low[0, 10] == np.float32(-np.pi / 2 - 1e-5)
    act = spaces.action_space()
    np.testing.assert_array_equal(act.low, [-1, -1, -1, 0])
    np.testing.assert_array_equal(act.high, [1, 1, 1, 1])
