"""BASELINE cfg5 models on the CPU oracle: random-IC box draws and Gauss-Markov gusts
(include/f16env.h F16_FLAG_RANDOM_IC / F16_FLAG_GUSTS; the reference has neither, so these
are build-defined and pinned by the numpy restatement in rng_ref.py, not by the reference)."""
from __future__ import annotations

import ctypes
import math

import numpy as np

from f16_jsb_amd.abi import (CFG5_BOX, F16C_GUST, F16C_WIND, F16_IC_N, F16_IC_H_SL_FT, F16_IC_U_FPS,
                             F16_IC_WIND_N_FPS, F16_FLAG_NO_AUTORESET, config_default)
from oracle_ref import OracleEnvs
from rng_ref import gust_normals, philox4x32, random_ic


def test_numpy_philox_random123_kat():
    kat = [([0, 0], [0, 0, 0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
           ([0xFFFFFFFF] * 2, [0xFFFFFFFF] * 4, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
           ([0xA4093822, 0x299F31D0], [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
            [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1])]
    for key, ctr, want in kat:
        assert philox4x32(*key, *ctr).tolist() == want


def test_config_cfg5_c_matches_python():
    from f16_jsb_amd._lib import lib
    c = config_default(n_envs=3, stack_k=4)
    lib().f16env_config_cfg5(ctypes.byref(c))
    p = config_default(n_envs=3, stack_k=4, cfg5=True)
    assert bytes(c) == bytes(p)


def _cfg5_box():
    c = config_default(cfg5=True)
    return np.array(c.ic_lo[:F16_IC_N]), np.array(c.ic_hi[:F16_IC_N])


def test_random_ic_reset_equals_explicit_ic():
    """A RANDOM_IC reset is exactly a reset with the numpy-drawn IC vector."""
    n, seed = 64, 11
    lo, hi = _cfg5_box()
    a = OracleEnvs(n, stack_k=2, seed=seed, cfg5=True)
    b = OracleEnvs(n, stack_k=2, seed=seed, cfg5=True)
    oa = a.reset()
    ic = random_ic(seed, np.arange(n), 0, lo, hi)
    for j, (l, h) in CFG5_BOX.items():
        assert np.all((ic[:, j] >= l) & (ic[:, j] <= h))
    assert ic[:, F16_IC_H_SL_FT].std() > 1000.0
    ob = b.reset(ic=ic)
    np.testing.assert_array_equal(oa, ob)
    sa, sb = a.get_state(), b.get_state()
    np.testing.assert_array_equal(sa, sb)
    np.testing.assert_array_equal(sa[:, F16C_WIND:F16C_WIND + 3], ic[:, F16_IC_WIND_N_FPS:F16_IC_WIND_N_FPS + 3])
    # second episode draws a different IC (episode counter in the Philox counter)
    ob2 = a.reset()
    assert not np.array_equal(ob2[:, 0, :3], oa[:, 0, :3])
    np.testing.assert_array_equal(ob2, b.reset(ic=random_ic(seed, np.arange(n), 1, lo, hi)))


def test_gust_start_and_update_follow_the_numpy_stream():
    n, seed = 32, 5
    e = OracleEnvs(n, stack_k=1, seed=seed, cfg5=True, flags=F16_FLAG_NO_AUTORESET)
    e.reset()
    cfg = e.cfg
    g0 = e.get_state()[:, F16C_GUST:F16C_GUST + 3]
    np.testing.assert_allclose(g0, cfg.gust_sigma_fps * gust_normals(seed, np.arange(n), 0, 0), rtol=1e-13, atol=1e-12)
    a = math.exp(-cfg.down_sample * cfg.dt / cfg.gust_tau_s)
    b = cfg.gust_sigma_fps * math.sqrt(1 - a * a)
    g = g0
    for s in range(1, 4):
        e.step(np.zeros((n, 4), np.float32))
        g = a * g + b * gust_normals(seed, np.arange(n), 0, s)
        np.testing.assert_allclose(e.get_state()[:, F16C_GUST:F16C_GUST + 3], g, rtol=1e-12, atol=1e-11)


def test_gust_process_statistics():
    """Stationary std-dev sigma and lag-1 autocorrelation a = exp(-T/tau) of the gust stream."""
    n, T = 20000, 60
    cfg = config_default(cfg5=True)
    a = math.exp(-cfg.down_sample * cfg.dt / cfg.gust_tau_s)
    b = cfg.gust_sigma_fps * math.sqrt(1 - a * a)
    g = cfg.gust_sigma_fps * gust_normals(3, np.arange(n), 0, 0)
    xs = [g]
    for s in range(1, T):
        g = a * g + b * gust_normals(3, np.arange(n), 0, s)
        xs.append(g)
    x = np.stack(xs)  # (T, n, 3)
    assert abs(x.std() - cfg.gust_sigma_fps) < 0.05 * cfg.gust_sigma_fps
    assert abs(x.mean()) < 0.05
    r1 = np.mean(x[1:] * x[:-1]) / np.mean(x * x)
    assert abs(r1 - a) < 0.01
