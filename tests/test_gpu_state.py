"""The 256-byte state (f16_device.h column map) and the kernel families it selects.

  * canonical round trip: get_state -> set_state -> get_state is bit-exact on the GPU, except
    the Earth angle and calibrated airspeed that the canonical form re-encodes (to 1e-6); the
    latch fields recomputed at load (p/q/r-aero, ground speed) agree with the oracle's stored
    latch at fp32 round-off, and the fields the HIP path does not carry (N1, the g-load PID's
    previous input, body force x) read 0;
  * wind routing: a reference-task handle runs the no-wind kernels; a lane that gets steady
    wind -- by set_state or by a per-lane reset IC -- switches the handle to the wind kernels
    (MODE bit 1) and then follows the oracle with the wind applied (TOL_RAND30 over 30
    random-action steps, flags bit-exact);
  * a config IC with wind selects the wind kernels at create.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle_ref import OracleEnvs, default_ic  # noqa: E402
from test_gpu_parity import TOL_RAND30, TOL_STEP, _assert_frames  # noqa: E402
from test_gpu_production import _run_parity  # noqa: E402

from f16_jsb_amd.abi import (F16_IC_WIND_N_FPS, F16C_BA, F16C_EPA_C, F16C_EPA_S, F16C_LX, F16C_N1,  # noqa: E402
                             F16C_PID_P_P, F16C_WIND, F16L_P_AERO, F16L_VC_KTS, F16L_VG_FPS)


@pytest.fixture(scope="module")
def torch_mod(gpu):
    import torch
    return torch


def _goals(n, seed=0):
    return np.random.default_rng(seed).uniform([-5000, -5000, 1000], [5000, 5000, 4000], (n, 3)).astype(np.float32)


def test_state_roundtrip_and_recomputed_latch(torch_mod):
    from f16_jsb_amd.env import F16Envs
    n = 256
    ref, g = OracleEnvs(n, stack_k=4, seed=3), F16Envs(n, stack_k=4, seed=3)
    goals = _goals(n)
    ref.reset(goals=goals), g.reset(goals=goals)
    for t in range(1, 11):
        ref.step(ref.sample_actions(4, t))
        g.step(g.sample_actions(4, t))
    s1 = g.get_state()
    g.set_state(s1)
    s2 = g.get_state().cpu().numpy()
    s = s1.cpu().numpy()
    # bit-exact except the fields the canonical form re-encodes: the Earth angle (cos, sin ->
    # atan2 -> cos, sin) and the calibrated airspeed (latched as impact pressure in fp32)
    enc = [F16C_EPA_C, F16C_EPA_S, F16C_LX + F16L_VC_KTS]
    keep = [c for c in range(s.shape[1]) if c not in enc]
    np.testing.assert_array_equal(s2[:, keep], s[:, keep])
    np.testing.assert_allclose(s2[:, enc], s[:, enc], rtol=1e-6, atol=1e-12)
    r = ref.get_state()
    assert np.all(s[:, F16C_N1] == 0) and np.all(s[:, F16C_PID_P_P] == 0) and np.all(s[:, F16C_BA] == 0)
    # recomputed latch vs the oracle's stored latch (10 steps of fp32 vs fp64 dynamics apart)
    np.testing.assert_allclose(s[:, F16C_LX + F16L_P_AERO:F16C_LX + F16L_P_AERO + 3],
                               r[:, F16C_LX + F16L_P_AERO:F16C_LX + F16L_P_AERO + 3], atol=5e-4)
    np.testing.assert_allclose(s[:, F16C_LX + F16L_VG_FPS], r[:, F16C_LX + F16L_VG_FPS], rtol=1e-4)


def test_wind_by_set_state_switches_kernels(torch_mod):
    from f16_jsb_amd.env import F16Envs
    n = 256
    ref, g = OracleEnvs(n, stack_k=4, seed=5), F16Envs(n, stack_k=4, seed=5)
    goals = _goals(n, 1)
    o = ref.reset(goals=goals)
    g.reset(goals=goals)
    assert g.step_kernel_name == "f16_step_kernel"
    s = ref.get_state()
    s[::2, F16C_WIND:F16C_WIND + 3] = [20.0, -15.0, 2.0]  # steady wind NED (fps) on half the lanes
    ref.set_state(s)
    g.set_state(s)
    g.set_obs(o)
    assert g.step_kernel_name == "f16_step_var_kernel<2, 1, false>"
    _run_parity(torch_mod, ref, g, 30, 6, TOL_RAND30)


def test_wind_by_reset_ic_switches_kernels(torch_mod):
    from f16_jsb_amd.env import F16Envs
    n = 256
    ic = np.tile(default_ic(), (n, 1))
    ic[1::2, F16_IC_WIND_N_FPS:F16_IC_WIND_N_FPS + 3] = [-10.0, 25.0, 0.0]
    ref, g = OracleEnvs(n, stack_k=4, seed=8), F16Envs(n, stack_k=4, seed=8)
    goals = _goals(n, 2)
    o_r = ref.reset(goals=goals, ic=ic)
    o_g = g.reset(goals=goals, ic=ic).cpu().numpy()
    _assert_frames(o_g[:, -1], o_r[:, -1], TOL_STEP, "IC frame")
    assert g.step_kernel_name == "f16_step_var_kernel<2, 1, false>"
    _run_parity(torch_mod, ref, g, 30, 9, TOL_RAND30, o_ref0=o_r)


def test_config_wind_selects_wind_kernels(torch_mod):
    from f16_jsb_amd.env import F16Envs
    ic = default_ic()
    ic[F16_IC_WIND_N_FPS] = 12.0
    g = F16Envs(64, stack_k=4, seed=1, ic=ic)
    assert g.step_kernel_name == "f16_step_var_kernel<2, 1, false>"
    g.reset()
    s = g.get_state().cpu().numpy()
    assert np.all(s[:, F16C_WIND] == 12.0)
    ref = OracleEnvs(64, stack_k=4, seed=1, ic=ic)
    ref.reset()
    # auto-resets go back to the config IC, wind included (template with its wind columns)
    g.set_state(ref.get_state())
    _run_parity(torch_mod, ref, g, 20, 3, TOL_RAND30)
