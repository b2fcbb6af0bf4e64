"""BASELINE cfg5 on the GPU: random-IC resets (device Philox box draw + RunIC, deferred to
f16_reset_done_kernel on auto-reset) and Gauss-Markov gusts, against the CPU oracle.
Tolerances as tests/test_gpu_parity.py; gust states: fp32 Box-Muller vs fp64, 1e-4 fps."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle_ref import OracleEnvs  # noqa: E402
from test_gpu_parity import TOL_RAND30, TOL_STEP, _assert_frames  # noqa: E402

from f16_jsb_amd.abi import F16C_GUST, F16C_STEP, F16C_WIND, F16_FLAG_NO_AUTORESET  # noqa: E402


@pytest.fixture(scope="module")
def torch_mod(gpu):
    import torch
    return torch


def _pair(n, k, **kw):
    from f16_jsb_amd.env import F16Envs
    return OracleEnvs(n, stack_k=k, cfg5=True, **kw), F16Envs(n, stack_k=k, cfg5=True, **kw)


def test_random_ic_reset_parity(torch_mod):
    n = 512
    ref, g = _pair(n, 4, seed=21)
    o_r = ref.reset()
    o_g = g.reset().cpu().numpy()
    np.testing.assert_array_equal(o_g[:, :, 12:], o_r[:, :, 12:])  # Philox goals
    _assert_frames(o_g[:, -1], o_r[:, -1], TOL_STEP, "random IC frame")
    assert o_r[:, -1, 2].std() > 1000.0  # altitudes really spread over the box
    s_r, s_g = ref.get_state(), g.get_state().cpu().numpy()
    np.testing.assert_allclose(s_g[:, F16C_WIND:F16C_WIND + 3], s_r[:, F16C_WIND:F16C_WIND + 3], atol=1e-5)
    np.testing.assert_allclose(s_g[:, F16C_GUST:F16C_GUST + 3], s_r[:, F16C_GUST:F16C_GUST + 3], atol=1e-4)


def test_gust_trajectory_parity(torch_mod):
    torch = torch_mod
    n = 256
    ref, g = _pair(n, 4, seed=8, flags=F16_FLAG_NO_AUTORESET)
    ref.reset()
    g.reset()
    g.set_state(ref.get_state())  # identical start, then both integrate their own gusts
    for t in range(1, 31):
        a = ref.sample_actions(3, t)
        o_r, r_r, te_r, tr_r, *_ = ref.step(a)
        out = g.step(torch.as_tensor(a).cuda())
        np.testing.assert_array_equal(out.terminated.cpu().numpy().astype(bool), te_r)
    s_r, s_g = ref.get_state(), g.get_state().cpu().numpy()
    np.testing.assert_allclose(s_g[:, F16C_GUST:F16C_GUST + 3], s_r[:, F16C_GUST:F16C_GUST + 3], atol=1e-4)
    assert np.abs(s_r[:, F16C_GUST:F16C_GUST + 3]).max() > 1.0
    _assert_frames(out.obs.cpu().numpy()[:, -1], o_r[:, -1], TOL_RAND30 * 2, "gust + random actions @30")


def test_deferred_autoreset_parity(torch_mod):
    """Lanes at max_steps-1 truncate on the next step; both paths auto-reset them to a
    random-IC episode: terminal obs, done list, new-episode frames (K copies) and state."""
    torch = torch_mod
    n = 300
    ref, g = _pair(n, 3, seed=99)
    o = ref.reset()
    g.reset()
    s = ref.get_state()
    ending = np.arange(n) % 3 == 0
    s[ending, F16C_STEP] = ref.cfg.max_steps - 1
    ref.set_state(s)
    g.set_state(s)
    g.set_obs(torch.as_tensor(o))
    a = ref.sample_actions(1, 1)
    o_r, r_r, te_r, tr_r, tobs_r, *_ = ref.step(a)
    done_idx = torch.zeros(n, dtype=torch.int32, device="cuda")
    n_done = torch.zeros(1, dtype=torch.int32, device="cuda")
    out = g.step(torch.as_tensor(a).cuda(), done_idx=done_idx, n_done=n_done)
    tr_g = out.truncated.cpu().numpy().astype(bool)
    np.testing.assert_array_equal(tr_g, tr_r)
    d = tr_r | te_r
    assert d.sum() >= n // 3
    nd = int(n_done.item())
    assert sorted(done_idx[:nd].cpu().tolist()) == np.flatnonzero(d).tolist()
    og = out.obs.cpu().numpy()
    _assert_frames(out.terminal_obs.cpu().numpy()[d, -1], tobs_r[d, -1], TOL_STEP, "terminal obs")
    assert np.all(og[d] == og[d][:, :1])                      # K copies of the reset frame
    np.testing.assert_array_equal(og[d][:, :, 12:], o_r[d][:, :, 12:])
    _assert_frames(og[d][:, -1], o_r[d][:, -1], TOL_STEP, "random-IC reset frame")
    _assert_frames(og[~d][:, -1], o_r[~d][:, -1], TOL_STEP, "running lanes")
    s_r, s_g = ref.get_state(), g.get_state().cpu().numpy()
    np.testing.assert_array_equal(s_g[d, F16C_STEP], 0)
    np.testing.assert_allclose(s_g[d, F16C_GUST:F16C_GUST + 3], s_r[d, F16C_GUST:F16C_GUST + 3], atol=1e-4)
