"""Flight-envelope edges against the oracle: the branches the BASELINE configs rarely or never
reach. The cfg3 / cfg5 tests fly 3 000-30 000 ft at 600-1 200 fps with small attitudes; here
every lane starts somewhere the kernels take a different path or clamp a table:

  * stratosphere and above: 36 089-75 000 ft (the atmosphere's wave-uniform layer search,
    isothermal and gradient layers above 11 km; the thrust tables clamp past 60 000 ft);
  * supersonic: up to Mach ~2.2 (the Rayleigh pitot branch of the impact pressure and the
    Newton solve of vcas_from_qc; the Mach tables clamp past 1.8);
  * alpha / beta far outside the aerodynamic tables (-10..45 deg, +-30 deg): clamped lookups;
  * inverted and near-vertical attitudes (|phi| up to pi, |theta| up to 85 deg: Euler-angle
    extraction near its singularity) and body rates up to 4 rad/s;
  * just above the 10 m crash floor, nose down: crash terminations in the first steps.

Every lane's IC frame and the first eight random-action steps are compared with the fp64
oracle at the one-step tolerance (growing linearly with the step), done flags bit-exact,
rewards within 2e-3 -- in the reference task and with cfg5 wind on the same states.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle_ref import OracleEnvs, default_ic  # noqa: E402
from parity_tools import frame_err  # noqa: E402
from reward_bound import RewardChecker  # noqa: E402
from test_gpu_parity import TOL_STEP  # noqa: E402


def _assert_frames(gpu, ref, tol, what):
    """As test_gpu_parity's, with the tolerance floored at 2 fp32 ulps of the reference value:
    above ~8 km the observed altitude (m) has a coarser fp32 spacing than TOL_STEP's 1e-3 m."""
    err = frame_err(gpu, ref)
    lim = np.maximum(tol, 2.0 * np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64))
    lim[..., 12:] = 0.0  # goals: exact
    bad = err > lim
    if bad.any():
        idx = tuple(np.argwhere(bad)[0])
        raise AssertionError("%s: component %d err %.3e > tol %.1e (gpu %r ref %r)" % (
            what, idx[-1], err[idx], lim[idx], gpu[idx[:-1]], ref[idx[:-1]]))


def _edge_ics(n, rng):
    ic = np.tile(default_ic(), (n, 1))
    q = n // 5
    # 0: stratosphere and above, transonic to supersonic
    ic[:q, 2] = rng.uniform(36089.0, 75000.0, q)
    ic[:q, 3] = rng.uniform(700.0, 2100.0, q)
    # 1: supersonic at low / mid altitude
    ic[q:2 * q, 2] = rng.uniform(5000.0, 35000.0, q)
    ic[q:2 * q, 3] = rng.uniform(1300.0, 2300.0, q)
    # 2: alpha / beta outside the tables (large w, v body velocities)
    ic[2 * q:3 * q, 3] = rng.uniform(250.0, 700.0, q)
    ic[2 * q:3 * q, 4] = rng.uniform(-450.0, 450.0, q)
    ic[2 * q:3 * q, 5] = rng.uniform(-350.0, 700.0, q)
    ic[2 * q:3 * q, 2] = rng.uniform(8000.0, 30000.0, q)
    # 3: inverted / near-vertical attitudes, high body rates
    ic[3 * q:4 * q, 6] = rng.uniform(-np.pi, np.pi, q)
    ic[3 * q:4 * q, 7] = rng.uniform(-1.48, 1.48, q)
    ic[3 * q:4 * q, 9:12] = rng.uniform(-4.0, 4.0, (q, 3))
    ic[3 * q:4 * q, 2] = rng.uniform(10000.0, 40000.0, q)
    # 4: just above the 10 m crash floor (jsbsim_gym.py:245), nose down
    ic[4 * q:, 2] = rng.uniform(40.0, 130.0, n - 4 * q)
    ic[4 * q:, 7] = rng.uniform(-0.8, -0.3, n - 4 * q)
    ic[:, 8] = rng.uniform(0.0, 2 * np.pi, n)
    ic[:, 15] = rng.uniform(0.0, 1.0, n)  # throttle at IC (augmentor above 0.5 x 2)
    return ic


@pytest.mark.parametrize("cfg5", [False, True], ids=["reference_task", "cfg5_wind"])
def test_flight_envelope_edges(gpu, cfg5):
    import torch
    from f16_jsb_amd.env import F16Envs
    n = 640
    rng = np.random.default_rng(17)
    ic = _edge_ics(n, rng)
    if cfg5:  # steady wind on the same states (the gust is the model's own draw)
        ic[:, 16:18] = rng.uniform(-30.0, 30.0, (n, 2))
    goals = rng.uniform(-5000, 5000, (n, 3)).astype(np.float32)
    goals[:, 2] = 60000.0  # no goal capture: the lanes end by crashing or not at all
    kw = dict(stack_k=4, seed=23, cfg5=cfg5)
    ref = OracleEnvs(n, **kw)
    g = F16Envs(n, **kw)
    o_r = ref.reset(goals=goals, ic=ic)
    o_g = g.reset(goals=goals, ic=ic).cpu().numpy()
    _assert_frames(o_g[:, -1], o_r[:, -1], TOL_STEP, "IC frame")
    rc = RewardChecker(o_g, o_r)
    alive = np.ones(n, bool)
    crashes = 0
    for t in range(1, 9):
        a = ref.sample_actions(31, t)
        o_r, r_r, te_r, tr_r, tobs_r, *_ = ref.step(a)
        out = g.step(torch.as_tensor(a).cuda())
        te_g = out.terminated.cpu().numpy().astype(bool)
        np.testing.assert_array_equal(te_g[alive], te_r[alive], err_msg="terminated @%d" % t)
        rc.check(out, o_r, r_r, tobs_r, te_r | tr_r, "reward @%d" % t, mask=alive)
        crashes += int((te_r & alive).sum())
        alive &= ~(te_r | tr_r)
        _assert_frames(out.obs.cpu().numpy()[alive, -1], o_r[alive, -1], TOL_STEP * t, "step %d" % t)
    assert crashes > 0 and alive.sum() > n // 2, (crashes, int(alive.sum()))
    # the edges were really visited
    st = g.get_state().cpu().numpy()
    assert (o_r[:, -1, 2] > 11000.0).sum() > 50        # above the tropopause (m)
    assert (o_r[:, -1, 3] > 1.2).sum() > 50            # supersonic
    assert (np.abs(o_r[:, -1, 4]) > 0.8).sum() > 10    # alpha beyond the 45-deg table end
    assert np.isfinite(st).all()
    ref.close()
    g.close()
