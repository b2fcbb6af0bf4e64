"""Reward parity bound derived from the frame parity in force.

TEST INFRASTRUCTURE. The reward of jsbsim_gym.py:237-261 + PositionReward (:487-507) is
    r = {-10 crash | +10 goal | 0} + gain * (last_d - d),   d = ||goal - (x, y, h)||_2 (3-D)
with last_d the distance of the lane's previous newest frame (its reset frame after a reset).
The done flags (hence the +-10) are compared bit-exactly elsewhere, so for lanes whose flags
agree the reward difference between two paths is the shaping term's:

    |r_a - r_b| <= gain * (|dp_prev| + |dp_now|)              (distance moves by at most |dp|)
                 + gain * 2 * (ulp32(d_prev) + ulp32(d_now))  (each fp32 norm3f within ~1 ulp,
                                                               on each side)
                 + ulp32(r) + 1e-7                            (the float32 reward)

where dp is the difference of the two paths' frame positions (lat*R, lon*R, h_m = the x, y, h
the distance is taken over). So the bound is per lane and per step, from the frames actually
compared -- not a blanket atol: at the one-step / 30-step frame tolerances it is ~1e-5..1e-4,
while a shaping term on the 2-D distance (jsbsim_gym.py:496-500 without the altitude) moves a
typical step's reward by ~1e-3 (the oracle's F16REF_TEST_SHAPING_2D negative control)."""
from __future__ import annotations

import numpy as np


def _ulp32(x):
    return np.spacing(np.abs(np.asarray(x, np.float32))).astype(np.float64)


def _dist(f):
    f = np.asarray(f, np.float64)
    return np.sqrt((f[:, 12] - f[:, 0]) ** 2 + (f[:, 13] - f[:, 1]) ** 2 + (f[:, 14] - f[:, 2]) ** 2)


def reward_bound(f_a_prev, f_b_prev, f_a, f_b, r_ref, gain=0.01):
    """Per-lane bound on |r_a - r_b| from the two paths' previous and current newest frames
    (N, 15) and the reference reward (N,)."""
    dp_prev = np.linalg.norm(np.asarray(f_a_prev, np.float64)[:, :3] - np.asarray(f_b_prev, np.float64)[:, :3], axis=1)
    dp_now = np.linalg.norm(np.asarray(f_a, np.float64)[:, :3] - np.asarray(f_b, np.float64)[:, :3], axis=1)
    d_prev, d_now = _dist(f_b_prev), _dist(f_b)
    return (gain * (dp_prev + dp_now) + gain * 2.0 * (_ulp32(d_prev) + _ulp32(d_now))
            + _ulp32(r_ref) + 1e-7)


def reward_atol(tol_frames, d_max=20000.0, gain=0.01):
    """The same bound as a blanket tolerance, for checks that only see some of the frames (golden
    fixtures, rollout slots): both frames' positions within tol_frames[:3] (m) and goal distances
    up to d_max (m): 2 gain |tol_pos| + 4 gain ulp32(d_max) + 1e-6. TOL_RAND30 -> 2.5e-4,
    TOL_CONST300 -> 1.8e-3."""
    t = np.asarray(tol_frames, np.float64)[:3]
    return float(2.0 * gain * np.linalg.norm(t) + 4.0 * gain * float(_ulp32(d_max)) + 1e-6)


def final_frames(out, o_g, o_r, tobs_r, done):
    """The frames a step's rewards were computed on, (gpu, ref): the newest frame of the returned
    observation, except for finished lanes, whose reward is on their final frame (the newest
    frame of the terminal observation; the returned one is already the reset frame)."""
    fin_g, fin_r = o_g[:, -1].copy(), np.asarray(o_r)[:, -1].copy()
    done = np.asarray(done, bool)
    if done.any():
        fin_g[done] = out.terminal_obs.cpu().numpy()[done, -1]
        fin_r[done] = np.asarray(tobs_r)[done, -1]
    return fin_g, fin_r


def assert_rewards_close(r_a, r_b, f_a_prev, f_b_prev, f_a, f_b, what="", gain=0.01, mask=None):
    """Raise AssertionError when any lane's |r_a - r_b| exceeds reward_bound (lanes in `mask`)."""
    r_a = np.asarray(r_a, np.float64)
    r_b = np.asarray(r_b, np.float64)
    bound = reward_bound(f_a_prev, f_b_prev, f_a, f_b, r_b, gain)
    err = np.abs(r_a - r_b)
    bad = err > bound
    if mask is not None:
        bad &= np.asarray(mask, bool)
    if bad.any():
        i = int(np.flatnonzero(bad)[0])
        raise AssertionError("%s: reward lane %d |%.9g - %.9g| = %.3e > bound %.3e (%d lanes over)"
                             % (what, i, r_a[i], r_b[i], err[i], bound[i], int(bad.sum())))
    return float(bound.max()) if bound.size else 0.0


class RewardChecker:
    """Per-step reward check along a run: keeps the previous newest frames of both paths (what
    each side's last_d was computed from). Start it with the two observations the run starts
    from, then call check() after every step."""

    def __init__(self, o_g0, o_r0, gain=0.01):
        self.fg = np.asarray(o_g0)[:, -1]
        self.fr = np.asarray(o_r0)[:, -1]
        self.gain = gain
        self.worst = 0.0

    def check(self, out, o_r, r_r, tobs_r, done, what="", mask=None, o_g=None):
        o_g = out.obs.cpu().numpy() if o_g is None else o_g
        fin_g, fin_r = final_frames(out, o_g, o_r, tobs_r, done)
        b = assert_rewards_close(out.rew.cpu().numpy(), r_r, self.fg, self.fr, fin_g, fin_r, what,
                                 gain=self.gain, mask=mask)
        self.worst = max(self.worst, b)
        self.fg, self.fr = o_g[:, -1], np.asarray(o_r)[:, -1]
        return b
