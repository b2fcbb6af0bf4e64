"""Randomised configurations through the whole step / reset / state surface (seeded, so every run
draws the same cases): env counts around the wave and workgroup edges (1, 63, 65, 257, ...),
stack depths 1-12, short histories (window restarts every few steps) in both window orders,
short and long TimeLimits, the reference task and cfg5 (random ICs + gusts), caller resets
(NO_AUTORESET) and masked resets with caller goals / ICs mid-run, get_state / set_state round
trips, the NaN guard and the observation-bounds diagnostic, 1, 2 or 4 FDM frames per step.

Each case runs three handles on identical inputs for 15 steps:
  * the windowed layout against the contiguous one: bit-identical observations, rewards, flags,
    episode statistics and terminal observations (one per-expression FMA contraction,
    build.py -ffp-contract=on); and the windowed handle's feature window (obs_features) equal
    to the whole-window feature transform;
  * the contiguous layout against the CPU oracle (oracle/f16ref.c): done flags and episode lengths
    bit-exact, rewards within the frame-derived bound (tests/reward_bound.py), newest frames within the random-action tolerance of
    tests/test_gpu_parity.py (the cfg5 transonic tail statistically, as test_gpu_production.py);
  * the diagnostic counters (quarantines, out-of-bounds frames) equal on the two GPU layouts
    and, for the out-of-bounds count, equal to the oracle's.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle_ref import OracleEnvs  # noqa: E402
from reward_bound import reward_atol  # noqa: E402
from test_gpu_parity import TOL_RAND30, _assert_frames, _random_ics  # noqa: E402
from test_gpu_production import _assert_frames_stat  # noqa: E402


def _cases(n_cases=64, seed=2026):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n_cases):
        k = int(rng.integers(1, 13))
        c = {
            "n": int(rng.choice([1, 2, 63, 64, 65, 255, 257, 1000, 2049, 3001])),
            "k": k,
            "T": int(rng.integers(2 * k, 3 * k + 4)),
            "order": "env" if rng.random() < 0.25 else "position",
            "max_steps": int(rng.choice([3, 5, 17, 40, 1200])),
            "cfg5": bool(rng.random() < 0.3),
            "autoreset": bool(rng.random() < 0.75),
            "down_sample": int(rng.choice([4, 4, 4, 2, 1])),
            "nan_guard": bool(rng.random() < 0.5),
            "obs_check": bool(rng.random() < 0.5),
            "ic": str(rng.choice(["config", "random", "goals"])),
            "seed": int(rng.integers(1, 1 << 30)),
        }
        out.append(c)
    return out


# F16_FUZZ_CASES: more cases for a one-off robustness run (the suite draws 64; the same seed, so the
# first 64 of a longer run are the suite's)
CASES = _cases(int(os.environ.get("F16_FUZZ_CASES", "64")))


def _np(x):
    return x.cpu().numpy()


@pytest.mark.parametrize("case", CASES, ids=["c%02d_n%d_k%d" % (i, c["n"], c["k"]) for i, c in enumerate(CASES)])
def test_fuzz_layouts_and_oracle(gpu, case):
    import torch
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.features import features
    c = case
    n, k = c["n"], c["k"]
    kw = dict(stack_k=k, seed=c["seed"], max_steps=c["max_steps"], cfg5=c["cfg5"], down_sample=c["down_sample"])
    gkw = dict(autoreset=c["autoreset"], nan_guard=c["nan_guard"], obs_check=c["obs_check"])
    from f16_jsb_amd.abi import F16_FLAG_NAN_GUARD, F16_FLAG_NO_AUTORESET, F16_FLAG_OBS_CHECK
    flags = (0 if c["autoreset"] else F16_FLAG_NO_AUTORESET) | (F16_FLAG_NAN_GUARD if c["nan_guard"] else 0) \
        | (F16_FLAG_OBS_CHECK if c["obs_check"] else 0)
    ref = OracleEnvs(n, flags=flags, **kw)
    a = F16Envs(n, **kw, **gkw)
    b = F16Envs(n, obs_layout="window", history=c["T"], window_order=c["order"], **kw, **gkw)
    rng = np.random.default_rng(c["seed"])
    goals = rng.uniform(-5000, 5000, (n, 3)).astype(np.float32)
    goals[:, 2] = np.abs(goals[:, 2]) + 500.0
    ic = _random_ics(n, rng) if c["ic"] == "random" else None
    g = goals if c["ic"] != "config" else None
    o_r = ref.reset(goals=g, ic=ic)
    o_a, o_b = a.reset(goals=g, ic=ic), b.reset(goals=g, ic=ic)
    np.testing.assert_array_equal(_np(o_b), _np(o_a))
    _assert_frames(_np(o_a)[:, -1], o_r[:, -1], TOL_RAND30, "reset frame")
    finished = 0
    for t in range(1, 16):
        if t == 6:  # get_state / set_state round trip on every handle (checkpoint / restore)
            s = ref.get_state()
            ref.set_state(s)
            a.set_state(a.get_state())
            b.set_state(b.get_state())
        if t in (9, 13):  # masked resets mid-run, with caller goals on some
            m = (rng.random(n) < 0.3).astype(np.uint8)
            if not c["autoreset"]:
                m |= (_np(a.term) | _np(a.trunc)).astype(np.uint8)  # the caller resets finished lanes
            gm = rng.uniform(-4000, 4000, (n, 3)).astype(np.float32)
            gm[:, 2] = np.abs(gm[:, 2]) + 500.0
            gm = gm if t == 9 else None
            r_r = ref.reset(mask=m, goals=gm)
            r_a = a.reset(mask=torch.as_tensor(m), goals=gm)
            r_b = b.reset(mask=torch.as_tensor(m), goals=gm)
            np.testing.assert_array_equal(_np(r_b), _np(r_a), err_msg="masked reset @%d" % t)
            mm = m.astype(bool)
            if mm.any():
                _assert_frames(_np(r_a)[mm][:, -1], r_r[mm][:, -1], TOL_RAND30, "masked reset frame @%d" % t)
        act = ref.sample_actions(c["seed"] + 1, t)
        o_r, rw_r, te_r, tr_r, tobs_r, eret_r, elen_r = ref.step(act)
        at = torch.as_tensor(act, device=a.device)
        sa, sb = a.step(at), b.step(at)
        # windowed vs contiguous: bit-identical
        np.testing.assert_array_equal(_np(sb.obs), _np(sa.obs), err_msg="obs @%d" % t)
        np.testing.assert_array_equal(_np(sb.rew), _np(sa.rew), err_msg="rew @%d" % t)
        np.testing.assert_array_equal(_np(sb.terminated), _np(sa.terminated), err_msg="term @%d" % t)
        np.testing.assert_array_equal(_np(sb.truncated), _np(sa.truncated), err_msg="trunc @%d" % t)
        if t % 4 != 3:  # the feature window (steps without a call in between: whole-window restarts)
            assert torch.equal(b.obs_features(), features(sb.obs)), "feature window @%d" % t
        te_a, tr_a = _np(sa.terminated).astype(bool), _np(sa.truncated).astype(bool)
        d = te_a | tr_a
        if d.any() and c["autoreset"]:
            np.testing.assert_array_equal(_np(sb.ep_len)[d], _np(sa.ep_len)[d])
            np.testing.assert_array_equal(_np(sb.ep_return)[d], _np(sa.ep_return)[d])
            np.testing.assert_array_equal(_np(sb.terminal_obs)[d], _np(sa.terminal_obs)[d], err_msg="tobs @%d" % t)
        # contiguous vs the oracle
        np.testing.assert_array_equal(te_a, te_r, err_msg="terminated vs oracle @%d" % t)
        np.testing.assert_array_equal(tr_a, tr_r, err_msg="truncated vs oracle @%d" % t)
        # the reward tolerance the frame tolerance in force implies (tests/reward_bound.py)
        np.testing.assert_allclose(_np(sa.rew), rw_r, atol=reward_atol(TOL_RAND30 * (10 if c["cfg5"] else 1)),
                                   err_msg="reward vs oracle @%d" % t)
        if d.any():
            finished += int(d.sum())
            np.testing.assert_array_equal(_np(sa.ep_len)[d], elen_r[d])
            if c["autoreset"]:
                _assert_frames(_np(sa.terminal_obs)[d][:, -1], tobs_r[d][:, -1], TOL_RAND30 * (10 if c["cfg5"] else 1),
                               "terminal frame @%d" % t)
        if c["cfg5"]:
            _assert_frames_stat(_np(sa.obs)[:, -1], o_r[:, -1], TOL_RAND30, TOL_RAND30 * 10, "frame @%d" % t)
        else:
            _assert_frames(_np(sa.obs)[:, -1], o_r[:, -1], TOL_RAND30, "frame @%d" % t)
    assert a.nonfinite_count == b.nonfinite_count
    assert a.obs_bounds_count == b.obs_bounds_count
    if c["obs_check"]:
        assert a.obs_bounds_count == ref.obs_bounds_count
    if c["max_steps"] <= 5 and c["autoreset"]:
        assert finished >= n, (finished, n)
    ref.close()
    a.close()
    b.close()


def _rollout_cases(n_cases=12, seed=4051):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n_cases):
        k = int(rng.integers(1, 13))
        out.append({"n": int(rng.choice([1, 63, 65, 257, 1001, 2048])), "k": k, "cfg5": bool(rng.random() < 0.4),
                    "max_steps": int(rng.choice([2, 7, 19, 1200])), "T": int(rng.choice([1, 2, 9, 33])),
                    "hist": int(rng.integers(2 * k, 3 * k + 4)), "seed": int(rng.integers(1, 1 << 30))})
    return out


ROLL_CASES = _rollout_cases()


def _linear_policy(dev, k, seed):
    """Deterministic policy(obs) -> (actions, values, log_probs) on the newest frame whose
    actions often leave the action Box (the in-kernel clip matters)."""
    import torch
    g = torch.Generator().manual_seed(seed)
    W = (torch.randn(15, 4, generator=g) * 0.5).to(dev)
    scale = torch.tensor([1e-4, 1e-4, 1e-3, 1.0, 5.0, 5.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1e-4, 1e-4, 1e-3], device=dev)

    def pf(obs):
        x = obs[:, -1, :] * scale
        a = (x @ W).contiguous()
        return a, x.sum(1), -(a * a).sum(1)

    return pf


@pytest.mark.parametrize("case", ROLL_CASES, ids=["r%02d_n%d_k%d%s" % (i, c["n"], c["k"], "_cfg5" if c["cfg5"] else "")
                                                  for i, c in enumerate(ROLL_CASES)])
def test_fuzz_rollouts_bit_identical(gpu, case):
    """Random rollout shapes (T down to 1, ragged N, K 1-12, TimeLimits down to 2 steps, short
    window histories, cfg5): the fused rollout steps and the persistent rollout launch, in both
    layouts, give the same actions, frames, rewards, episode starts, final observation and state,
    bit for bit, over two consecutive rollouts (the second starts from the first's carry-over);
    and a policy in the loop (actions clipped in-kernel) gives the same buffers in both layouts."""
    import torch
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout
    c = case
    n, k, T = c["n"], c["k"], c["T"]

    def run(layout, persistent, policy):
        e = F16Envs(n, stack_k=k, seed=c["seed"], max_steps=c["max_steps"], cfg5=c["cfg5"], obs_layout=layout,
                    history=c["hist"] if layout == "window" else 0)
        e.reset()
        pf = _linear_policy(gpu, k, c["seed"]) if policy else None
        out = {}
        for r in range(2):
            b = DeviceRolloutBuffer(T, n, k, gpu)
            _, last_d = collect_rollout(e, b, c["seed"] + r, step0=r * T, persistent=persistent, policy_fn=pf)
            for f in ("frames", "actions", "rewards", "episode_starts", "obs0"):
                out["%s%d" % (f, r)] = getattr(b, f).clone()
            out["last_d%d" % r] = last_d.clone()
        out["obs"] = e.obs.clone()
        out["state"] = e.get_state()
        e.close()
        return out

    runs = {(lay, p): run(lay, p, False) for lay in ("contiguous", "window") for p in (False, True)}
    base = runs[("contiguous", False)]
    for key, r in runs.items():
        for f in base:
            assert torch.equal(r[f], base[f]), (key, f)
    pol = {lay: run(lay, False, True) for lay in ("contiguous", "window")}
    for f in pol["contiguous"]:
        assert torch.equal(pol["window"][f], pol["contiguous"][f]), ("policy", f)
