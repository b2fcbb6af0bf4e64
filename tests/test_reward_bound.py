"""The reward parity bound (tests/reward_bound.py) on the CPU: it accepts two identical oracle
runs and rejects the deliberate 2-D shaping distance (VERDICT r05 item 3's negative control;
the GPU side of the same control is tests/test_gpu_parity.py::test_reward_bound_rejects_2d_shaping)."""
from __future__ import annotations

import numpy as np
import pytest

from oracle_ref import OracleEnvs, lib
from reward_bound import assert_rewards_close

SHAPING_2D = 0x10  # oracle/f16ref.h F16REF_TEST_SHAPING_2D


def _pair_runs(n, steps, mask_b, seed=5, act_seed=99):
    """Two oracle batches on identical lanes and actions; batch b runs under physics mask mask_b.
    Yields per step (r_a, r_b, f_a_prev, f_b_prev, f_a, f_b)."""
    L = lib()
    goals = np.random.default_rng(0).uniform([-5000, -5000, 1000], [5000, 5000, 4000], (n, 3)).astype(np.float32)
    a, b = OracleEnvs(n, stack_k=4, seed=seed), OracleEnvs(n, stack_k=4, seed=seed)
    try:
        fa = a.reset(goals=goals)[:, -1]
        L.f16ref_set_physics_mask(mask_b)
        try:
            fb = b.reset(goals=goals)[:, -1]
        finally:
            L.f16ref_set_physics_mask(0)
        for t in range(1, steps + 1):
            act = a.sample_actions(act_seed, t)
            oa, ra, *_ = a.step(act)
            L.f16ref_set_physics_mask(mask_b)
            try:
                ob, rb, *_ = b.step(act)
            finally:
                L.f16ref_set_physics_mask(0)
            yield ra, rb, fa, fb, oa[:, -1], ob[:, -1]
            fa, fb = oa[:, -1], ob[:, -1]
    finally:
        a.close()
        b.close()


def test_bound_accepts_identical_runs():
    worst = 0.0
    for ra, rb, fap, fbp, fa, fb in _pair_runs(128, 30, 0):
        np.testing.assert_array_equal(ra, rb)
        worst = max(worst, assert_rewards_close(ra, rb, fap, fbp, fa, fb, "identical"))
    # rounding-only bound at the reference task's distances (a few km): well under 1e-4
    assert worst < 1e-4, worst


def test_bound_rejects_2d_shaping_distance():
    """The 2-D distance leaves the physics (frames) bit-identical and moves the shaping term:
    the bound -- rounding only, since the frames agree -- rejects it at every step, and per lane
    it rejects the lane-steps the blanket atol=2e-3 of rounds 1-5 accepted (a level lane far
    from its goal: the altitude offset barely moves the distance's rate)."""
    from reward_bound import reward_bound
    rejected_steps, new_rej, old_acc, n_ls = 0, 0, 0, 0
    for ra, rb, fap, fbp, fa, fb in _pair_runs(128, 30, SHAPING_2D):
        np.testing.assert_array_equal(fa, fb)  # physics untouched by the defect
        with pytest.raises(AssertionError):
            assert_rewards_close(ra, rb, fap, fbp, fa, fb, "2-D shaping")
        rejected_steps += 1
        d = np.abs(ra.astype(np.float64) - rb)
        moved = d > 0
        n_ls += int(moved.sum())
        new_rej += int((moved & (d > reward_bound(fap, fbp, fa, fb, rb))).sum())
        old_acc += int((moved & (d <= 2e-3)).sum())
    assert rejected_steps == 30
    # lane-steps the defect moved: the bound rejects nearly all; the old atol accepted many
    assert new_rej >= 0.95 * n_ls, (new_rej, n_ls)
    assert old_acc >= 0.2 * n_ls, (old_acc, n_ls)
