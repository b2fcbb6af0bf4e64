"""HIP path (fp32 kernel, fp64 ECI position) vs the CPU oracle (fp64), through the C ABI.

Tolerances (calibrated from tests/parity_report.py on MI355X, with >= 10x margin):
  * IC / one env step from an identical injected state: fp32 round-off level
      positions 1e-3 m, angles / alpha / beta 5e-6 rad, mach 5e-6, body rates 5e-5 rad/s;
  * constant-action trajectories (non-chaotic), 300 steps = 10 s:
      positions 0.05 m, angles 1e-4 rad, mach 1e-5, rates 5e-5 rad/s;
  * random-action trajectories diverge chaotically: checked to 30 steps
      (1 s) at positions 5e-3 m, angles 5e-5 rad, rates 5e-4 rad/s; beyond that only the
      divergence report (parity_report.py) is produced;
  * integer / RNG / env-logic outputs (actions, goals, done flags, step counters,
      compacted done list) are bit-exact.
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle_ref import OracleEnvs, default_ic  # noqa: E402
from parity_tools import frame_err  # noqa: E402
from reward_bound import RewardChecker, assert_rewards_close, final_frames  # noqa: E402

# per frame component atol: lat*R lon*R h mach alpha beta p q r phi theta psi goal(3)
TOL_STEP = np.array([1e-3, 1e-3, 1e-3, 5e-6, 5e-6, 5e-6, 5e-5, 5e-5, 5e-5, 5e-6, 5e-6, 5e-6, 0, 0, 0])
TOL_CONST300 = np.array([5e-2, 5e-2, 5e-2, 1e-5, 1e-5, 1e-5, 5e-5, 5e-5, 5e-5, 1e-4, 1e-4, 1e-4, 0, 0, 0])
TOL_RAND30 = np.array([5e-3, 5e-3, 5e-3, 2e-5, 5e-5, 5e-5, 5e-4, 5e-4, 5e-4, 5e-5, 5e-5, 5e-5, 0, 0, 0])


def _assert_frames(gpu, ref, tol, what):
    err = frame_err(gpu, ref)
    bad = err > tol
    if bad.any():
        idx = np.argwhere(bad)[0]
        raise AssertionError("%s: component %d err %.3e > tol %.1e (gpu %r ref %r)" % (
            what, idx[-1], err[tuple(idx)], tol[idx[-1]], gpu[tuple(idx[:-1])], ref[tuple(idx[:-1])]))


def _random_ics(n, rng):
    ic = np.tile(default_ic(), (n, 1))
    ic[:, 2] = rng.uniform(3000, 30000, n)          # h ft
    ic[:, 3] = rng.uniform(600, 1200, n)            # u fps
    ic[:, 6] = rng.uniform(-0.17, 0.17, n)          # phi
    ic[:, 7] = rng.uniform(-0.17, 0.17, n)          # theta
    ic[:, 8] = rng.uniform(0, 2 * np.pi, n)         # psi
    ic[:, 9:12] = rng.uniform(-0.05, 0.05, (n, 3))  # p q r
    ic[:, 15] = rng.uniform(0.0, 1.0, n)            # throttle cmd at IC
    return ic


@pytest.fixture(scope="module")
def torch_mod(gpu):
    import torch
    return torch


def _pair(n, k, **kw):
    from f16_jsb_amd.env import F16Envs
    return OracleEnvs(n, stack_k=k, **kw), F16Envs(n, stack_k=k, **kw)


def test_ic_parity_random_ics(torch_mod):
    n = 128
    rng = np.random.default_rng(0)
    ic = _random_ics(n, rng)
    goals = rng.uniform(-5000, 5000, (n, 3)).astype(np.float32)
    ref, g = _pair(n, 4, seed=1)
    o_r = ref.reset(goals=goals, ic=ic)
    o_g = g.reset(goals=goals, ic=ic).cpu().numpy()
    _assert_frames(o_g[:, -1], o_r[:, -1], TOL_STEP, "IC frame")
    assert np.all(o_g == o_g[:, :1])


def test_one_step_parity_from_identical_states(torch_mod):
    torch = torch_mod
    n = 128
    rng = np.random.default_rng(1)
    goals = rng.uniform(-5000, 5000, (n, 3)).astype(np.float32)
    ref, g = _pair(n, 4, seed=3)
    obs = ref.reset(goals=goals, ic=_random_ics(n, rng))
    g.reset(goals=goals)
    checked = 0
    for t in range(120):
        a = ref.sample_actions(5, t)
        if t % 15 == 14:
            g.set_state(ref.get_state())
            g.set_obs(torch.as_tensor(obs))
            o_r, r_r, te_r, tr_r, *_ = ref.step(a)
            out = g.step(torch.as_tensor(a).cuda())
            alive = ~(te_r | tr_r)
            _assert_frames(out.obs.cpu().numpy()[alive, -1], o_r[alive, -1], TOL_STEP, "one step @%d" % t)
            np.testing.assert_allclose(out.rew.cpu().numpy()[alive], r_r[alive], atol=1e-4)
            checked += int(alive.sum())
            obs = o_r
        else:
            obs = ref.step(a)[0]
    assert checked > 200


def test_constant_action_trajectory(torch_mod):
    torch = torch_mod
    n = 32
    rng = np.random.default_rng(2)
    goals = rng.uniform(-5000, 5000, (n, 3)).astype(np.float32)
    ref, g = _pair(n, 4, seed=4)
    ref.reset(goals=goals)
    g.reset(goals=goals)
    act = np.tile(np.array([[0.05, -0.1, 0.02, 0.7]], np.float32), (n, 1))
    act[:, 3] = np.linspace(0.2, 1.0, n)
    ta = torch.as_tensor(act).cuda()
    for t in range(300):
        o_r, r_r, te_r, tr_r, *_ = ref.step(act)
        out = g.step(ta)
        np.testing.assert_array_equal(out.terminated.cpu().numpy().astype(bool), te_r)
    _assert_frames(out.obs.cpu().numpy()[:, -1], o_r[:, -1], TOL_CONST300, "constant action @300")


def test_random_action_short_horizon(torch_mod):
    n = 256
    rng = np.random.default_rng(3)
    goals = rng.uniform(-5000, 5000, (n, 3)).astype(np.float32)
    ref, g = _pair(n, 4, seed=5)
    f_r = ref.reset(goals=goals)[:, -1]
    f_g = g.reset(goals=goals).cpu().numpy()[:, -1]
    worst = 0.0
    for t in range(1, 31):
        a = ref.sample_actions(99, t)
        o_r, r_r, te_r, tr_r, tobs_r, _, _ = ref.step(a)
        out = g.step(g.sample_actions(99, t))
        np.testing.assert_array_equal(out.terminated.cpu().numpy().astype(bool), te_r)
        np.testing.assert_array_equal(out.truncated.cpu().numpy().astype(bool), tr_r)
        o_g = out.obs.cpu().numpy()
        fin_g, fin_r = final_frames(out, o_g, o_r, tobs_r, te_r | tr_r)
        worst = max(worst, assert_rewards_close(out.rew.cpu().numpy(), r_r, f_g, f_r, fin_g, fin_r,
                                                "reward @%d" % t))
        f_g, f_r = o_g[:, -1], o_r[:, -1]
    # the derived bound stays at the one-step test's 1e-4 through step 30
    assert worst <= 1e-4, worst
    _assert_frames(out.obs.cpu().numpy()[:, -1], o_r[:, -1], TOL_RAND30, "random actions @30")


def test_reward_bound_rejects_2d_shaping(torch_mod):
    """Negative control: the oracle with a deliberately 2-D shaping distance
    (F16REF_TEST_SHAPING_2D: PositionReward over (x, y), jsbsim_gym.py:496-500 without the
    altitude; the physics untouched) against the HIP path -- the reward check above must reject
    it within the same 30 steps, on most lane-steps."""
    from oracle_ref import lib
    from reward_bound import reward_bound
    n = 256
    rng = np.random.default_rng(3)
    goals = rng.uniform(-5000, 5000, (n, 3)).astype(np.float32)
    goals[:, 2] = np.abs(goals[:, 2])
    ref, g = _pair(n, 4, seed=5)
    L = lib()
    L.f16ref_set_physics_mask(0x10)
    try:
        f_r = ref.reset(goals=goals)[:, -1]
        f_g = g.reset(goals=goals).cpu().numpy()[:, -1]
        rejected, moved = 0, 0
        for t in range(1, 31):
            o_r, r_r, *_ = ref.step(ref.sample_actions(99, t))
            out = g.step(g.sample_actions(99, t))
            o_g, r_g = out.obs.cpu().numpy(), out.rew.cpu().numpy()
            err = np.abs(r_g.astype(np.float64) - r_r)
            rejected += int((err > reward_bound(f_g, f_r, o_g[:, -1], o_r[:, -1], r_r)).sum())
            moved += n
            f_g, f_r = o_g[:, -1], o_r[:, -1]
    finally:
        L.f16ref_set_physics_mask(0)
    assert rejected >= 0.9 * moved, (rejected, moved)


def test_sample_actions_bitexact(torch_mod):
    n = 1000
    ref, g = _pair(n, 1, env_id_base=12345)
    for step in (0, 1, 7, 2**33 + 5):
        np.testing.assert_array_equal(g.sample_actions(42, step).cpu().numpy(), ref.sample_actions(42, step))
    a = g.sample_actions(42, 3).cpu().numpy()
    assert a[:, :3].min() >= -1 and a.max() < 1 and a[:, 3].min() >= 0


def test_autoreset_crash_parity(torch_mod):
    """Diving lanes crash (-10, jsbsim_gym.py:245-247), auto-reset (dummy_vec_env.py:68-71):
    terminal obs, Monitor return/length, Philox goals of the new episode are bit-exact."""
    torch = torch_mod
    n = 64
    ic = np.tile(default_ic(), (n, 1))
    ic[:, 2] = np.linspace(150.0, 600.0, n)   # ft
    ic[:, 7] = -0.6                           # steep dive
    goals = np.tile(np.array([[3000.0, 3000.0, 2000.0]], np.float32), (n, 1))
    ref, g = _pair(n, 4, seed=77)
    rc = RewardChecker(g.reset(goals=goals, ic=ic).cpu().numpy(), ref.reset(goals=goals, ic=ic))
    act = np.zeros((n, 4), np.float32)
    ta = torch.as_tensor(act).cuda()
    saw = np.zeros(n, bool)
    for t in range(40):
        o_r, r_r, te_r, tr_r, tobs_r, eret_r, elen_r = ref.step(act)
        out = g.step(ta)
        te_g = out.terminated.cpu().numpy().astype(bool)
        np.testing.assert_array_equal(te_g, te_r)
        rc.check(out, o_r, r_r, tobs_r, te_r | tr_r, "reward @%d" % t)  # -10 + shaping on the final frame
        if te_r.any():
            d = te_r
            saw |= d
            np.testing.assert_allclose(out.ep_return.cpu().numpy()[d], eret_r[d], atol=1e-3)
            np.testing.assert_array_equal(out.ep_len.cpu().numpy()[d], elen_r[d])
            _assert_frames(out.terminal_obs.cpu().numpy()[d, -1], tobs_r[d, -1], TOL_CONST300, "terminal obs")
            og = out.obs.cpu().numpy()[d]
            # new episode: K copies of the IC frame, goal from the device Philox stream (bit-exact)
            np.testing.assert_array_equal(og[:, :, 12:], o_r[d][:, :, 12:])
            _assert_frames(og[:, -1], o_r[d][:, -1], TOL_STEP, "reset frame")
    assert saw.all()


def test_autoreset_goal_reached_parity(torch_mod):
    """Goal reached (jsbsim_gym.py:248-255: horizontal distance < dg = 100 m and |h - gz| <
    100 m -> +10, terminated) at staggered steps, then auto-reset: done flags and episode
    lengths bit-exact, rewards / returns / terminal obs within the step tolerances. Goals
    are placed along the IC heading (north, frame x = lat*R), one group out of reach by
    altitude (never terminates)."""
    torch = torch_mod
    n = 64
    act1 = np.array([[0.0, 0.0, 0.0, 0.6]], np.float32)
    # the flight path does not depend on the goal: probe it once, then put env i's goal so
    # that it comes within 100 m half-way between steps i and i+1 (~4.5 m from either side
    # of the threshold, far beyond the fp32 position error)
    probe = OracleEnvs(1, stack_k=4, seed=91)
    probe.reset(goals=np.array([[0.0, 0.0, 9000.0]], np.float32), ic=default_ic()[None])
    xs = [0.0] + [float(probe.step(act1)[0][0, -1, 0]) for _ in range(50)]
    probe.close()
    ic = np.tile(default_ic(), (n, 1))
    goals = np.zeros((n, 3), np.float32)
    y = np.linspace(-60.0, 60.0, 48)
    goals[:48, 1] = y
    goals[:48, 0] = [0.5 * (xs[i] + xs[i + 1]) + np.sqrt(1e4 - y[i] ** 2) for i in range(48)]
    goals[:, 2] = 1524.0
    goals[48:, 0] = np.linspace(30.0, 600.0, 16)
    goals[48:, 2] = 1524.0 + 400.0                 # out of reach in altitude
    ref, g = _pair(n, 4, seed=91)
    rc = RewardChecker(g.reset(goals=goals, ic=ic).cpu().numpy(), ref.reset(goals=goals, ic=ic))
    act = np.tile(act1, (n, 1))
    ta = torch.as_tensor(act).cuda()
    first = np.zeros(n, bool)
    for t in range(60):
        o_r, r_r, te_r, tr_r, tobs_r, eret_r, elen_r = ref.step(act)
        out = g.step(ta)
        te_g = out.terminated.cpu().numpy().astype(bool)
        np.testing.assert_array_equal(te_g, te_r, err_msg="terminated @%d" % t)
        rc.check(out, o_r, r_r, tobs_r, te_r | tr_r, "reward @%d" % t)
        d = te_r & ~first  # each env's first episode end (later ones start from a Philox goal)
        if d.any():
            assert (r_r[d] > 9.0).all()  # the +10 goal reward, not the -10 crash
            np.testing.assert_allclose(out.ep_return.cpu().numpy()[d], eret_r[d], atol=1e-3)
            np.testing.assert_array_equal(out.ep_len.cpu().numpy()[d], elen_r[d])
            _assert_frames(out.terminal_obs.cpu().numpy()[d, -1], tobs_r[d, -1], TOL_CONST300, "terminal obs")
            first |= d
            if t < 48:
                assert d[t]  # env t reaches its goal at step t + 1
    assert first[:48].all() and not first[48:].any()


def test_autoreset_frame_equals_reset_kernel_frame(torch_mod):
    """The step kernel's auto-reset copies frame 0 of the IC template, evaluated once at create
    (f16_ic_kernel); f16env_reset evaluates it per lane (f16_reset_kernel). For the same IC
    and goal both give the same K x 15 rows, bit for bit."""
    torch = torch_mod
    from f16_jsb_amd.env import F16Envs
    n = 512
    ic = np.tile(default_ic(), (n, 1))
    ic[:, 2] = np.linspace(150.0, 900.0, n)   # ft
    ic[:, 7] = -0.6                           # dive: every lane crashes within ~2 s
    g = F16Envs(n, stack_k=4, seed=21)
    g.reset(ic=ic)
    act = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
    seen = 0
    for t in range(80):
        out = g.step(act)
        d = (out.terminated | out.truncated).bool()
        if not bool(d.any()):
            continue
        auto = out.obs[d].clone()
        assert torch.equal(auto, auto[:, :1].expand_as(auto))
        goals = out.obs[:, 0, 12:15].contiguous()
        r = g.reset(mask=d, goals=goals)          # rewrites the same rows in place
        assert torch.equal(r[d], auto)
        seen += int(d.sum())
    assert seen >= n // 2
    g.close()


def test_trim_parity_and_level_flight(torch_mod):
    torch = torch_mod
    n = 16
    ic = np.tile(default_ic(), (n, 1))
    ic[:, 2] = np.linspace(3000, 30000, n)
    ic[:, 3] = np.linspace(700, 1100, n)
    ref, g = _pair(n, 1, seed=0)
    t_r, res_r = ref.trim(ic)
    t_g, res_g = g.trim(ic)
    t_g, res_g = t_g.cpu().numpy(), res_g.cpu().numpy()
    assert np.all(res_r < 1e-3)
    assert np.all(res_g < 2e-2), res_g
    np.testing.assert_allclose(t_g[:, 7], t_r[:, 7], atol=2e-4)     # alpha = theta
    np.testing.assert_allclose(t_g[:, 13], t_r[:, 13], atol=2e-3)   # elevator cmd
    np.testing.assert_allclose(t_g[:, 15], t_r[:, 15], atol=2e-3)   # throttle cmd
    # fly the oracle's trim on both paths: smooth, so the tolerance holds over 40 s
    goals = np.zeros((n, 3), np.float32)
    o_r = ref.reset(goals=goals, ic=t_r)
    g.reset(goals=goals, ic=t_r)
    act = np.zeros((n, 4), np.float32)
    act[:, 1], act[:, 3] = t_r[:, 13], t_r[:, 15]
    ta = torch.as_tensor(act).cuda()
    h0 = o_r[:, 0, 2].copy()
    for t in range(1199):  # step 1200 truncates and auto-resets
        o_r, *_ = ref.step(act)
        out = g.step(ta)
    o_g = out.obs.cpu().numpy()
    tol = np.array([2.0, 2.0, 0.5, 1e-4, 1e-4, 1e-4, 1e-4, 1e-4, 1e-4, 1e-3, 1e-4, 1e-3, 0, 0, 0])
    _assert_frames(o_g[:, -1], o_r[:, -1], tol, "trimmed flight @1199")
    assert np.all(np.abs(o_r[:, -1, 2] - h0) < 60.0)


@pytest.mark.parametrize("n,k,steps", [(65536, 4, 200), (4171, 2, 40), (2113, 10, 40), (1000, 8, 40), (777, 3, 40),
                                       (65, 1, 40), (300, 11, 40), (1, 4, 40), (63, 10, 40)])
def test_large_batch_properties(torch_mod, n, k, steps):
    """65 536 envs (BASELINE cfg3 shape), 200 random-action steps: finite outputs, the
    ordered-stack invariant obs[t][:, :-1] == obs[t-1][:, 1:] on continuing lanes
    (bit-exact), auto-reset rows are K copies, determinism across handles, and the
    in-place (obs_prev == obs) ABI mode equals the ping-pong mode bit for bit. Smaller
    ragged batches (partial last wave) and other stack depths cover the split early/late
    obs rebuild and the flat-copy fallback."""
    torch = torch_mod
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd._lib import lib
    a = F16Envs(n, stack_k=k, seed=9)
    b = F16Envs(n, stack_k=k, seed=9)
    a.reset()
    b.reset()
    prev = a.obs.clone()
    inplace = b.obs  # b steps in place through the raw ABI
    L = lib()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    n_done_total = 0
    for t in range(steps):
        act = a.sample_actions(3, t)
        out = a.step(act)
        rc = L.f16env_step(b._h, stream, act.data_ptr(), inplace.data_ptr(), inplace.data_ptr(), b.rew.data_ptr(),
                           b.term.data_ptr(), b.trunc.data_ptr(), b.terminal_obs.data_ptr(), b.ep_return.data_ptr(),
                           b.ep_len.data_ptr(), None, None)
        assert rc == 0
        done = (out.terminated | out.truncated).bool()
        n_done_total += int(done.sum())
        assert torch.isfinite(out.obs).all()
        assert torch.equal(out.obs, inplace)
        assert torch.equal(out.rew, b.rew)
        cont = ~done
        assert torch.equal(out.obs[cont, :-1], prev[cont, 1:])
        if done.any():
            assert torch.equal(out.terminal_obs[done, :-1], prev[done, 1:])
            r = out.obs[done]
            assert torch.equal(r, r[:, :1].expand_as(r))
        prev = out.obs.clone()
    assert n_done_total > 0 or n < 65536


def test_done_index_compaction(torch_mod):
    torch = torch_mod
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd._lib import lib
    n = 5000
    ic = np.tile(default_ic(), (n, 1))
    ic[:, 2] = np.linspace(100.0, 3000.0, n)
    ic[:, 7] = -0.8
    e = F16Envs(n, stack_k=2, seed=1)
    e.reset(ic=ic)
    idx = torch.zeros(n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    L = lib()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    act = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
    seen = 0
    for t in range(20):
        nxt = e._obs[e._cur ^ 1]
        rc = L.f16env_step(e._h, stream, act.data_ptr(), e.obs.data_ptr(), nxt.data_ptr(), e.rew.data_ptr(),
                           e.term.data_ptr(), e.trunc.data_ptr(), e.terminal_obs.data_ptr(), e.ep_return.data_ptr(),
                           e.ep_len.data_ptr(), idx.data_ptr(), cnt.data_ptr())
        assert rc == 0
        e._cur ^= 1
        want = torch.nonzero((e.term | e.trunc).bool()).flatten().cpu().numpy()
        got = np.sort(idx[: int(cnt.item())].cpu().numpy())
        np.testing.assert_array_equal(got, want)
        seen += len(want)
    assert seen > 0


def test_vecenv_sb3_contract(torch_mod):
    from f16_jsb_amd import F16VecEnv, reference_goal
    n = 8
    env = F16VecEnv(num_envs=n, stack_k=10, seed=0)
    assert env.observation_space.shape == (10, 15) and env.action_space.shape == (4,)
    seeds = env.seed(100)
    obs = env.reset()
    assert isinstance(obs, np.ndarray) and obs.shape == (n, 10, 15) and obs.dtype == np.float32
    for i, s in enumerate(seeds):
        np.testing.assert_array_equal(obs[i, 0, 12:], reference_goal(s))
    total = 0
    for t in range(1300):
        obs, rew, dones, infos = env.step(np.tile(np.array([[0, -0.2, 0, 0.8]], np.float32), (n, 1)))
        assert obs.shape == (n, 10, 15) and rew.dtype == np.float32 and dones.dtype == bool
        assert len(infos) == n and all("TimeLimit.truncated" in i for i in infos)
        for i in np.flatnonzero(dones):
            assert infos[i]["terminal_observation"].shape == (10, 15)
            ep = infos[i]["episode"]
            assert set(ep) == {"r", "l", "t"} and ep["l"] <= 1200
            total += 1
    assert total >= n  # every lane finished at least once (crash / goal / 1200-step truncation)
    env.close()


@pytest.mark.parametrize("k,cfg5", [(4, False), (10, False), (4, True)])
def test_vecenv_host_window_matches_full_copy(torch_mod, k, cfg5):
    """F16VecEnv numpy mode with the host window mirror (_HostWindow: only the step's new frame
    slots cross PCIe, the host repeats the kernel's reset-window fills) against whole-observation
    copies (copy_obs=True) on identical handles: observations, rewards, dones, terminal
    observations and episode statistics bit-identical at every step, through short episodes
    (auto-resets every few steps, cfg5's in-step resets), device window restarts (history 16)
    and host ring restarts (Th = 2K + 3); the obs returned one step earlier is unchanged."""
    from f16_jsb_amd.env import F16VecEnv, _HostStaging, _HostWindow
    n = 700
    kw = dict(num_envs=n, stack_k=k, seed=3, max_steps=7, history=max(16, 2 * k), cfg5=cfg5)
    a = F16VecEnv(**kw)
    a._host = _HostWindow(a.envs, th=2 * k + 3)
    b = F16VecEnv(copy_obs=True, **kw)
    assert isinstance(b._host, _HostStaging) and not isinstance(b._host, _HostWindow)
    np.testing.assert_array_equal(a.reset(), b.reset())
    rng = np.random.default_rng(1)
    prev = None
    ended = 0
    for t in range(60):
        act = rng.uniform([-1, -1, -1, 0], [1, 1, 1, 1], (n, 4)).astype(np.float32)
        oa, ra, da, ia = a.step(act)
        ob, rb, db, ib = b.step(act)
        np.testing.assert_array_equal(oa, ob, err_msg="obs @%d" % t)
        np.testing.assert_array_equal(ra, rb)
        np.testing.assert_array_equal(da, db)
        for i in np.flatnonzero(db):
            np.testing.assert_array_equal(ia[i]["terminal_observation"], ib[i]["terminal_observation"])
            assert ia[i]["episode"]["r"] == ib[i]["episode"]["r"] and ia[i]["episode"]["l"] == ib[i]["episode"]["l"]
            assert ia[i]["TimeLimit.truncated"] == ib[i]["TimeLimit.truncated"]
            ended += 1
        if prev is not None:
            np.testing.assert_array_equal(prev[0], prev[1], err_msg="previous obs changed @%d" % t)
        prev = (oa, oa.copy())
    assert ended > n
    a.close()
    b.close()


def test_global_table_variant_bit_identical(torch_mod, monkeypatch):
    """The global-table step kernel (chosen when the K-frame stack image fills LDS, e.g. the
    reference's K = 10) runs the same arithmetic as the LDS-table kernel: forced on a K = 4
    handle (F16ENV_GT=1) it must reproduce the default handle bit for bit, and at K = 10 it
    is the variant the handle picks."""
    torch = torch_mod
    from f16_jsb_amd.env import F16Envs
    n = 3000
    a = F16Envs(n, stack_k=4, seed=5)
    monkeypatch.setenv("F16ENV_GT", "1")
    b = F16Envs(n, stack_k=4, seed=5)
    monkeypatch.delenv("F16ENV_GT")
    assert a.step_kernel_name == "f16_step_kernel" and b.step_kernel_name.startswith("f16_step_gt_kernel")
    a.reset()
    b.reset()
    for t in range(60):
        act = a.sample_actions(11, t)
        oa, ob = a.step(act), b.step(act)
        assert torch.equal(oa.obs, ob.obs) and torch.equal(oa.rew, ob.rew)
        assert torch.equal(oa.terminated, ob.terminated) and torch.equal(oa.truncated, ob.truncated)
    assert torch.equal(a.get_state(), b.get_state())
    c = F16Envs(256, stack_k=10, seed=5)
    assert c.step_kernel_name.startswith("f16_step_gt_kernel")
    for h in (a, b, c):
        h.close()


def test_cfg2_trimmed_level_flight_4096(torch_mod):
    """BASELINE cfg2: 4096 envs on a 64 x 64 grid of altitudes [3000, 30000] ft x
    airspeeds [600, 1200] fps, each trimmed for level flight (the oracle's trim, the
    reference never trims), constant trim action, both paths flown 1199 steps (step 1200
    truncates). Per-state comparison at steps {1, 10, 100, 1199}; the trimmed aircraft hold
    altitude. Tolerances: 4x the step tolerance at 1-10 steps, the 300-step constant-action
    tolerance at 100, and tol_long (below) after 40 s."""
    torch = torch_mod
    n = 4096
    ic = np.tile(default_ic(), (n, 1))
    hh, uu = np.meshgrid(np.linspace(3000, 30000, 64), np.linspace(600, 1200, 64), indexing="ij")
    ic[:, 2], ic[:, 3] = hh.ravel(), uu.ravel()
    ref, g = _pair(n, 4, seed=3)
    t_r, res_r = ref.trim(ic)
    ok = res_r.max(axis=1) < 1e-3  # corners of the envelope (slow and high) may not trim
    assert ok.mean() > 0.8, ok.mean()
    goals = np.zeros((n, 3), np.float32)
    goals[:, 2] = 50000.0  # no goal capture
    o_r = ref.reset(goals=goals, ic=t_r)
    g.reset(goals=goals, ic=t_r)
    act = np.zeros((n, 4), np.float32)
    act[:, 1], act[:, 3] = t_r[:, 13], t_r[:, 15]
    ta = torch.as_tensor(act).cuda()
    h0 = o_r[:, 0, 2].copy()
    # after 40 s (measured max over the grid on MI355X: positions 1.3 m, mach 9.7e-5, theta
    # 2.1e-4 rad -- the lightly damped phugoid amplifies fp32-vs-fp64 differences), ~2.5-5x margin
    tol_long = np.array([3.0, 3.0, 3.0, 3e-4, 5e-5, 1e-5, 5e-5, 5e-5, 1e-5, 2e-4, 6e-4, 5e-5, 0, 0, 0])
    for t in range(1, 1200):
        o_r, r_r, te_r, tr_r, *_ = ref.step(act)
        out = g.step(ta)
        if t in (1, 10, 100, 1199):
            te_g = out.terminated.cpu().numpy().astype(bool)
            live = ok & ~te_r & ~te_g
            tol = TOL_STEP * 4 if t <= 10 else (TOL_CONST300 if t == 100 else tol_long)
            _assert_frames(out.obs.cpu().numpy()[live, -1], o_r[live, -1], tol, "cfg2 trimmed @%d" % t)
    assert np.median(np.abs(o_r[ok, -1, 2] - h0[ok])) < 30.0


def test_cfg2_device_trim_grid_4096(torch_mod):
    """BASELINE cfg2 as bench.py runs it: the DEVICE trim (f16_trim_kernel, fp32 Newton) of the
    64 x 64 altitude x airspeed grid against the oracle's fp64 trim of the same grid: wherever
    the oracle converges (residual < 1e-3), the device trim converges too (residual < 1e-3) to
    the same (alpha, elevator, throttle); then the device-trimmed ICs are flown 1 199 steps on
    both paths with their constant trim action (the reference never trims: jsbsim_gym.py:
    166-170), per state at steps {1, 10, 100, 1199} as test_cfg2_trimmed_level_flight_4096."""
    torch = torch_mod
    n = 4096
    ic = np.tile(default_ic(), (n, 1))
    hh, uu = np.meshgrid(np.linspace(3000, 30000, 64), np.linspace(600, 1200, 64), indexing="ij")
    ic[:, 2], ic[:, 3] = hh.ravel(), uu.ravel()
    ref, g = _pair(n, 4, seed=3)
    t_r, res_r = ref.trim(ic)
    t_g, res_g = g.trim(ic)
    t_g, res_g = t_g.cpu().numpy(), res_g.cpu().numpy()
    ok_r = res_r.max(axis=1) < 1e-3
    ok_g = res_g.max(axis=1) < 1e-3
    print("cfg2 grid: oracle trimmed %.4f, device trimmed %.4f, device residual on the oracle's set: max %.2e "
          "p99 %.2e; |d alpha| max %.2e, |d ele| %.2e, |d thr| %.2e" % (
              ok_r.mean(), ok_g.mean(), res_g[ok_r].max(), np.percentile(res_g[ok_r].max(axis=1), 99),
              np.abs(t_g[ok_r, 7] - t_r[ok_r, 7]).max(), np.abs(t_g[ok_r, 13] - t_r[ok_r, 13]).max(),
              np.abs(t_g[ok_r, 15] - t_r[ok_r, 15]).max()))
    assert ok_r.mean() > 0.95, ok_r.mean()
    assert ok_g[ok_r].all(), "device trim residual >= 1e-3 where the oracle converged: %s" % res_g[ok_r & ~ok_g][:4]
    np.testing.assert_allclose(t_g[ok_r, 7], t_r[ok_r, 7], atol=2e-4)    # alpha = theta
    np.testing.assert_allclose(t_g[ok_r, 13], t_r[ok_r, 13], atol=2e-3)  # elevator cmd
    np.testing.assert_allclose(t_g[ok_r, 15], t_r[ok_r, 15], atol=2e-3)  # throttle cmd
    goals = np.zeros((n, 3), np.float32)
    goals[:, 2] = 50000.0
    o_r = ref.reset(goals=goals, ic=t_g)
    g.reset(goals=goals, ic=t_g)
    act = np.zeros((n, 4), np.float32)
    act[:, 1], act[:, 3] = t_g[:, 13], t_g[:, 15]
    ta = torch.as_tensor(act).cuda()
    h0 = o_r[:, 0, 2].copy()
    tol_long = np.array([3.0, 3.0, 3.0, 3e-4, 5e-5, 1e-5, 5e-5, 5e-5, 1e-5, 2e-4, 6e-4, 5e-5, 0, 0, 0])
    for t in range(1, 1200):
        o_r, r_r, te_r, tr_r, *_ = ref.step(act)
        out = g.step(ta)
        if t in (1, 10, 100, 1199):
            te_g = out.terminated.cpu().numpy().astype(bool)
            np.testing.assert_array_equal(te_g, te_r)
            live = ok_r & ~te_r
            tol = TOL_STEP * 4 if t <= 10 else (TOL_CONST300 if t == 100 else tol_long)
            _assert_frames(out.obs.cpu().numpy()[live, -1], o_r[live, -1], tol, "cfg2 device trim @%d" % t)
    assert np.median(np.abs(o_r[ok_r, -1, 2] - h0[ok_r])) < 30.0


def test_gymnasium_vector_env_contract(torch_mod):
    """gymnasium VectorEnv surface (F16GymVectorEnv, autoreset SAME_STEP): batched spaces,
    reset(seed=s) seeds env i with s + i (reference goals, bit-exact), step -> (obs, rew,
    terminated, truncated, infos) with final_obs / episode + their "_" masks on the lanes that
    finished, and the same transitions as the SB3 VecEnv over the same kernel."""
    import f16_jsb_amd
    from f16_jsb_amd import F16VecEnv, reference_goal
    n = 16
    env = f16_jsb_amd.make_vec("JSBSim-v0", num_envs=n, stack_k=4, seed=0, max_steps=7)
    sb3 = F16VecEnv(num_envs=n, stack_k=4, seed=0, max_steps=7)
    assert env.single_observation_space.shape == (4, 15) and env.observation_space.shape == (n, 4, 15)
    assert env.single_action_space.shape == (4,) and env.action_space.shape == (n, 4)
    assert env.metadata["autoreset_mode"] == "SameStep"
    obs, info = env.reset(seed=42)
    sb3.seed(42)
    obs_s = sb3.reset()
    assert info == {} and obs.shape == (n, 4, 15) and obs.dtype == np.float32
    for i in range(n):
        np.testing.assert_array_equal(obs[i, 0, 12:], reference_goal(42 + i))
    np.testing.assert_array_equal(obs, obs_s)
    act = np.tile(np.array([[0.1, -0.1, 0.0, 0.7]], np.float32), (n, 1))
    finished = 0
    for t in range(15):
        obs, rew, term, trunc, infos = env.step(act)
        obs_s, rew_s, dones_s, infos_s = sb3.step(act)
        np.testing.assert_array_equal(obs, obs_s)
        np.testing.assert_array_equal(rew, rew_s)
        done = term | trunc
        np.testing.assert_array_equal(done, dones_s)
        assert term.dtype == bool and trunc.dtype == bool and rew.dtype == np.float32
        if done.any():
            assert set(infos) == {"final_obs", "_final_obs", "episode", "_episode"}
            np.testing.assert_array_equal(infos["_final_obs"], done)
            for i in np.flatnonzero(done):
                np.testing.assert_array_equal(infos["final_obs"][i], infos_s[i]["terminal_observation"])
                assert infos["episode"]["l"][i] == infos_s[i]["episode"]["l"]
                assert infos["episode"]["r"][i] == infos_s[i]["episode"]["r"]
                finished += 1
        else:
            assert infos == {}
    assert finished >= 2 * n  # truncation at 7 steps
    env.close()
    sb3.close()


def test_nan_guard_quarantines_nonfinite_lanes(torch_mod):
    """F16_FLAG_NAN_GUARD (failure detection): lanes whose state is poisoned (NaN
    inertial velocity injected through f16env_set_state) end their next step terminated == 3
    with reward 0, come back as finite reset rows, and are counted; the other lanes step bit for
    bit as without the guard. Without the guard the NaN reaches the observation, as it would in
    the reference (jsbsim_gym.py:268-285 only prints a warning)."""
    torch = torch_mod
    from f16_jsb_amd.abi import F16C_VI
    from f16_jsb_amd.env import F16Envs
    n = 256
    a = F16Envs(n, stack_k=4, seed=2, nan_guard=True)
    b = F16Envs(n, stack_k=4, seed=2)
    a.reset()
    b.reset()
    for t in range(5):
        act = a.sample_actions(1, t)
        a.step(act)
        b.step(act)
    bad = [3, 77, 200]
    for h in (a, b):
        s = h.get_state()
        s[bad, F16C_VI] = float("nan")
        h.set_state(s)
    act = a.sample_actions(1, 99)
    oa, ob = a.step(act), b.step(act)
    term = oa.terminated.cpu().numpy()
    assert list(np.flatnonzero(term == 3)) == bad
    assert (oa.rew.cpu().numpy()[bad] == 0).all()
    assert torch.isfinite(oa.obs).all()
    assert a.nonfinite_count == len(bad) and b.nonfinite_count == 0
    good = torch.as_tensor(np.setdiff1d(np.arange(n), bad)).cuda()
    assert torch.equal(oa.obs[good], ob.obs[good]) and torch.equal(oa.rew[good], ob.rew[good])
    assert not bool(torch.isfinite(ob.obs[bad]).all())
    a.close()
    b.close()


@pytest.mark.parametrize("layout", ["contiguous", "window"])
def test_obs_bounds_diagnostic_counts_like_oracle(torch_mod, layout):
    """F16_FLAG_OBS_CHECK: the device counterpart of jsbsim_gym.py:268-285 (a FINITE value
    outside the observation space, SINGLE_OBS_LOW / HIGH :28-53). Lanes given a goal below
    ground (goal z < 0 through set_state) put a finite out-of-bounds value into every new frame;
    the device count of such lane-steps equals the oracle's, the physics is unchanged (same
    frames as a handle without the check), and in-bounds flight counts nothing."""
    torch = torch_mod
    from f16_jsb_amd.abi import F16_FLAG_OBS_CHECK, F16C_GOAL
    from f16_jsb_amd.env import F16Envs
    n, steps = 512, 20
    ref = OracleEnvs(n, stack_k=4, seed=9, flags=F16_FLAG_OBS_CHECK)
    g = F16Envs(n, stack_k=4, seed=9, obs_check=True, obs_layout=layout)
    plain = F16Envs(n, stack_k=4, seed=9, obs_layout=layout)
    o = ref.reset()
    g.reset()
    plain.reset()
    for t in range(1, 4):  # in bounds: nothing counted
        a = ref.sample_actions(2, t)
        ref.step(a)
        g.step(torch.as_tensor(a).cuda())
        plain.step(torch.as_tensor(a).cuda())
    assert g.obs_bounds_count == 0 and ref.obs_bounds_count == 0
    s = ref.get_state()
    bad = np.arange(n) % 7 == 0
    s[bad, F16C_GOAL + 2] = -100.0
    ref.set_state(s)
    for h in (g, plain):
        h.set_state(s)
    for t in range(4, 4 + steps):
        a = ref.sample_actions(2, t)
        ref.step(a)
        og = g.step(torch.as_tensor(a).cuda())
        op = plain.step(torch.as_tensor(a).cuda())
        assert torch.equal(og.obs, op.obs) and torch.equal(og.rew, op.rew)
    assert ref.obs_bounds_count == int(bad.sum()) * steps
    assert g.obs_bounds_count == ref.obs_bounds_count
    for h in (ref, g, plain):
        h.close()


def test_host_checks_refuse_misshaped_buffers(torch_mod):
    """Buffers the kernels index by env are shape-checked on the host before any launch (a
    wrong size would be an out-of-bounds device access), and the handle stays usable."""
    torch = torch_mod
    from f16_jsb_amd.env import F16Envs
    n = 70
    g = F16Envs(n, stack_k=4, seed=2)
    g.reset()
    a = g.sample_actions(1, 0)
    i32 = dict(dtype=torch.int32, device="cuda")
    f32 = dict(dtype=torch.float32, device="cuda")
    with pytest.raises(ValueError):
        g.reset(mask=torch.ones(n - 1, dtype=torch.bool, device="cuda"))
    with pytest.raises(ValueError):
        g.step(a[:-1])
    with pytest.raises(ValueError):
        g.step(a, done_idx=torch.zeros(n - 6, **i32), n_done=torch.zeros(1, **i32))
    with pytest.raises(ValueError):
        g.step(a, done_idx=torch.zeros(n, **i32))
    with pytest.raises(ValueError):
        g.step_rollout(1, 0, frame=torch.zeros(n, 14, **f32))
    with pytest.raises(ValueError):
        g.step_rollout(1, 0, rewards=torch.zeros(n, dtype=torch.float64, device="cuda"))
    out = g.step(a, done_idx=torch.zeros(n, **i32), n_done=torch.zeros(1, **i32))
    assert torch.isfinite(out.obs).all()
    g.close()


@pytest.mark.parametrize("layout", ["contiguous", "window"])
def test_obs_bounds_counted_in_persistent_rollout(torch_mod, layout):
    """F16_FLAG_OBS_CHECK in the one-launch rollout (f16_rollout_kernel counts its frames the way
    the step kernel does): the same lane-steps as the oracle stepping the same
    Philox actions, with a seventh of the lanes given an underground goal."""
    torch = torch_mod
    from f16_jsb_amd.abi import F16_FLAG_OBS_CHECK, F16C_GOAL
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout
    n, T = 512, 20
    ref = OracleEnvs(n, stack_k=4, seed=9, flags=F16_FLAG_OBS_CHECK)
    g = F16Envs(n, stack_k=4, seed=9, obs_check=True, obs_layout=layout)
    o = ref.reset()
    g.reset()
    s = ref.get_state()
    bad = np.arange(n) % 7 == 0
    s[bad, F16C_GOAL + 2] = -100.0
    o[bad, :, 14] = -100.0
    ref.set_state(s)
    g.set_state(s)
    g.set_obs(torch.as_tensor(o))
    collect_rollout(g, DeviceRolloutBuffer(T, n, 4, g.device), 2, step0=4)  # one persistent launch
    for t in range(T):
        ref.step(ref.sample_actions(2, 4 + t))
    assert ref.obs_bounds_count > 0
    assert g.obs_bounds_count == ref.obs_bounds_count
    ref.close()
    g.close()
