"""Windowed observations (f16env_step_window, F16Envs(obs_layout="window")) against the
contiguous ping-pong layout (f16env_step) on identical handles: done flags and episode lengths
bit-identical, observations, rewards, episode returns and terminal observations equal up to
fp32 rounding (rtol 1e-5: the two layouts are different kernel instances of the same physics,
which the compiler may contract differently, e.g. one ulp in one of 30 720 terminal-frame
values of the cfg5 build) at every step -- across
history restarts (T small), auto-resets (short TimeLimit), deferred cfg5 resets, caller resets
(NO_AUTORESET), set_state / set_obs, one- and two-waves-per-SIMD builds -- and an observation
must stay unchanged until the step after next (the validity the ping-pong buffers give).

The reference's stack is JSBSimEnv.obs_buffer, a deque(maxlen=K) appended once per step
(jsbsim_gym.py:150, :235); the window layout is its device form: per env a frame history the
observation is a (N, K, 15) view of.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu



def _pair(n, k, T, **kw):
    from f16_jsb_amd.env import F16Envs
    a = F16Envs(n, stack_k=k, seed=7, **kw)
    b = F16Envs(n, stack_k=k, seed=7, obs_layout="window", history=T, **kw)
    return a, b


def _np(x):
    return x.cpu().numpy()


def _close(x, y, msg):
    # bit-identical: both layouts run the same per-expression FMA contraction (build.py
    # -ffp-contract=on), whatever kernel instance each picks
    np.testing.assert_array_equal(x, y, err_msg=msg)


def _compare(oa, ob, t, check_tobs=True):
    _close(_np(ob.obs), _np(oa.obs), "obs @%d" % t)
    _close(_np(ob.rew), _np(oa.rew), "rew @%d" % t)
    np.testing.assert_array_equal(_np(ob.terminated), _np(oa.terminated), err_msg="terminated @%d" % t)
    np.testing.assert_array_equal(_np(ob.truncated), _np(oa.truncated), err_msg="truncated @%d" % t)
    d = _np(oa.terminated).astype(bool) | _np(oa.truncated).astype(bool)
    if d.any():
        np.testing.assert_array_equal(_np(ob.ep_len)[d], _np(oa.ep_len)[d])
        _close(_np(ob.ep_return)[d], _np(oa.ep_return)[d], "episode return @%d" % t)
        if check_tobs:
            _close(_np(ob.terminal_obs)[d], _np(oa.terminal_obs)[d], "terminal obs @%d" % t)
    return int(d.sum())


def _run(a, b, steps, seed=3, validity=True):
    import torch
    oa, ob = a.reset(), b.reset()
    np.testing.assert_array_equal(_np(ob), _np(oa))  # the same reset kernel: bit-identical
    finished = 0
    prev = None  # (view returned one step ago, its values then)
    for t in range(1, steps + 1):
        act = a.sample_actions(seed, t)
        sa = a.step(act)
        sb = b.step(act)
        if validity and prev is not None:  # obs(t-1) must survive step t unchanged
            torch.testing.assert_close(prev[0], prev[1], rtol=0, atol=0)
        finished += _compare(sa, sb, t)
        prev = (sb.obs, sb.obs.clone())
    return finished


@pytest.mark.parametrize("k,T,n,max_steps", [(4, 8, 1000, 7), (1, 4, 300, 5), (2, 4, 500, 6), (10, 20, 600, 9),
                                             (4, 128, 4096, 1200)])
def test_window_matches_contiguous(gpu, k, T, n, max_steps):
    a, b = _pair(n, k, T, max_steps=max_steps)
    steps = 60 if max_steps < 1200 else 40
    finished = _run(a, b, steps)
    if max_steps < 1200:
        assert finished > n, "short episodes must auto-reset many lanes (%d)" % finished
    assert b.T == T


def test_window_headline_size(gpu):
    """BASELINE cfg3 size (65 536 envs, K = 4): the one-wave window kernel over a restart."""
    a, b = _pair(65536, 4, 16, max_steps=1200)
    assert b.step_kernel_name == "f16_step_win_nt_kernel<0, 1, false>"
    _run(a, b, 20, validity=False)


def test_window_two_waves_per_simd(gpu, monkeypatch):
    """The 256-register two-waves-per-SIMD build (F16ENV_OCC=2) in both layouts."""
    monkeypatch.setenv("F16ENV_OCC", "2")
    a, b = _pair(2048, 4, 8, max_steps=6)
    assert a.waves_per_simd == 2 and b.waves_per_simd == 2
    _run(a, b, 30)


@pytest.mark.parametrize("period", ["0", "1", "32"])
def test_window_cfg5_deferred_resets(gpu, monkeypatch, period):
    """cfg5 modes: random IC + gusts. The windowed step resets finished lanes itself from the
    reset cache (f16_ic_fill_kernel every `period` steps; a lane that finishes twice within a
    period runs its RunIC in the step): period 1 -- every reset a cache hit; 32 -- with
    max_steps 5, hits and in-step RunICs; 0 -- the deferred f16_reset_done_kernel instead.
    Against the contiguous layout's deferred resets: identical done flags, values to fp32
    rounding. (Round 2's all-zero rewards of this kernel instance were a register-allocation
    miscompile, see tests/test_isa_lint.py.)"""
    monkeypatch.setenv("F16ENV_ICC_PERIOD", period)
    a, b = _pair(512, 4, 8, max_steps=5, cfg5=True)
    assert b.step_kernel_name == "f16_step_win_nt_kernel<3, 1, false>"
    assert _run(a, b, 30) > 512


def test_window_deferred_reset_rollout_refused_before_launch(gpu, monkeypatch):
    """the deferred-reset windowed step (cfg5, F16ENV_ICC_PERIOD=0) cannot write a
    rollout slot's next_frame; the call is refused BEFORE any launch, so the state, the
    observation and the episode bookkeeping are those of before the call, and the handle keeps
    stepping bit-identically with a twin that never saw the refused call."""
    import torch
    from f16_jsb_amd._lib import F16EnvError
    from f16_jsb_amd.env import F16Envs
    monkeypatch.setenv("F16ENV_ICC_PERIOD", "0")
    kw = dict(stack_k=4, seed=9, max_steps=5, obs_layout="window", history=12, cfg5=True)
    a, b = F16Envs(300, **kw), F16Envs(300, **kw)
    a.reset(), b.reset()
    for t in range(1, 4):
        act = a.sample_actions(4, t)
        a.step(act), b.step(act)
    s0, o0 = a.get_state().clone(), a.obs.clone()
    nf = torch.zeros((300, 15), dtype=torch.float32, device=a.device)
    with pytest.raises(F16EnvError, match="deferred-reset"):
        a.step_rollout(7, 4, next_frame=nf)
    torch.cuda.synchronize()
    assert torch.equal(a.get_state(), s0) and torch.equal(a.obs, o0)
    assert float(nf.abs().max()) == 0.0
    for t in range(4, 12):  # keeps stepping as its twin (crashes / truncations at max_steps 5)
        act = a.sample_actions(4, t)
        sa, sb = a.step(act), b.step(act)
        assert torch.equal(sa.obs, sb.obs) and torch.equal(sa.rew, sb.rew)
        assert torch.equal(sa.terminated, sb.terminated) and torch.equal(sa.truncated, sb.truncated)


def test_window_caller_resets(gpu):
    """NO_AUTORESET: finished lanes keep stepping until the caller resets them (mask)."""
    import torch
    a, b = _pair(700, 4, 8, max_steps=4, autoreset=False)
    a.reset(), b.reset()
    for t in range(1, 25):
        act = a.sample_actions(11, t)
        sa, sb = a.step(act), b.step(act)
        _compare(sa, sb, t, check_tobs=False)
        done = (sa.terminated | sa.truncated).to(torch.uint8)
        if t % 3 == 0:
            ra, rb = a.reset(mask=done), b.reset(mask=done)
            m = _np(done).astype(bool)  # the reset rows come from the same reset kernel: bit-exact
            np.testing.assert_array_equal(_np(rb)[m], _np(ra)[m])
            _close(_np(rb)[~m], _np(ra)[~m], "unreset rows @%d" % t)


def test_window_set_state_and_obs(gpu):
    """A window handle takes a contiguous handle's state + observation mid-run and continues
    bit-identically (set_obs writes both histories' windows)."""
    from f16_jsb_amd.env import F16Envs
    a = F16Envs(800, stack_k=4, seed=5, max_steps=8)
    a.reset()
    for t in range(1, 6):
        a.step(a.sample_actions(2, t))
    b = F16Envs(800, stack_k=4, seed=5, max_steps=8, obs_layout="window", history=12)
    b.set_state(a.get_state())
    b.set_obs(a.obs)
    for t in range(6, 40):
        act = a.sample_actions(2, t)
        _compare(a.step(act), b.step(act), t)


@pytest.mark.parametrize("cfg5", [False, True], ids=["reference_task", "cfg5"])
def test_window_reset_then_set_state_keeps_fresh(gpu, cfg5):
    """reset -> set_state(get_state()) -> steps, with no set_obs (bench.py's spread_phases
    sequence): the windowed handle keeps each lane's "reset since the last step" mark across
    set_state, so the first observation after it carries K-1 copies of the reset frame, as the
    contiguous layout's does (a fresh handle's other history is still all zeros)."""
    a, b = _pair(700, 4, 16, max_steps=50, cfg5=cfg5)
    np.testing.assert_array_equal(_np(b.reset()), _np(a.reset()))
    a.set_state(a.get_state())
    b.set_state(b.get_state())
    for t in range(1, 13):
        act = a.sample_actions(5, t)
        _compare(a.step(act), b.step(act), t)


def test_window_views_and_layout(gpu):
    """The observation is a strided view of position-major 64-B frame slots: (N, K, 15), strides
    (16, N*16, 1), the slots' 16th float 0. (The rollout entry points take the window layout since
    round 4, tests/test_gpu_policy_rollout.py; their buffers are checked before any launch.)"""
    from f16_jsb_amd.env import F16Envs
    e = F16Envs(64, stack_k=4, seed=1, obs_layout="window", history=16)
    o = e.reset()
    assert tuple(o.shape) == (64, 4, 15) and o.stride() == (16, 64 * 16, 1)
    for t in range(1, 30):  # across a restart
        e.step(e.sample_actions(1, t))
    assert float(e._hist[..., 15].abs().max()) == 0.0
    with pytest.raises(ValueError):
        e.rollout_random(0, 0, 2, None, None, None, None, None)


@pytest.mark.parametrize("k,T", [(4, 8), (1, 4)])
def test_window_env_major_order(gpu, k, T):
    """window_order="env" ([N][T][16] histories, view strides (T*16, 16, 1)) against the
    contiguous layout: the kernel's generic (position, env) slot addressing."""
    from f16_jsb_amd.env import F16Envs
    a = F16Envs(700, stack_k=k, seed=7, max_steps=6)
    b = F16Envs(700, stack_k=k, seed=7, max_steps=6, obs_layout="window", history=T, window_order="env")
    assert _run(a, b, 40) > 700
    assert b.obs.stride() == (T * 16, 16, 1)
