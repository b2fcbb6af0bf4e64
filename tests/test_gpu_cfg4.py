"""BASELINE cfg4's per-GPU share through the kernel that runs it: 32 768 envs x PPO n_steps
2 048, K = 4, one f16_rollout_kernel launch (f16env_rollout_random / f16env_window_rollout_random
in the windowed layout; bench.py rollout_bench),
which replaces n_steps iterations of collect_rollouts' env.step + RolloutBuffer.add
(on_policy_algorithm.py:194-262, buffers.py:440-479; the env step is jsbsim_gym.py:199-287).

  * oracle parity: the first 30 slots against oracle/f16ref.c stepping the same Philox
    actions from the same state -- actions and episode starts bit-exact, rewards 2e-3, the
    slot frames (newest frame of the observation each action acted on) at TOL_RAND30 at slot
    30 and within TOL_STEP at slot 1; a third of the lanes' step counters are staggered so
    they truncate and auto-reset inside the window;
  * properties over the whole T = 2 048 rollout from there: every value finite; per lane the
    episode starts agree with the state's episode counter and step counter before / after
    (each start is one reset, the step counter after equals the steps since the last start);
    no episode longer than max_steps (TimeLimit, jsbsim_gym.py:159); the env's final
    observation continues the stack rebuilt from the buffer (rebuild_observations, the
    frame-deduplicated layout the RCCL gather ships), and is K copies of the reset frame
    where the last slot ended an episode (dummy_vec_env.py:68-71).
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle_ref import OracleEnvs  # noqa: E402
from reward_bound import reward_atol  # noqa: E402
from test_gpu_parity import TOL_RAND30, TOL_STEP, _assert_frames  # noqa: E402

from f16_jsb_amd.abi import F16C_EP_COUNT, F16C_STEP  # noqa: E402

N, K, T, SEED = 32768, 4, 2048, 71


@pytest.mark.parametrize("layout", ["window", "contiguous"])
def test_cfg4_rollout_kernel_per_gpu_share(gpu, layout):
    """window: f16env_window_rollout_random (the final observation written into both window
    histories); contiguous: f16env_rollout_random -- the same kernel, f16_rollout_kernel<0, 1>."""
    import torch
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout, rebuild_observations
    ref, g = OracleEnvs(N, stack_k=K, seed=SEED), F16Envs(N, stack_k=K, seed=SEED, obs_layout=layout)
    o = ref.reset()
    g.reset()
    s = ref.get_state()
    k = np.arange(N)
    sel = k % 3 == 0
    s[sel, F16C_STEP] = ref.cfg.max_steps - 1 - (k[sel] // 3) % 25
    ref.set_state(s)
    g.set_state(s)
    g.set_obs(torch.as_tensor(o))

    # --- 30 slots against the oracle -------------------------------------------------------
    t30 = 30
    buf = DeviceRolloutBuffer(t30, N, K, gpu)
    collect_rollout(g, buf, SEED, step0=0)
    fr = buf.frames.cpu().numpy()
    ac = buf.actions.cpu().numpy()
    rw = buf.rewards.cpu().numpy()
    st = buf.episode_starts.cpu().numpy()
    last_start = g._last_episode_starts.cpu().numpy()
    o_prev = o
    resets = 0
    for t in range(t30):
        a = ref.sample_actions(SEED, t)
        np.testing.assert_array_equal(ac[t], a, err_msg="actions @%d" % t)
        tol = TOL_STEP if t == 0 else TOL_RAND30
        _assert_frames(fr[t], o_prev[:, -1], tol, "slot frame @%d" % t)
        o_r, r_r, te_r, tr_r, *_ = ref.step(a)
        np.testing.assert_allclose(rw[t], r_r, atol=reward_atol(TOL_RAND30), err_msg="reward @%d" % t)
        d = (te_r | tr_r).astype(np.float32)
        nxt = st[t + 1] if t + 1 < t30 else last_start
        np.testing.assert_array_equal(nxt, d, err_msg="episode starts @%d" % (t + 1))
        resets += int(d.sum())
        o_prev = o_r
    assert resets >= N // 3, resets
    _assert_frames(g.obs.cpu().numpy()[:, -1], o_prev[:, -1], TOL_RAND30, "env obs after 30 slots")
    ref.close()
    del buf

    # --- the whole PPO rollout (n_steps = 2 048) as bench.py runs it: properties -------------
    s0 = g.get_state().cpu().numpy()
    buf = DeviceRolloutBuffer(T, N, K, gpu)
    collect_rollout(g, buf, SEED + 1, step0=t30)
    torch.cuda.synchronize()
    s1 = g.get_state().cpu().numpy()
    last = g._last_episode_starts
    for name in ("frames", "actions", "rewards", "episode_starts"):
        assert bool(torch.isfinite(getattr(buf, name)).all()), name
    starts = torch.cat([buf.episode_starts[1:], last[None]])  # starts[t] = episode ended at step t
    n_starts = starts.sum(0).cpu().numpy().astype(np.int64)
    np.testing.assert_array_equal(s1[:, F16C_EP_COUNT] - s0[:, F16C_EP_COUNT], n_starts)
    # step counter after = steps since the last reset (or since the rollout began + before)
    tt = torch.arange(T, device=gpu, dtype=torch.float32)[:, None]
    last_end = torch.where(starts.bool(), tt, torch.full_like(tt.expand(T, N), -1.0)).max(0).values.cpu().numpy()
    want = np.where(last_end >= 0, T - 1 - last_end, s0[:, F16C_STEP] + T)
    np.testing.assert_array_equal(s1[:, F16C_STEP], want)
    # TimeLimit: no episode runs past max_steps
    ends = torch.nonzero(starts.T.bool())  # (env, t) sorted by env then t
    e_idx, t_idx = ends[:, 0].cpu().numpy(), ends[:, 1].cpu().numpy()
    first = np.r_[True, e_idx[1:] != e_idx[:-1]]
    prev_end = np.where(first, -1 - s0[e_idx, F16C_STEP], np.r_[0, t_idx[:-1]])
    assert (t_idx - prev_end).max() <= g.cfg.max_steps
    assert int(n_starts.sum()) > N, "expected many episode ends over 2 048 steps"
    # the final observation continues the rebuilt stack (newest frame appended), or is the reset
    # stack where the last step ended an episode
    last_obs = rebuild_observations(buf.frames, buf.obs0, buf.episode_starts, K, steps=[T - 1])[0]
    fin = g.obs
    cont = ~last.bool()
    assert torch.equal(fin[cont, :-1], last_obs[cont, 1:])
    assert torch.equal(fin[~cont], fin[~cont, :1].expand(-1, K, -1))
    assert bool(torch.isfinite(fin).all())
    g.close()
