"""GPU rollout path: HIP GAE kernel vs SB3's float32 numpy recurrence (bit-exact), and the
deduplicated device rollout buffer against the stacked observations the env kernel returns."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def numpy_gae(rewards, values, episode_starts, last_values, dones, gamma, gae_lambda):
    """stable_baselines3/common/buffers.py:403-438 restated (float32 numpy arrays)."""
    n = rewards.shape[0]
    adv = np.zeros_like(rewards)
    last_gae_lam = 0
    for step in reversed(range(n)):
        if step == n - 1:
            next_non_terminal = 1.0 - dones.astype(np.float32)
            next_values = last_values
        else:
            next_non_terminal = 1.0 - episode_starts[step + 1]
            next_values = values[step + 1]
        delta = rewards[step] + np.float32(gamma) * next_values * next_non_terminal - values[step]
        last_gae_lam = delta + np.float32(gamma * gae_lambda) * next_non_terminal * last_gae_lam
        adv[step] = last_gae_lam
    return adv, adv + values


@pytest.mark.parametrize("T,N", [(257, 1000), (2048, 32768), (37, 65541), (15, 70)])
def test_gae_bitexact(gpu, T, N):
    """The pipelined GAE kernel (32-step load blocks, a ragged top block first, full waves) at
    cfg4's per-GPU share 2 048 x 32 768, a ragged 65 541 envs and short rollouts (no whole block),
    bit for bit against buffers.py:403-438's numpy float32 recurrence."""
    import torch
    from f16_jsb_amd.rollout import DeviceRolloutBuffer
    rng = np.random.default_rng(T)
    buf = DeviceRolloutBuffer(T, N, 1, gpu, gamma=0.99, gae_lambda=0.95)
    r = rng.normal(size=(T, N)).astype(np.float32)
    v = rng.normal(size=(T, N)).astype(np.float32)
    st = (rng.random((T, N)) < 0.05).astype(np.float32)
    lv = rng.normal(size=N).astype(np.float32)
    dn = rng.random(N) < 0.1
    buf.rewards.copy_(torch.as_tensor(r))
    buf.values.copy_(torch.as_tensor(v))
    buf.episode_starts.copy_(torch.as_tensor(st))
    buf.pos = T
    buf.compute_returns_and_advantage(torch.as_tensor(lv).cuda(), torch.as_tensor(dn).cuda())
    adv, ret = numpy_gae(r, v, st, lv, dn, 0.99, 0.95)
    np.testing.assert_array_equal(buf.advantages.cpu().numpy(), adv)
    np.testing.assert_array_equal(buf.returns.cpu().numpy(), ret)


def test_rollout_buffer_rebuilds_env_observations(gpu):
    """Collect 96 steps from the HIP env (random actions, crashes/resets included): the
    stacks rebuilt from the deduplicated frames equal the env's returned observations."""
    import torch
    from oracle_ref import default_ic
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.rollout import DeviceRolloutBuffer
    n, k, T = 512, 4, 96
    ic = np.tile(default_ic(), (n, 1))
    ic[:, 2] = np.linspace(200.0, 8000.0, n)  # low lanes crash and auto-reset during the rollout
    ic[:, 7] = -0.3
    env = F16Envs(n, stack_k=k, seed=2)
    obs = env.reset(ic=ic).clone()
    buf = DeviceRolloutBuffer(T, n, k, gpu)
    starts = torch.ones(n, device=gpu)
    seen = []
    for t in range(T):
        act = env.sample_actions(1, t)
        buf.add(obs, act, torch.zeros(n, device=gpu), starts, torch.zeros(n, device=gpu), torch.zeros(n, device=gpu))
        seen.append(obs.clone())
        out = env.step(act)
        obs = out.obs.clone()
        starts = (out.terminated | out.truncated).float()
    assert int(buf.episode_starts[1:].sum().item()) > 0, "expected auto-resets in the rollout"
    rebuilt = buf.observations()
    assert torch.equal(rebuilt, torch.stack(seen))


def test_two_wave_variant_matches_one_wave_variant(gpu, monkeypatch):
    """The occupancy-2 build of the step kernel (picked above 64 x 4 x CUs envs) computes
    the same results as the one-wave build: forced on a small batch via F16ENV_OCC."""
    import torch
    from f16_jsb_amd.env import F16Envs
    n = 2048
    outs = []
    for occ in ("1", "2"):
        monkeypatch.setenv("F16ENV_OCC", occ)
        e = F16Envs(n, stack_k=4, seed=9)
        assert e.waves_per_simd == int(occ)
        e.reset()
        for t in range(40):
            o = e.step(e.sample_actions(4, t))
        outs.append((o.obs.clone(), o.rew.clone(), e.get_state()))
        e.close()
    torch.testing.assert_close(outs[1][0], outs[0][0], rtol=0, atol=0)
    torch.testing.assert_close(outs[1][1], outs[0][1], rtol=0, atol=0)
    torch.testing.assert_close(outs[1][2], outs[0][2], rtol=0, atol=0)


@pytest.mark.parametrize("n,k", [(4096, 4), (1000, 10), (777, 3)])
def test_fused_rollout_step_equals_sample_step_add(gpu, n, k):
    """f16env_step_rollout (one launch: in-kernel Philox actions + the slot's frame / actions /
    rewards / next episode starts) fills the buffer bit-identically to the unfused
    sample_actions -> step -> RolloutBuffer.add sequence, and leaves the envs in the same
    state; crashing lanes exercise the done-row paths, ragged N the partial last wave."""
    import torch
    from oracle_ref import default_ic
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout
    T = 48
    ic = np.tile(default_ic(), (n, 1))
    ic[:, 2] = np.linspace(150.0, 9000.0, n)
    ic[:, 7] = -0.35
    bufs, envs = [], []
    for fused in (False, True):
        e = F16Envs(n, stack_k=k, seed=4)
        e.reset(ic=ic)
        b = DeviceRolloutBuffer(T, n, k, gpu)
        collect_rollout(e, DeviceRolloutBuffer(3, n, k, gpu), 17, fused=fused, persistent=False)  # carry-over starts
        last_v, last_d = collect_rollout(e, b, 21, step0=100, fused=fused, persistent=False)
        bufs.append((b, last_d.clone()))
        envs.append(e)
    (b0, d0), (b1, d1) = bufs
    assert int(b0.episode_starts[1:].sum().item()) > 0, "expected auto-resets in the rollout"
    for f in ("frames", "actions", "rewards", "episode_starts", "obs0"):
        assert torch.equal(getattr(b0, f), getattr(b1, f)), f
    assert torch.equal(d0, d1)
    assert torch.equal(envs[0].obs, envs[1].obs)
    assert torch.equal(envs[0].get_state(), envs[1].get_state())
    # the rebuilt stacks are the env's observations
    assert torch.equal(b1.observations(steps=[T - 1])[0], b1.observations()[T - 1])
    for e in envs:
        e.close()


@pytest.mark.parametrize("cfg5", [False, True], ids=["reference_task", "cfg5"])
@pytest.mark.parametrize("layout", ["contiguous", "window"])
def test_persistent_rollout_two_wave_build_matches_fused_steps(gpu, monkeypatch, cfg5, layout):
    """the persistent rollout's 256-register build (f16_rollout_kernel<MODE, 2>, the
    launch's pick above 4 x CUs x 64 envs; forced here by F16ENV_ROLL_OCC=2 at a small N)
    against the fused rollout steps: bit-identical slots, final observation and state."""
    import torch
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout
    n, k, T = 1000, 4, 40
    kw = dict(stack_k=k, seed=6, max_steps=25, obs_layout=layout, cfg5=cfg5)
    if layout == "window":
        kw["history"] = 3 * k + T
    bufs, envs = [], []
    for persistent in (False, True):
        if persistent:
            monkeypatch.setenv("F16ENV_ROLL_OCC", "2")
        e = F16Envs(n, **kw)
        e.reset()
        b = DeviceRolloutBuffer(T, n, k, gpu)
        _, last_d = collect_rollout(e, b, 31, persistent=persistent)
        bufs.append((b, last_d.clone()))
        envs.append(e)
    monkeypatch.delenv("F16ENV_ROLL_OCC", raising=False)
    (b0, d0), (b1, d1) = bufs
    assert int(b0.episode_starts[1:].sum().item()) > 0, "expected auto-resets in the rollout"
    for f in ("frames", "actions", "rewards", "episode_starts", "obs0"):
        assert torch.equal(getattr(b0, f), getattr(b1, f)), f
    assert torch.equal(d0, d1)
    assert torch.equal(envs[0].obs, envs[1].obs)
    assert torch.equal(envs[0].get_state(), envs[1].get_state())
    for e in envs:
        e.close()


@pytest.mark.parametrize("order", ["position", "env"])
@pytest.mark.parametrize("warm", [1, 2])
def test_window_rollout_random_shortest_history(gpu, order, warm):
    """a windowed handle at the shortest history (T = 2K) whose window sits where no
    output window fits beside it (p in [K, 2K-2], after 1 or 2 steps): rollout_random moves the
    windows to the front first, and matches a contiguous twin bit for bit (slots, the final
    observation), then both keep stepping alike."""
    import torch
    from f16_jsb_amd.env import F16Envs
    n, k, steps = 500, 4, 6
    a = F16Envs(n, stack_k=k, seed=8, max_steps=5)
    b = F16Envs(n, stack_k=k, seed=8, max_steps=5, obs_layout="window", history=2 * k, window_order=order)
    a.reset(), b.reset()
    f32 = torch.float32
    for t in range(warm):
        act = a.sample_actions(3, t)
        a.step(act), b.step(act)
    assert k <= b._p <= 2 * k - 2
    outs = []
    for e in (a, b):
        fr = torch.empty((steps, n, 15), dtype=f32, device=gpu)
        ac = torch.empty((steps, n, 4), dtype=f32, device=gpu)
        rw = torch.empty((steps, n), dtype=f32, device=gpu)
        ns = torch.empty((steps - 1, n), dtype=f32, device=gpu)
        ls = torch.empty(n, dtype=f32, device=gpu)
        e.rollout_random(21, 10, steps, fr, ac, rw, ns, ls)
        outs.append((fr, ac, rw, ns, ls, e.obs.clone()))
    for x, y in zip(*outs):
        assert torch.equal(x, y)
    for t in range(20, 32):  # across restarts of the short history
        act = a.sample_actions(3, t)
        sa, sb = a.step(act), b.step(act)
        assert torch.equal(sa.obs, sb.obs) and torch.equal(sa.rew, sb.rew)
    a.close(), b.close()


@pytest.mark.parametrize("n,k,T", [(4096, 4, 64), (777, 3, 33), (300, 8, 1), (65, 1, 20)])
def test_persistent_rollout_matches_fused_steps(gpu, n, k, T):
    """f16env_rollout_random (the whole rollout in ONE launch, state kept on-chip, frames in an
    LDS ring) against T fused f16env_step_rollout launches: bit-identical -- actions, episode
    structure (Philox stream, crash / truncation / auto-reset steps), frames, rewards, the final
    observation and state. (Until round 3 they agreed only to fp32 rounding: the compiler
    contracted a few products differently in the two kernels; the library now fuses per source
    expression, build.py -ffp-contract=on.)"""
    import torch
    from oracle_ref import default_ic
    from parity_tools import frame_err
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout
    ic = np.tile(default_ic(), (n, 1))
    ic[:, 2] = np.linspace(150.0, 9000.0, n)
    ic[:, 7] = -0.35
    bufs, envs = [], []
    for persistent in (False, True):
        e = F16Envs(n, stack_k=k, seed=4, max_steps=40)
        e.reset(ic=ic)
        b = DeviceRolloutBuffer(T, n, k, gpu)
        collect_rollout(e, DeviceRolloutBuffer(3, n, k, gpu), 17, persistent=persistent)  # carry-over starts
        last_v, last_d = collect_rollout(e, b, 21, step0=100, persistent=persistent)
        bufs.append((b, last_d.clone()))
        envs.append(e)
    (b0, d0), (b1, d1) = bufs
    if T > 20:
        assert int(b0.episode_starts[1:].sum().item()) > 0, "expected auto-resets in the rollout"
    assert torch.equal(b0.actions, b1.actions)
    assert torch.equal(b0.episode_starts, b1.episode_starts)
    assert torch.equal(d0, d1)
    for f0, f1 in ((b0.frames, b1.frames), (b0.obs0, b1.obs0), (envs[0].obs, envs[1].obs)):
        assert torch.equal(f0, f1), np.unravel_index(np.argmax(frame_err(f1.cpu().numpy(), f0.cpu().numpy())), f0.shape)
    assert torch.equal(b0.rewards, b1.rewards)
    assert torch.equal(envs[0].get_state(), envs[1].get_state())
    for e in envs:
        e.close()
