"""Rollout-side host logic on CPU: stack rebuild from deduplicated frames, timeout bootstrap,
and the rank-0 gather over a world_size-2 gloo group (the RCCL path's CPU stand-in)."""
from __future__ import annotations

import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from f16_jsb_amd.rollout import DeviceRolloutBuffer, bootstrap_timeouts, env_major, gather_to_rank0, rebuild_observations


def _simulate_stacks(T, N, K, rng):
    """Run a deque-based stacker (jsbsim_gym.py:150,234-235,263 + reset fill :325-329) over
    random frames with random resets; return obs per step, newest frames, episode starts."""
    frames = rng.normal(size=(T, N, 15)).astype(np.float32)
    starts = (rng.random((T, N)) < 0.1).astype(np.float32)
    init = rng.normal(size=(N, K, 15)).astype(np.float32)  # stack before step 0
    stacks = init.copy()
    obs = np.zeros((T, N, K, 15), np.float32)
    for t in range(T):
        for e in range(N):
            if starts[t, e]:   # reset observation: K copies of the first frame
                stacks[e] = np.repeat(frames[t, e][None], K, axis=0)
            else:              # deque append
                stacks[e] = np.concatenate([stacks[e][1:], frames[t, e][None]])
            obs[t, e] = stacks[e]
    obs0 = obs[0].copy()
    return obs, frames, starts, obs0


@pytest.mark.parametrize("K", [1, 4, 10])
def test_rebuild_matches_deque_stacker(K):
    rng = np.random.default_rng(K)
    T, N = 37, 9
    obs, frames, starts, obs0 = _simulate_stacks(T, N, K, rng)
    got = rebuild_observations(torch.as_tensor(frames), torch.as_tensor(obs0), torch.as_tensor(starts), K).numpy()
    np.testing.assert_array_equal(got, obs)
    # subset of steps
    got2 = rebuild_observations(torch.as_tensor(frames), torch.as_tensor(obs0), torch.as_tensor(starts), K,
                                steps=[0, 5, 36]).numpy()
    np.testing.assert_array_equal(got2, obs[[0, 5, 36]])


def test_buffer_add_and_rebuild_cpu():
    rng = np.random.default_rng(0)
    T, N, K = 16, 5, 4
    obs, frames, starts, obs0 = _simulate_stacks(T, N, K, rng)
    buf = DeviceRolloutBuffer(T, N, K, "cpu")
    for t in range(T):
        buf.add(torch.as_tensor(obs[t]), torch.zeros(N, 4), torch.zeros(N), torch.as_tensor(starts[t]),
                torch.zeros(N), torch.zeros(N))
    assert buf.full
    np.testing.assert_array_equal(buf.observations().numpy(), obs)
    with pytest.raises(RuntimeError):
        buf.add(torch.as_tensor(obs[0]), torch.zeros(N, 4), torch.zeros(N), torch.zeros(N), torch.zeros(N), torch.zeros(N))
    with pytest.raises(RuntimeError):
        buf.compute_returns_and_advantage(torch.zeros(N), torch.zeros(N))


def test_bootstrap_timeouts_semantics():
    """on_policy_algorithm.py:236-245: only truncated-and-not-terminated lanes bootstrap."""
    r = torch.tensor([1.0, 2.0, 3.0, 4.0])
    term = torch.tensor([0, 1, 0, 1], dtype=torch.uint8)
    trunc = torch.tensor([1, 1, 0, 0], dtype=torch.uint8)
    v = torch.tensor([10.0, 20.0, 30.0, 40.0])
    out = bootstrap_timeouts(r, term, trunc, v, 0.99)
    want = np.array([np.float32(1.0) + np.float32(np.float32(0.99) * np.float32(10.0)), 2.0, 3.0, 4.0], np.float32)
    np.testing.assert_array_equal(out.numpy(), want)


def _gather_worker(rank, world, path, T, N, K, chunk, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    dist.init_process_group("gloo", init_method="file://" + path, rank=rank, world_size=world)
    g = torch.Generator().manual_seed(100 + rank)
    buf = DeviceRolloutBuffer(T, N, K, "cpu")
    for t in range(T):
        obs = torch.randn(N, K, 15, generator=g)
        buf.add(obs, torch.randn(N, 4, generator=g), torch.randn(N, generator=g),
                (torch.rand(N, generator=g) < 0.2).float(), torch.randn(N, generator=g), torch.randn(N, generator=g))
    buf.advantages.copy_(torch.randn(T, N, generator=g))
    buf.returns.copy_(buf.advantages + buf.values)
    out = gather_to_rank0(buf, chunk_steps=chunk)
    local = {k: v.clone() for k, v in buf.state_dict().items()}
    if rank == 0:
        q.put(("out", {k: v.numpy() for k, v in out.items()}))
    else:
        assert out is None
    q.put(("local%d" % rank, {k: v.numpy() for k, v in local.items()}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunk", [(2, 3), (3, 3)], ids=["world2", "world3_uneven_chunk"])
def test_gather_to_rank0_gloo(world, chunk):
    """Rank-major gather into one preallocated output: out[f][r] == rank r's shard, bit for bit,
    with T = 7 steps in chunks of 3 (3 + 3 + 1: a short last chunk)."""
    T, N, K = 7, 6, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "rdzv")
        procs = [ctx.Process(target=_gather_worker, args=(r, world, path, T, N, K, chunk, q)) for r in range(world)]
        for p in procs:
            p.start()
        got = dict(q.get(timeout=120) for _ in range(world + 1))
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
    out = got["out"]
    for f, v in out.items():
        want = np.stack([got["local%d" % r][f] for r in range(world)])
        np.testing.assert_array_equal(v, want, err_msg=f)
        if f != "obs0":  # the single-GPU (T, world * N) layout
            np.testing.assert_array_equal(env_major(torch.as_tensor(v)).numpy(),
                                          np.concatenate([got["local%d" % r][f] for r in range(world)], axis=1))
    assert out["frames"].shape == (world, T, N, 15) and out["obs0"].shape == (world, N, K, 15)


def test_np_clip_actions_matches_numpy():
    """The clip SB3 applies before env.step (on_policy_algorithm.py:216), numpy's semantics
    including NaN and signed zero (the kernel's np_clip computes the same)."""
    from f16_jsb_amd.rollout import ACTION_HIGH, ACTION_LOW, np_clip_actions
    rng = np.random.default_rng(3)
    a = (rng.normal(size=(257, 4)) * 2).astype(np.float32)
    a[:4] = [[np.nan, -0.0, np.inf, -0.0], [-np.inf, 0.0, -1.0, 1.0], [1.0, -1.0, -0.0, 0.0], [2.0, -2.0, 0.5, -3.0]]
    want = np.clip(a, np.array(ACTION_LOW, np.float32), np.array(ACTION_HIGH, np.float32))
    got = np_clip_actions(torch.as_tensor(a)).numpy()
    np.testing.assert_array_equal(got, want)
    assert np.array_equal(np.signbit(got), np.signbit(want))


def _linear_policy(scale=3.0):
    """A deterministic stand-in for SB3's policy(obs) -> (actions, values, log_probs) whose actions
    leave the Box (so the clip matters) and whose value depends on the observation."""
    g = torch.Generator().manual_seed(5)
    W = torch.randn(15, 4, generator=g)
    calls = []

    def policy(obs):
        x = obs[:, -1, :].to(torch.float32)
        a = scale * torch.tanh(x @ W * 0.1) + torch.tensor([0.0, 0.0, 0.0, -0.5])
        v = x[:, 1] * 0.25 - x[:, 0]
        lp = -(a * a).sum(-1)
        calls.append((obs.clone(), a.clone(), v.clone(), lp.clone()))
        return a, v, lp

    return policy, calls


def test_collect_rollout_policy_in_the_loop_cpu():
    """collect_rollouts (on_policy_algorithm.py:199-262) with a policy, host path over the CPU
    stand-in env: the env steps the clipped actions, the buffer keeps the unclipped ones with the
    values and log-probs, truncated-only lanes bootstrap gamma * V(terminal_obs), the last values
    are V(final obs) -- against a direct restatement of SB3's loop on a second env."""
    from fake_envs import FakeEnvs
    from f16_jsb_amd.rollout import ACTION_HIGH, ACTION_LOW, collect_rollout
    n, k, T, gamma = 6, 3, 11, 0.9
    env = FakeEnvs(n, k=k, max_steps=4)
    env.reset()
    policy, calls = _linear_policy()
    buf = DeviceRolloutBuffer(T, n, k, "cpu", gamma=gamma)
    last_v, last_d = collect_rollout(env, buf, policy_fn=policy)
    # SB3's loop, restated on numpy (float32), on an identical env
    ref = FakeEnvs(n, k=k, max_steps=4)
    obs = ref.reset().clone()
    starts = np.ones(n, np.float32)
    low, high = np.array(ACTION_LOW, np.float32), np.array(ACTION_HIGH, np.float32)
    boot = 0
    for t in range(T):
        a, v, lp = policy(obs)
        a, v, lp = a.numpy(), v.numpy(), lp.numpy()
        out = ref.step(torch.as_tensor(np.clip(a, low, high)))
        rewards = out.rew.numpy().copy()
        term, trunc = out.terminated.numpy().astype(bool), out.truncated.numpy().astype(bool)
        for idx in range(n):
            if (term[idx] or trunc[idx]) and trunc[idx] and not term[idx]:
                tv = policy(out.terminal_obs[idx][None].clone())[1].numpy()[0]
                rewards[idx] = np.float32(rewards[idx] + np.float32(np.float32(gamma) * tv))
                boot += 1
        np.testing.assert_array_equal(buf.actions[t].numpy(), a, err_msg="unclipped actions @%d" % t)
        np.testing.assert_array_equal(buf.values[t].numpy(), v)
        np.testing.assert_array_equal(buf.log_probs[t].numpy(), lp)
        np.testing.assert_array_equal(buf.rewards[t].numpy(), rewards, err_msg="bootstrapped rewards @%d" % t)
        np.testing.assert_array_equal(buf.episode_starts[t].numpy(), starts)
        np.testing.assert_array_equal(buf.frames[t].numpy(), obs[:, -1].numpy())
        starts = (term | trunc).astype(np.float32)
        obs = out.obs.clone()
    assert boot > 0, "expected truncations inside the rollout"
    np.testing.assert_array_equal(last_d.numpy(), starts)
    np.testing.assert_array_equal(last_v.numpy(), policy(obs)[1].numpy())
    # the env saw the clipped actions: FakeEnvs records a lane's action in its frame [3:7]
    np.testing.assert_array_equal(env.obs.numpy(), obs.numpy())
    assert np.abs(np.concatenate([c[1].numpy() for c in calls])).max() > 1.0  # the clip mattered
