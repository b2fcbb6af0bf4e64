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
