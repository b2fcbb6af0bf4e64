"""Device-resident PPO rollout storage, GAE and the rank-0 gather (BASELINE cfg 4).

The caller side of the hot path: SB3's `collect_rollouts`
(on_policy_algorithm.py:162-268) fills a numpy `RolloutBuffer` (buffers.py:343-522) one env at
a time. Here the buffer lives in HBM as [n_steps][n_envs] tensors, GAE runs as the HIP kernel
`f16env_gae` (bit-exact with buffers.py:403-438's float32 numpy recurrence), and after a
rollout every rank's shard lands on rank 0 with RCCL gathers over xGMI
(`torch.distributed` backend "nccl" is RCCL on ROCm).

Frame dedup: a stacked observation is K overlapping frames, so the buffer keeps
only the newest frame per step plus the stack before step 0, and rebuilds any step's stack
from those and `episode_starts` (a reset observation is K copies of its first frame). That
cuts the gathered observation bytes by K.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import torch

from .abi import F16_FLAG_GUSTS, F16_FLAG_NO_AUTORESET, F16_FLAG_RANDOM_IC, F16_OBS_DIM

FIELDS = ("frames", "actions", "rewards", "episode_starts", "values", "log_probs", "advantages", "returns")


class DeviceRolloutBuffer:
    def __init__(self, n_steps: int, n_envs: int, stack_k: int, device, gamma: float = 0.99,
                 gae_lambda: float = 0.95, act_dim: int = 4):
        self.n_steps, self.n_envs, self.k = int(n_steps), int(n_envs), int(stack_k)
        self.gamma, self.gae_lambda = float(gamma), float(gae_lambda)
        self.device = torch.device(device)
        f32 = torch.float32
        z = lambda *s: torch.zeros(*s, dtype=f32, device=self.device)  # noqa: E731
        self.frames = z(self.n_steps, self.n_envs, F16_OBS_DIM)       # newest frame of obs[t]
        self.obs0 = z(self.n_envs, self.k, F16_OBS_DIM)                # full stack of obs[0]
        self.actions = z(self.n_steps, self.n_envs, act_dim)
        self.rewards = z(self.n_steps, self.n_envs)
        self.episode_starts = z(self.n_steps, self.n_envs)
        self.values = z(self.n_steps, self.n_envs)
        self.log_probs = z(self.n_steps, self.n_envs)
        self.advantages = z(self.n_steps, self.n_envs)
        self.returns = z(self.n_steps, self.n_envs)
        self.pos = 0

    def reset(self):
        self.pos = 0

    @property
    def full(self) -> bool:
        return self.pos == self.n_steps

    def add(self, obs, action, reward, episode_start, value, log_prob):
        """RolloutBuffer.add (buffers.py:440-479) with device tensors; obs is (N, K, 15)."""
        if self.pos >= self.n_steps:
            raise RuntimeError("rollout buffer is full")
        t = self.pos
        if t == 0:
            self.obs0.copy_(obs)
        self.frames[t].copy_(obs[:, -1])
        self.actions[t].copy_(action.reshape(self.n_envs, -1))
        self.rewards[t].copy_(reward.reshape(-1))
        self.episode_starts[t].copy_(episode_start.reshape(-1).to(torch.float32))
        self.values[t].copy_(value.reshape(-1))
        self.log_probs[t].copy_(log_prob.reshape(-1))
        self.pos += 1

    def compute_returns_and_advantage(self, last_values, dones, stream=None):
        """buffers.py:403-438 on the GPU (HIP kernel f16env_gae)."""
        from ._lib import check, lib

        if self.device.type != "cuda":
            raise RuntimeError("GAE runs on the GPU (f16env_gae); buffer is on %s" % self.device)
        lv = torch.as_tensor(last_values).reshape(-1).to(self.device, torch.float32).contiguous()
        dn = torch.as_tensor(dones).reshape(-1).to(self.device, torch.uint8).contiguous()
        if lv.numel() != self.n_envs or dn.numel() != self.n_envs:  # the kernel reads n_envs of each
            raise ValueError("last_values and dones must hold n_envs = %d entries, got %d and %d"
                             % (self.n_envs, lv.numel(), dn.numel()))
        s = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        check(lib().f16env_gae(ctypes.c_void_p(s), self.n_steps, self.n_envs, self.rewards.data_ptr(),
                               self.values.data_ptr(), self.episode_starts.data_ptr(), lv.data_ptr(),
                               dn.data_ptr(), self.gamma, self.gae_lambda, self.advantages.data_ptr(),
                               self.returns.data_ptr()), "f16env_gae")

    # ----------------------------------------------------------------------------------------
    def observations(self, steps=None):
        return rebuild_observations(self.frames, self.obs0, self.episode_starts, self.k, steps)

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {f: getattr(self, f) for f in FIELDS} | {"obs0": self.obs0}


def collect_rollout(envs, buf: DeviceRolloutBuffer, seed: int, step0: int = 0, values_fn=None, fused: bool = True,
                    persistent: bool = True):
    """collect_rollouts (on_policy_algorithm.py:162-268) over device tensors with random
    policy actions from the device Philox stream (the policy network is out of scope; values
    and log-probs are zeros unless ``values_fn(obs) -> (values, log_probs)`` is given).
    Starts from envs' current observation; returns (last_values, last_dones) for GAE.

    fused: each step is ONE launch (f16env_step_rollout) that draws the actions in-kernel and
    writes the slot's frame / actions / rewards / next episode starts itself, instead of a
    sampling launch, the step and six buffer copies (RolloutBuffer.add, buffers.py:440-479).
    persistent (with no values_fn, the reference task and K <= 8): the whole rollout is ONE
    launch (f16env_rollout_random) that keeps every env's state on-chip across the steps: the
    same actions and episode starts, frames / rewards equal up to fp32 rounding."""
    dev = buf.device
    n = buf.n_envs
    zeros = torch.zeros(n, dtype=torch.float32, device=dev)
    obs = envs.obs
    starts = getattr(envs, "_last_episode_starts", None)
    if starts is None:
        starts = torch.ones(n, dtype=torch.float32, device=dev)
    buf.reset()
    use_fused = fused and hasattr(envs, "step_rollout") and buf.frames[0].data_ptr() % 16 == 0 \
        and (n * F16_OBS_DIM * 4) % 16 == 0
    use_persistent = (use_fused and persistent and values_fn is None and hasattr(envs, "rollout_random")
                      and envs.k <= 8 and not (envs.cfg.flags & (F16_FLAG_NO_AUTORESET | F16_FLAG_RANDOM_IC | F16_FLAG_GUSTS))
                      and buf.actions.data_ptr() % 16 == 0)
    if use_persistent:
        carry = torch.empty(n, dtype=torch.float32, device=dev)
        buf.obs0.copy_(obs)
        buf.episode_starts[0].copy_(starts)
        T = buf.n_steps
        envs.rollout_random(seed, step0, T, buf.frames, buf.actions, buf.rewards,
                            buf.episode_starts[1:] if T > 1 else None, carry)
        obs = envs.obs
        buf.pos = T
        starts = carry
    elif use_fused:
        carry = torch.empty(n, dtype=torch.float32, device=dev)
        buf.obs0.copy_(obs)
        buf.episode_starts[0].copy_(starts)
        T = buf.n_steps
        for t in range(T):
            if values_fn is not None:
                v, lp = values_fn(obs)
                buf.values[t].copy_(v.reshape(-1))
                buf.log_probs[t].copy_(lp.reshape(-1))
            nxt = buf.episode_starts[t + 1] if t + 1 < T else carry
            out = envs.step_rollout(seed, step0 + t, frame=buf.frames[t], actions=buf.actions[t],
                                    rewards=buf.rewards[t], next_start=nxt)
            if values_fn is not None:
                tv, _ = values_fn(out.terminal_obs)
                buf.rewards[t].copy_(bootstrap_timeouts(buf.rewards[t], out.terminated, out.truncated, tv, buf.gamma))
            obs = out.obs
        buf.pos = T
        starts = carry
    else:
        for t in range(buf.n_steps):
            act = envs.sample_actions(seed, step0 + t)
            v, lp = values_fn(obs) if values_fn is not None else (zeros, zeros)
            out = envs.step(act)
            rew = out.rew
            if values_fn is not None:
                tv, _ = values_fn(out.terminal_obs)
                rew = bootstrap_timeouts(rew, out.terminated, out.truncated, tv, buf.gamma)
            buf.add(obs, act, rew, starts, v, lp)
            obs = out.obs
            starts = (out.terminated | out.truncated).to(torch.float32)
    envs._last_episode_starts = starts
    last_v = values_fn(obs)[0] if values_fn is not None else zeros
    return last_v, starts


def bootstrap_timeouts(rewards, terminated, truncated, terminal_values, gamma: float):
    """on_policy_algorithm.py:236-245 vectorised: for lanes that ended by truncation only,
    rewards += gamma * V(terminal_observation) (float32 per-op rounding as SB3)."""
    mask = truncated.bool() & ~terminated.bool()
    g = torch.tensor(gamma, dtype=torch.float32, device=rewards.device)
    add = g * terminal_values.reshape(-1).to(torch.float32)
    return torch.where(mask, rewards + add, rewards)


def rebuild_observations(frames, obs0, episode_starts, k: int, steps=None):
    """Stacked observations (T, N, K, 15) from newest frames, the initial stack and
    episode starts: obs[t][j] = frame[max(t - (K-1) + j, s_t)] where s_t is the last episode
    start <= t; indices before step 0 come from the initial stack (oldest first)."""
    T, N, D = frames.shape
    dev = frames.device
    tt = torch.arange(T, device=dev)
    if steps is None:
        steps = tt
    steps = torch.as_tensor(steps, device=dev)
    # last episode start at or before t, per env (-inf if none)
    marks = torch.where(episode_starts.bool(), tt[:, None].expand(T, N), torch.full((T, N), -(1 << 30), device=dev))
    last_start = torch.cummax(marks, dim=0).values                      # (T, N)
    j = torch.arange(k, device=dev)
    src = steps[:, None] - (k - 1) + j[None, :]                          # (S, K)
    ls = last_start[steps]                                               # (S, N)
    idx = torch.maximum(src[:, None, :], ls[:, :, None])                # (S, N, K)
    from_frames = idx >= 0
    fi = idx.clamp(min=0)
    e = torch.arange(N, device=dev)[None, :, None].expand_as(fi)
    out_f = frames[fi, e]                                                # (S, N, K, D)
    oi = (idx + (k - 1)).clamp(0, k - 1)                                 # position in obs0
    out_0 = obs0[e, oi]                                                  # (S, N, K, D)
    return torch.where(from_frames[..., None], out_f, out_0)


def gather_to_rank0(buf: DeviceRolloutBuffer, group=None, chunk_steps: Optional[int] = None,
                    fields=FIELDS) -> Optional[Dict[str, torch.Tensor]]:
    """Gather every rank's rollout shard to rank 0 (RCCL over xGMI on MI355X, gloo in CPU
    tests). Returns on rank 0 a dict of RANK-MAJOR tensors (world, n_steps, n_envs, ...) -- rank
    r's shard at [r], i.e. global envs [r * n_envs, (r + 1) * n_envs) as env_id_base assigns them
    -- plus 'obs0' (world, n_envs, K, 15); None on other ranks. ``env_major`` turns a field into
    the (n_steps, world * n_envs, ...) layout of a single-GPU buffer.

    The output is allocated once and every collective writes straight into it: chunk [t0, t1)
    of rank r lands in the contiguous view out[r, t0:t1], so rank 0 moves each byte once (no
    per-chunk temporaries, no strided re-copy). Gathers are chunked over steps (chunk_steps) to
    bound each collective's size; a short last chunk is fine."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    T = buf.n_steps
    chunk = T if not chunk_steps else max(1, int(chunk_steps))
    out = {}
    for f in tuple(fields) + ("obs0",):
        x = getattr(buf, f)
        if not x.is_contiguous():
            x = x.contiguous()
        res = torch.empty((world,) + tuple(x.shape), dtype=x.dtype, device=x.device) if rank == 0 else None
        if f == "obs0":
            dist.gather(x, list(res.unbind(0)) if rank == 0 else None, dst=0, group=group)
        else:
            for t0 in range(0, T, chunk):
                t1 = min(T, t0 + chunk)
                dist.gather(x[t0:t1], [res[r, t0:t1] for r in range(world)] if rank == 0 else None, dst=0, group=group)
        if rank == 0:
            out[f] = res
    return out if rank == 0 else None


def env_major(x: torch.Tensor) -> torch.Tensor:
    """(world, T, N, ...) rank-major gather output -> (T, world * N, ...) (a copy)."""
    w, T, N = x.shape[:3]
    return x.transpose(0, 1).reshape((T, w * N) + tuple(x.shape[3:]))
