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

from .abi import F16_FLAG_NO_AUTORESET, F16_OBS_DIM, F16_SLOT_CLIP, RolloutSlot

FIELDS = ("frames", "actions", "rewards", "episode_starts", "values", "log_probs", "advantages", "returns")
# device memory the deferred timeout bootstrap may take for its stash of terminal observations
STASH_MAX_BYTES = 1 << 30


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


ACTION_LOW = (-1.0, -1.0, -1.0, 0.0)   # jsbsim_gym.py:143-148 action Box
ACTION_HIGH = (1.0, 1.0, 1.0, 1.0)


def np_clip_actions(a):
    """np.clip(actions, action_space.low, action_space.high) (on_policy_algorithm.py:216) in
    torch with numpy's clip-ufunc semantics: min(max(x, lo), hi), max(a, b) = a if a is NaN or
    a > b else b (so NaN passes and -0 clips to +0 at a 0 bound) -- the in-kernel clip
    (f16env.hip np_clip) computes the same."""
    lo = torch.tensor(ACTION_LOW, dtype=a.dtype, device=a.device)
    hi = torch.tensor(ACTION_HIGH, dtype=a.dtype, device=a.device)
    m = torch.where(torch.isnan(a) | (a > lo), a, lo)
    return torch.where(torch.isnan(m) | (m < hi), m, hi)


def collect_rollout(envs, buf: DeviceRolloutBuffer, seed: int = 0, step0: int = 0, policy_fn=None, value_fn=None,
                    fused: bool = True, persistent: bool = True, bootstrap: str = "deferred"):
    """collect_rollouts (on_policy_algorithm.py:162-268) over device tensors. Starts from the
    envs' current observation; returns (last_values, last_dones) for GAE (:258-262).

    policy_fn(obs) -> (actions, values, log_probs): the policy in the loop (:199-202), called on
    the (N, K, 15) device observation. The env steps np.clip(actions, low, high) (:216; clipped
    in the step kernel), the buffer stores the UNCLIPPED actions with the values and log-probs
    (:247-254); a lane that ended by truncation alone bootstraps rewards += gamma *
    V(terminal_obs) (:236-245, f16env_bootstrap_timeouts: V is evaluated on the whole batch of
    terminal observations, no host sync, only those lanes' rewards change); V = value_fn(obs) ->
    values when given, else policy_fn's values; last_values = V(final obs).
    policy_fn None: the uniform random policy from the device Philox stream (seed, step0 + t),
    values and log-probs zero, no bootstrap.

    fused: each step is ONE launch (f16env_step_rollout / f16env_window_step_rollout) that takes
    (or draws) the actions and writes the slot's actions / rewards / next episode starts and one
    frame of the frame-deduplicated log itself, instead of a sampling launch, the step and six
    buffer copies (RolloutBuffer.add, buffers.py:440-479).
    persistent (no policy_fn): the whole rollout is ONE launch (f16env_rollout_random /
    f16env_window_rollout_random) that keeps every env's state on-chip across the steps:
    bit-identical to the fused launches.
    bootstrap "deferred" (fused path, auto-resetting handles): the terminal observations of the
    lanes that end by truncation alone are appended to a device stash after each step
    (f16env_bootstrap_stash, no host sync) and V runs ONCE over the stash after the loop
    (f16env_bootstrap_apply scatters gamma * V into the rewards) -- the value network does not
    change during a rollout, so this is :236-245's arithmetic with one evaluation instead of one
    per step over the whole batch; "per_step": V over the step's whole batch of terminal
    observations every step (f16env_bootstrap_timeouts). The two agree bit for bit when V's value
    for a row does not depend on the batch it is evaluated in. SB3 itself evaluates each terminal
    observation in a batch of ONE (`predict_values(terminal_obs)[0]` inside its per-env loop,
    :236-245); both modes here evaluate a batch, so for a value head whose GEMMs round a row
    differently at another batch size the bootstrapped rewards may differ from SB3's, and between
    the two modes, in the last bits (tests/test_gpu_policy_rollout.py
    test_bootstrap_modes_vs_batch_of_one bounds it); the lanes that bootstrap are the same."""

    dev = buf.device
    n = buf.n_envs
    T = buf.n_steps
    zeros = torch.zeros(n, dtype=torch.float32, device=dev)
    obs = envs.obs
    starts = getattr(envs, "_last_episode_starts", None)
    if starts is None:
        starts = torch.ones(n, dtype=torch.float32, device=dev)
    buf.reset()
    window = bool(getattr(envs, "window", False))
    vfn = value_fn if value_fn is not None else (lambda o: policy_fn(o)[1])
    use_fused = fused and hasattr(envs, "step_rollout") and buf.actions.data_ptr() % 16 == 0 \
        and (window or (buf.frames[0].data_ptr() % 16 == 0 and (n * F16_OBS_DIM * 4) % 16 == 0))
    use_persistent = use_fused and persistent and policy_fn is None and hasattr(envs, "rollout_random") \
        and not (envs.cfg.flags & F16_FLAG_NO_AUTORESET)
    last_v = zeros
    if use_persistent:
        carry = torch.empty(n, dtype=torch.float32, device=dev)
        buf.obs0.copy_(obs)
        buf.episode_starts[0].copy_(starts)
        envs.rollout_random(seed, step0, T, buf.frames, buf.actions, buf.rewards,
                            buf.episode_starts[1:] if T > 1 else None, carry)
        obs = envs.obs
        buf.pos = T
        starts = carry
    elif use_fused:
        from ._lib import check, lib
        carry = torch.empty(n, dtype=torch.float32, device=dev)
        buf.obs0.copy_(obs)
        buf.episode_starts[0].copy_(starts)
        if window:  # the log's first frame; step t then writes frames[t + 1] (the returned obs's newest)
            buf.frames[0].copy_(obs[:, -1])
        # the slot is built once and its row addresses moved per step (the buffer was allocated
        # with these shapes on this device: no per-step checks on the launch path)
        if getattr(envs, "device", dev) != dev:
            raise ValueError("rollout buffer on %s, envs on %s" % (dev, envs.device))
        raw = hasattr(envs, "_step_rollout_raw")
        slot = RolloutSlot(int(seed) & 0xFFFFFFFFFFFFFFFF, 0, None, None, None, None, None, None,
                           F16_SLOT_CLIP if policy_fn is not None else 0, 0)
        fr0, ac0, rw0, st0 = (buf.frames.data_ptr(), buf.actions.data_ptr(), buf.rewards.data_ptr(),
                              buf.episode_starts.data_ptr())
        fb, ab, rb = n * F16_OBS_DIM * 4, n * 16, n * 4
        L = lib()
        boot = L.f16env_bootstrap_timeouts
        defer = policy_fn is not None and bootstrap == "deferred" \
            and not (int(getattr(envs, "cfg").flags) & F16_FLAG_NO_AUTORESET)
        if bootstrap not in ("deferred", "per_step"):
            raise ValueError("bootstrap must be 'deferred' or 'per_step'")
        # a lane truncates at most once per max_steps steps (auto-reset restarts its counter),
        # so it enters the stash at most (T - 1) // max_steps + 1 times in T steps; a stash that
        # would pass STASH_MAX_BYTES (very short TimeLimits) falls back to the per-step bootstrap
        cap = n * ((T - 1) // max(1, int(envs.cfg.max_steps)) + 1)
        defer = defer and cap * buf.k * F16_OBS_DIM * 4 <= STASH_MAX_BYTES
        if defer:
            stash = torch.empty((cap, buf.k, F16_OBS_DIM), dtype=torch.float32, device=dev)
            stash_idx = torch.empty(cap, dtype=torch.int64, device=dev)
            stash_n = torch.zeros(1, dtype=torch.int32, device=dev)
            stash_fn = L.f16env_bootstrap_stash
        for t in range(T):
            act_ptr = None
            if policy_fn is not None:
                act, v, lp = policy_fn(obs)
                if not (act.dtype == torch.float32 and act.is_contiguous() and act.shape == (n, 4)
                        and act.device == dev and act.data_ptr() % 16 == 0):
                    act = act.reshape(n, 4).to(device=dev, dtype=torch.float32).contiguous()
                    if act.data_ptr() % 16:
                        act = act.clone()
                act_ptr = act.data_ptr()
                buf.values[t].copy_(v.reshape(-1))
                buf.log_probs[t].copy_(lp.reshape(-1))
            if raw:
                slot.act_step = (int(step0) + t) & 0xFFFFFFFFFFFFFFFF
                if window:
                    slot.next_frame = fr0 + (t + 1) * fb if t + 1 < T else None
                else:
                    slot.frame = fr0 + t * fb
                slot.actions, slot.rewards = ac0 + t * ab, rw0 + t * rb
                slot.next_start = st0 + (t + 1) * rb if t + 1 < T else carry.data_ptr()
                out = envs._step_rollout_raw(slot, act_ptr)
            else:
                nxt = buf.episode_starts[t + 1] if t + 1 < T else carry
                frame_kw = ({"next_frame": buf.frames[t + 1] if t + 1 < T else None} if window
                            else {"frame": buf.frames[t]})
                out = envs.step_rollout(seed, step0 + t, actions=buf.actions[t], rewards=buf.rewards[t],
                                        next_start=nxt, policy_actions=act if policy_fn is not None else None,
                                        clip=policy_fn is not None, **frame_kw)
            if defer:  # the truncated lanes' terminal observations into the stash
                tobs = out.terminal_obs
                check(stash_fn(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream), n, buf.k, tobs.data_ptr(),
                               tobs.stride(0), tobs.stride(1), out.terminated.data_ptr(), out.truncated.data_ptr(),
                               t * n, stash.data_ptr(), stash_idx.data_ptr(), stash_n.data_ptr(), cap),
                      "f16env_bootstrap_stash")
            elif policy_fn is not None:  # timeout bootstrap on the step's terminal observations
                tv = vfn(out.terminal_obs).reshape(-1).to(torch.float32).contiguous()
                check(boot(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream), n, rw0 + t * rb,
                           out.terminated.data_ptr(), out.truncated.data_ptr(), tv.data_ptr(), buf.gamma),
                      "f16env_bootstrap_timeouts")
            obs = out.obs
        if defer:  # V once over every stashed terminal observation, then rewards += gamma * V
            m = int(stash_n.item())
            if m > cap:
                raise RuntimeError("bootstrap stash overflow (%d > %d)" % (m, cap))
            if m:
                tv = vfn(stash[:m]).reshape(-1).to(torch.float32).contiguous()
                check(L.f16env_bootstrap_apply(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream), m, rw0,
                                               stash_idx.data_ptr(), tv.data_ptr(), buf.gamma),
                      "f16env_bootstrap_apply")
        buf.pos = T
        starts = carry
    else:
        for t in range(T):
            obs = obs.clone()  # (an env may reuse its observation buffer in the step below)
            if policy_fn is not None:
                act, v, lp = policy_fn(obs)
                act = act.reshape(n, -1).to(torch.float32)
                out = envs.step(np_clip_actions(act).contiguous())
            else:
                act, v, lp = envs.sample_actions(seed, step0 + t), zeros, zeros
                out = envs.step(act)
            rew = out.rew
            if policy_fn is not None:
                rew = bootstrap_timeouts(rew, out.terminated, out.truncated, vfn(out.terminal_obs), buf.gamma)
            buf.add(obs, act, rew, starts, v, lp)
            obs = out.obs
            starts = (out.terminated | out.truncated).to(torch.float32)
    envs._last_episode_starts = starts
    if policy_fn is not None:
        last_v = vfn(obs).reshape(-1).to(torch.float32)
    return last_v, starts


def bootstrap_timeouts(rewards, terminated, truncated, terminal_values, gamma: float):
    """on_policy_algorithm.py:236-245 vectorised: for lanes that ended by truncation only,
    rewards += gamma * V(terminal_observation) (float32 per-op rounding as SB3; the HIP kernel
    f16env_bootstrap_timeouts computes the same in place)."""
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
