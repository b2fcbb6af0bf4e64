"""Host side of the MI355X F-16 environment.

``F16Envs``   -- thin owner of one libf16env handle: device tensors in, device tensors out
                 (the throughput path; no per-step allocation, no host sync).
``F16VecEnv`` -- drop-in for the reference's VecEnv boundary
                 (stable_baselines3/common/vec_env/base_vec_env.py:50-357 VecEnv ABC,
                 dummy_vec_env.py:56-83 auto-reset / info contract, monitor.py:85-111
                 episode stats) over ``F16Envs``, returning numpy like DummyVecEnv.
``reference_goal`` -- jsbsim_gym.py:312-323 with numpy's default_rng(seed), used for
                 seeded resets so seeded goals match the reference bit for bit.
"""
from __future__ import annotations

import ctypes
import time
from collections import namedtuple
from copy import deepcopy
from typing import Any, Optional, Sequence

import numpy as np

from . import spaces
from ._lib import F16EnvError, check, lib
from .abi import (RolloutSlot, F16C_N, F16_IC_N, F16_OBS_DIM, F16_FLAG_GUSTS, F16_FLAG_NAN_GUARD, F16_FLAG_NO_AUTORESET,
                  F16_FLAG_RANDOM_IC,
                  EnvConfig, algorithmic_bytes_per_env_step, config_default)

StepOut = namedtuple("StepOut", "obs rew terminated truncated terminal_obs ep_return ep_len")


def reference_goal(seed) -> np.ndarray:
    """Goal of JSBSimEnv.reset(seed) (jsbsim_gym.py:312-323), float32 (x, y, alt)."""
    rng = np.random.default_rng(seed)
    distance_m = rng.uniform(1000.0, 10000.0)
    bearing_rad = rng.uniform(0, 2 * np.pi)
    altitude_m = rng.uniform(1000.0, 4000.0)
    g = np.zeros(3, dtype=np.float32)
    g[0] = distance_m * np.cos(bearing_rad)
    g[1] = distance_m * np.sin(bearing_rad)
    g[2] = altitude_m
    return g


def _ptr(t) -> Optional[int]:
    return None if t is None else t.data_ptr()


class F16Envs:
    """N F-16 envs on one GPU behind the C ABI. All tensors are torch tensors on ``device``."""

    def __init__(self, n_envs: int, stack_k: int = 10, device=None, seed: int = 0,
                 env_id_base: int = 0, max_steps: int = 1200, down_sample: int = 4,
                 autoreset: bool = True, ic=None, nan_guard: bool = False, **cfg_kw):
        import torch

        if not torch.cuda.is_available():
            raise F16EnvError("F16Envs needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.torch = torch
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise F16EnvError("device must be a cuda (ROCm) device, got %s" % self.device)
        self.n = int(n_envs)
        self.k = int(stack_k)
        flags = int(cfg_kw.pop("flags", 0)) | (0 if autoreset else F16_FLAG_NO_AUTORESET) \
            | (F16_FLAG_NAN_GUARD if nan_guard else 0)
        self.cfg: EnvConfig = config_default(n_envs=n_envs, stack_k=stack_k, seed=seed, env_id_base=env_id_base,
                                             max_steps=max_steps, down_sample=down_sample, flags=flags, ic=ic,
                                             **cfg_kw)
        L = lib()
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(L.f16env_create(ctypes.byref(self.cfg), self.device.index or 0, ctypes.byref(h)), "f16env_create")
        self._h = h
        f32, dev = torch.float32, self.device
        n, k = self.n, self.k
        self._obs = [torch.zeros((n, k, F16_OBS_DIM), dtype=f32, device=dev) for _ in range(2)]
        self._cur = 0
        self.rew = torch.zeros(n, dtype=f32, device=dev)
        self.term = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.trunc = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.terminal_obs = torch.zeros((n, k, F16_OBS_DIM), dtype=f32, device=dev)
        self.ep_return = torch.zeros(n, dtype=torch.float64, device=dev)
        self.ep_len = torch.zeros(n, dtype=torch.int32, device=dev)
        self._act = torch.zeros((n, 4), dtype=f32, device=dev)
        # the handle's own buffers never move: their addresses are taken once, not per step
        self._obs_ptr = [o.data_ptr() for o in self._obs]
        self._out_ptr = (self.rew.data_ptr(), self.term.data_ptr(), self.trunc.data_ptr(),
                         self.terminal_obs.data_ptr(), self.ep_return.data_ptr(), self.ep_len.data_ptr())
        self._step_fn = L.f16env_step

    # --------------------------------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def _stream_int(self) -> int:
        return self.torch.cuda.current_stream(self.device).cuda_stream

    @property
    def obs(self):
        return self._obs[self._cur]

    def close(self):
        if getattr(self, "_h", None):
            lib().f16env_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def waves_per_simd(self) -> int:
        """Occupancy the step kernel variant of this handle is built for (1 or 2)."""
        return int(lib().f16env_step_waves_per_simd(self._h))

    @property
    def step_kernel_name(self) -> str:
        mode = (1 if self.cfg.flags & F16_FLAG_RANDOM_IC else 0) | (2 if self.cfg.flags & F16_FLAG_GUSTS else 0)
        variant = int(lib().f16env_step_variant(self._h))
        if variant == 2:
            return "f16_step_gt_kernel<%d>" % mode
        occ = 2 if variant == 1 else 1
        return "f16_step_kernel" if (mode, occ) == (0, 1) else "f16_step_var_kernel<%d, %d>" % (mode, occ)

    @property
    def state_bytes_per_env(self) -> int:
        return int(lib().f16env_state_bytes_per_env())

    def algorithmic_bytes_per_env_step(self) -> int:
        return algorithmic_bytes_per_env_step(self.k, self.state_bytes_per_env)

    # --------------------------------------------------------------------------------------
    def reset(self, mask=None, goals=None, ic=None):
        """Reset lanes (mask: bool/uint8 (N,) or None=all). goals (N,3) float32 or None
        (device RNG); ic (N, F16_IC_N) float64 or None (config IC). Returns obs (N,K,15)."""
        t = self.torch
        m = None if mask is None else t.as_tensor(mask, device=self.device).to(t.uint8).contiguous()
        g = None if goals is None else t.as_tensor(goals, device=self.device, dtype=t.float32).contiguous()
        c = None if ic is None else t.as_tensor(ic, device=self.device, dtype=t.float64).contiguous()
        if m is not None and tuple(m.shape) != (self.n,):
            raise ValueError("mask must be (N,), got %s" % (tuple(m.shape),))
        if g is not None and tuple(g.shape) != (self.n, 3):
            raise ValueError("goals must be (N, 3)")
        if c is not None and tuple(c.shape) != (self.n, F16_IC_N):
            raise ValueError("ic must be (N, %d)" % F16_IC_N)
        out = self._obs[self._cur]
        check(lib().f16env_reset(self._h, self._stream(), _ptr(m), _ptr(g), _ptr(c), _ptr(out)), "f16env_reset")
        return out

    def _need(self, x, shape, dtype, name):
        """Host-side check of a caller buffer the kernel indexes by env: a wrong shape would be
        an out-of-bounds access on the device, so it is refused before the launch."""
        t = self.torch
        if x is None:
            return
        if not isinstance(x, t.Tensor) or x.device != self.device or x.dtype != dtype or not x.is_contiguous() \
                or tuple(x.shape) != tuple(shape):
            raise ValueError("%s must be a contiguous %s %s tensor on %s" % (name, dtype, tuple(shape), self.device))

    def step(self, actions, done_idx=None, n_done=None, features=None) -> StepOut:
        """One env step for all lanes; ``actions`` (N,4) float32 device tensor (or host
        array, copied). Returns device tensors; obs alternates between two buffers.
        done_idx (N,) / n_done (1,) int32 device tensors receive the compacted list of lanes
        that finished (optional). features: an (N, K, 17) float32 device tensor that receives
        the policy features of the returned obs (features.py:37-67) in the same call."""
        if features is not None:
            return self.step_rollout(0, 0, features=features, policy_actions=actions)
        t = self.torch
        if done_idx is None and n_done is None and isinstance(actions, t.Tensor) and actions.device == self.device \
                and actions.dtype == t.float32 and actions.is_contiguous() and actions.shape == (self.n, 4):
            ap = actions.data_ptr()
            if ap % 16 == 0:  # the common case: one ctypes call on cached addresses
                cur = self._cur
                check(self._step_fn(self._h, self._stream_int(), ap, self._obs_ptr[cur], self._obs_ptr[cur ^ 1],
                                    *self._out_ptr, None, None), "f16env_step")
                self._cur = cur ^ 1
                return StepOut(self._obs[cur ^ 1], self.rew, self.term, self.trunc, self.terminal_obs,
                               self.ep_return, self.ep_len)
        if isinstance(actions, t.Tensor) and actions.device == self.device and actions.dtype == t.float32 \
                and actions.is_contiguous() and actions.data_ptr() % 16 == 0:
            act = actions
        else:
            self._act.copy_(t.as_tensor(actions, dtype=t.float32).reshape(self.n, 4), non_blocking=True)
            act = self._act
        if tuple(act.shape) != (self.n, 4):
            raise ValueError("actions must be (N, 4), got %s" % (tuple(act.shape),))
        if (done_idx is None) != (n_done is None):
            raise ValueError("done_idx and n_done go together")
        self._need(done_idx, (self.n,), t.int32, "done_idx")
        self._need(n_done, (1,), t.int32, "n_done")
        prev = self._obs[self._cur]
        nxt = self._obs[self._cur ^ 1]
        check(lib().f16env_step(self._h, self._stream(), _ptr(act), _ptr(prev), _ptr(nxt), _ptr(self.rew),
                                _ptr(self.term), _ptr(self.trunc), _ptr(self.terminal_obs),
                                _ptr(self.ep_return), _ptr(self.ep_len), _ptr(done_idx), _ptr(n_done)), "f16env_step")
        self._cur ^= 1
        return StepOut(nxt, self.rew, self.term, self.trunc, self.terminal_obs, self.ep_return, self.ep_len)

    def step_rollout(self, seed: int, step: int, frame=None, actions=None, rewards=None, next_start=None,
                     policy_actions=None, features=None) -> StepOut:
        """One env step that also writes one rollout-buffer slot (f16env_step_rollout): the
        newest frame of the observation acted on, the actions, the rewards and the next slot's
        episode starts, with no extra launch. policy_actions None: actions drawn in-kernel
        from the sample_actions(seed, step) stream (bit-identical)."""
        t = self.torch
        act = None
        if policy_actions is not None:
            if isinstance(policy_actions, t.Tensor) and policy_actions.device == self.device \
                    and policy_actions.dtype == t.float32 and policy_actions.is_contiguous() \
                    and policy_actions.data_ptr() % 16 == 0:
                act = policy_actions
            else:
                self._act.copy_(t.as_tensor(policy_actions, dtype=t.float32).reshape(self.n, 4), non_blocking=True)
                act = self._act
            if tuple(act.shape) != (self.n, 4):
                raise ValueError("policy_actions must be (N, 4), got %s" % (tuple(act.shape),))
        self._need(frame, (self.n, F16_OBS_DIM), t.float32, "frame")
        self._need(actions, (self.n, 4), t.float32, "actions")
        self._need(rewards, (self.n,), t.float32, "rewards")
        self._need(next_start, (self.n,), t.float32, "next_start")
        if features is not None and (tuple(features.shape) != (self.n, self.k, 17) or features.dtype != t.float32
                                     or not features.is_contiguous()):
            raise ValueError("features must be a contiguous float32 (N, K, 17) tensor")
        slot = RolloutSlot(int(seed) & 0xFFFFFFFFFFFFFFFF, int(step) & 0xFFFFFFFFFFFFFFFF, _ptr(frame),
                           _ptr(actions), _ptr(rewards), _ptr(next_start), _ptr(features))
        prev = self._obs[self._cur]
        nxt = self._obs[self._cur ^ 1]
        check(lib().f16env_step_rollout(self._h, self._stream(), ctypes.byref(slot), _ptr(act), _ptr(prev), _ptr(nxt),
                                        _ptr(self.rew), _ptr(self.term), _ptr(self.trunc), _ptr(self.terminal_obs),
                                        _ptr(self.ep_return), _ptr(self.ep_len), None, None), "f16env_step_rollout")
        self._cur ^= 1
        return StepOut(nxt, self.rew, self.term, self.trunc, self.terminal_obs, self.ep_return, self.ep_len)

    def rollout_random(self, seed: int, step0: int, n_steps: int, frames, actions, rewards, next_start,
                       last_start) -> None:
        """n_steps env steps in ONE launch under the uniform random policy (f16env_rollout_random:
        actions from the sample_actions(seed, step0 + t) stream, state kept on-chip): writes the
        rollout slots frames (T, N, 15), actions (T, N, 4), rewards (T, N), next_start (T-1, N)
        (episode starts of slots 1..T-1) and last_start (N,), and leaves the env at its
        observation after the last step (self.obs). The same actions and episode starts as n_steps
        step_rollout calls; frames and rewards equal up to fp32 rounding."""
        T = int(n_steps)
        n = self.n
        for name, x, shape in (("frames", frames, (T, n, F16_OBS_DIM)), ("actions", actions, (T, n, 4)),
                               ("rewards", rewards, (T, n)), ("last_start", last_start, (n,))):
            if tuple(x.shape) != shape or x.dtype != self.torch.float32 or not x.is_contiguous():
                raise ValueError("%s must be a contiguous float32 %s tensor" % (name, shape))
        if T > 1 and (next_start is None or tuple(next_start.shape) != (T - 1, n) or not next_start.is_contiguous()):
            raise ValueError("next_start must be a contiguous float32 (T-1, N) tensor")
        prev = self._obs[self._cur]
        nxt = self._obs[self._cur ^ 1]
        check(lib().f16env_rollout_random(self._h, self._stream(), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                          int(step0) & 0xFFFFFFFFFFFFFFFF, T, _ptr(prev), _ptr(nxt), _ptr(frames),
                                          _ptr(actions), _ptr(rewards), _ptr(next_start), _ptr(last_start)),
              "f16env_rollout_random")
        self._cur ^= 1

    def profile_kernel(self, fn, launches: int):
        """Run fn() (which issues `launches` steps) with the step kernel's own dispatch events
        recording each launch; returns (avg_ms, min_ms, launches timed)."""
        L = lib()
        check(L.f16env_profile_begin(self._h, int(launches)), "f16env_profile_begin")
        fn()
        avg, mn, cnt = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        check(L.f16env_profile_end(self._h, ctypes.byref(avg), ctypes.byref(mn), ctypes.byref(cnt)), "f16env_profile_end")
        return avg.value, mn.value, cnt.value

    @property
    def nonfinite_count(self) -> int:
        """Lanes quarantined by the NaN guard (nan_guard=True) since creation; waits for the
        handle's stream. A quarantined lane ended its step terminated (terminated == 3) with
        reward 0 and was reset."""
        c = ctypes.c_uint64()
        check(lib().f16env_nonfinite_count(self._h, self._stream(), ctypes.byref(c)), "f16env_nonfinite_count")
        return int(c.value)

    def get_state(self):
        s = self.torch.zeros((self.n, F16C_N), dtype=self.torch.float64, device=self.device)
        check(lib().f16env_get_state(self._h, self._stream(), _ptr(s)), "f16env_get_state")
        return s

    def set_state(self, canon):
        s = self.torch.as_tensor(canon, dtype=self.torch.float64, device=self.device).contiguous()
        if tuple(s.shape) != (self.n, F16C_N):
            raise ValueError("state must be (N, %d)" % F16C_N)
        check(lib().f16env_set_state(self._h, self._stream(), _ptr(s)), "f16env_set_state")
        self.torch.cuda.current_stream(self.device).synchronize()

    def set_obs(self, obs):
        self._obs[self._cur].copy_(self.torch.as_tensor(obs, dtype=self.torch.float32))

    def trim(self, ic):
        t = self.torch
        c = t.as_tensor(ic, dtype=t.float64, device=self.device).contiguous()
        out = t.zeros_like(c)
        res = t.zeros((self.n, 3), dtype=t.float64, device=self.device)
        check(lib().f16env_trim(self._h, self._stream(), _ptr(c), _ptr(out), _ptr(res)), "f16env_trim")
        return out, res

    def sample_actions(self, seed: int, step: int, out=None):
        if out is None:
            out = self.torch.empty((self.n, 4), dtype=self.torch.float32, device=self.device)
        check(lib().f16env_sample_actions(self._h, self._stream(), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                          int(step) & 0xFFFFFFFFFFFFFFFF, _ptr(out)), "f16env_sample_actions")
        return out


class F16VecEnv:
    """Vectorised drop-in for ``DummyVecEnv([lambda: Monitor(gym.make("JSBSim-v0"))] * N)``.

    Honours the SB3 VecEnv contract (base_vec_env.py:50-357): ``reset() -> obs``,
    ``step_async/step_wait -> (obs, rews, dones, infos)``, auto-reset with
    ``infos[i]["terminal_observation"]`` and ``infos[i]["TimeLimit.truncated"]``
    (dummy_vec_env.py:56-73), Monitor's ``infos[i]["episode"] = {r, l, t}``
    (monitor.py:96-109), ``seed()`` applied at the next reset (:292-309).
    ``return_numpy=False`` keeps everything on the GPU (infos list is then omitted: the
    caller reads ``last_step`` device tensors)."""

    metadata = {"render_modes": []}

    def __init__(self, num_envs: int = 1, stack_k: int = 10, device=None, seed: int = 0,
                 return_numpy: bool = True, env_id_base: int = 0, **kw):
        self.num_envs = int(num_envs)
        self.envs = F16Envs(num_envs, stack_k=stack_k, device=device, seed=seed, env_id_base=env_id_base, **kw)
        self.observation_space = spaces.observation_space(stack_k)
        self.action_space = spaces.action_space()
        self.render_mode = None
        self.return_numpy = bool(return_numpy)
        self.reset_infos: list = [{} for _ in range(self.num_envs)]
        self._seeds: list = [None for _ in range(self.num_envs)]
        self._options: list = [{} for _ in range(self.num_envs)]
        self._actions = None
        self._t_start = time.time()
        self.last_step: Optional[StepOut] = None
        self._attrs: dict = {}

    # -- VecEnv API -------------------------------------------------------------------------
    def reset(self):
        goals = None
        if any(s is not None for s in self._seeds):
            # seeded lanes follow the reference's numpy stream; unseeded lanes use the device RNG
            dev_goals = None
            if not all(s is not None for s in self._seeds):
                self.envs.reset()  # draw device goals for every lane first
                dev_goals = self.envs.get_state()[:, 62:65].float().cpu().numpy()
            goals = np.zeros((self.num_envs, 3), np.float32)
            for i, s in enumerate(self._seeds):
                goals[i] = reference_goal(s) if s is not None else dev_goals[i]
        obs = self.envs.reset(goals=goals)
        self._seeds = [None for _ in range(self.num_envs)]
        self._options = [{} for _ in range(self.num_envs)]
        self.reset_infos = [{} for _ in range(self.num_envs)]
        return obs.cpu().numpy() if self.return_numpy else obs

    def step_async(self, actions) -> None:
        self._actions = actions

    def step_wait(self):
        out = self.envs.step(self._actions)
        self.last_step = out
        if not self.return_numpy:
            dones = (out.terminated | out.truncated).bool()
            return out.obs, out.rew, dones, None
        obs = out.obs.cpu().numpy()
        rew = out.rew.cpu().numpy()
        term_u8 = out.terminated.cpu().numpy()
        term = term_u8.astype(bool)
        trunc = out.truncated.cpu().numpy().astype(bool)
        dones = term | trunc
        infos = [{"TimeLimit.truncated": False} for _ in range(self.num_envs)]
        idx = np.flatnonzero(dones)
        if idx.size:
            tobs = out.terminal_obs[idx].cpu().numpy()
            eret = out.ep_return[idx].cpu().numpy()
            elen = out.ep_len[idx].cpu().numpy()
            t = round(time.time() - self._t_start, 6)
            for j, i in enumerate(idx):
                infos[i]["TimeLimit.truncated"] = bool(trunc[i] and not term[i])
                infos[i]["terminal_observation"] = tobs[j]
                infos[i]["episode"] = {"r": round(float(eret[j]), 6), "l": int(elen[j]), "t": t}
                if term_u8[i] & 2:  # NaN guard quarantine (nan_guard=True)
                    infos[i]["nonfinite"] = True
        return obs, rew, dones, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self) -> None:
        self.envs.close()

    def seed(self, seed: Optional[int] = None) -> Sequence[Optional[int]]:
        if seed is None:
            seed = int(np.random.randint(0, np.iinfo(np.uint32).max, dtype=np.uint32))
        self._seeds = [seed + idx for idx in range(self.num_envs)]
        return self._seeds

    def set_options(self, options=None) -> None:
        if options is None:
            options = {}
        self._options = deepcopy([options] * self.num_envs) if isinstance(options, dict) else deepcopy(options)

    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices

    def get_attr(self, attr_name: str, indices=None) -> list:
        if attr_name in self._attrs:
            v = self._attrs[attr_name]
        elif attr_name in ("render_mode", "observation_space", "action_space", "metadata"):
            v = getattr(self, attr_name)
        elif attr_name == "spec":
            v = None
        else:
            raise AttributeError(attr_name)
        return [v for _ in self._indices(indices)]

    def set_attr(self, attr_name: str, value: Any, indices=None) -> None:
        self._attrs[attr_name] = value

    def env_method(self, method_name: str, *method_args, indices=None, **method_kwargs) -> list:
        raise AttributeError("F16VecEnv lanes expose no per-env methods (%s)" % method_name)

    def env_is_wrapped(self, wrapper_class, indices=None) -> list:
        name = getattr(wrapper_class, "__name__", str(wrapper_class))
        # Monitor / TimeLimit / PositionReward semantics are built into the kernel
        wrapped = name in ("Monitor", "TimeLimit", "PositionReward")
        return [wrapped for _ in self._indices(indices)]

    def has_attr(self, attr_name: str) -> bool:
        try:
            self.get_attr(attr_name)
            return True
        except AttributeError:
            return False

    def get_images(self):
        raise NotImplementedError("rendering is out of scope (SURVEY.md component #9)")

    def render(self, mode: Optional[str] = None):
        return None

    @property
    def unwrapped(self):
        return self


class F16GymVectorEnv:
    """gymnasium.vector.VectorEnv surface over the same kernel (the north star's "Gymnasium
    VectorEnv step()/reset()"), for gymnasium-native learners; duck-typed (gymnasium is not a
    dependency). Autoreset mode SAME_STEP -- what the kernel does: a lane that terminates or
    truncates returns its reset observation in the same step, and

      infos["final_obs"] / infos["_final_obs"]   final (K,15) observation / mask
      infos["episode"] = {"r", "l", "t"}, infos["_episode"]   (RecordEpisodeStatistics keys)

    are filled for the finished lanes (gymnasium's vector-info convention: a value array plus a
    "_key" boolean mask). ``reset(seed=s)`` seeds env i with s + i (the reference's
    default_rng(seed) goal, jsbsim_gym.py:312-323). Single-env semantics are jsbsim_gym.py's
    JSBSimEnv wrapped in TimeLimit(1200) and PositionReward(1e-2) (jsbsim_gym.py:537-545)."""

    metadata = {"autoreset_mode": "SameStep", "render_modes": []}

    def __init__(self, num_envs: int = 1, stack_k: int = 10, device=None, seed: int = 0,
                 return_numpy: bool = True, **kw):
        self.num_envs = int(num_envs)
        self.envs = F16Envs(num_envs, stack_k=stack_k, device=device, seed=seed, **kw)
        self.single_observation_space = spaces.observation_space(stack_k)
        self.single_action_space = spaces.action_space()
        self.observation_space = spaces.batch_space(self.single_observation_space, self.num_envs)
        self.action_space = spaces.batch_space(self.single_action_space, self.num_envs)
        self.render_mode = None
        self.spec = None
        self.closed = False
        self.return_numpy = bool(return_numpy)
        self._t_start = time.time()

    def _out(self, t):
        return t.cpu().numpy() if self.return_numpy else t

    def reset(self, *, seed=None, options=None):
        goals = None
        if seed is not None:
            seeds = [seed + i for i in range(self.num_envs)] if isinstance(seed, int) else list(seed)
            if len(seeds) != self.num_envs:
                raise ValueError("need one seed per env")
            if any(s is None for s in seeds):
                self.envs.reset()
                dev_goals = self.envs.get_state()[:, 62:65].float().cpu().numpy()
            goals = np.stack([reference_goal(s) if s is not None else dev_goals[i] for i, s in enumerate(seeds)])
        obs = self.envs.reset(goals=goals)
        self._t_start = time.time()
        return self._out(obs), {}

    def step(self, actions):
        out = self.envs.step(actions)
        term, trunc = out.terminated.bool(), out.truncated.bool()
        done = term | trunc
        infos = {}
        if bool(done.any()):
            t = round(time.time() - self._t_start, 6)
            mask = done.cpu().numpy()
            infos["final_obs"] = self._out(out.terminal_obs.clone())
            infos["_final_obs"] = mask
            eret = out.ep_return.cpu().numpy()
            elen = out.ep_len.cpu().numpy()
            infos["episode"] = {"r": np.where(mask, np.round(eret, 6), 0.0), "l": np.where(mask, elen, 0),
                                "t": np.where(mask, t, 0.0)}
            infos["_episode"] = mask
        return self._out(out.obs), self._out(out.rew), self._out(term), self._out(trunc), infos

    def close(self, **kwargs):
        if not self.closed:
            self.envs.close()
            self.closed = True

    def render(self):
        return None

    @property
    def unwrapped(self):
        return self
