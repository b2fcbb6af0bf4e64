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
                  F16_FLAG_OBS_CHECK, F16_SLOT_CLIP, F16_SLOT_FEATURE_WINDOW, F16_STEP_FEATURE_WINDOW,
                  F16_STEP_POSES, F16_FLAG_RANDOM_IC,
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


def _default_history(k: int) -> int:
    """Default window history T (positions per history): max(256, 2K) -- a restart (K-1
    positions moved to the front) every T-K+1 steps; 2 x 256 x 64 B = 32 KiB per env."""
    return max(256, 2 * k)


class F16Envs:
    """N F-16 envs on one GPU behind the C ABI. All tensors are torch tensors on ``device``."""

    def __init__(self, n_envs: int, stack_k: int = 10, device=None, seed: int = 0,
                 env_id_base: int = 0, max_steps: int = 1200, down_sample: int = 4,
                 autoreset: bool = True, ic=None, nan_guard: bool = False, obs_check: bool = False,
                 obs_layout: str = "contiguous",
                 history: int = 0, window_order: str = "position", fused_features: bool = False,
                 fused_poses: bool = False, **cfg_kw):
        """obs_layout "contiguous": observations in two ping-pong (N, K, 15) buffers (f16env_step).
        obs_layout "window": observations are (N, K, 15) views of two per-env frame histories of
        `history` positions of 64-B frame slots, position-major [T][N][16] (f16env_step_window:
        only the new frame is written per step, one contiguous block per position; view strides
        (16, N*16, 1)); history 0 = max(256, 2K) (a restart every T-K+1 steps); window_order
        "env" keeps the histories env-major [N][T][16] instead (strides (T*16, 16, 1)). Both
        layouts give identical values and the same validity (an observation stays valid until
        the step after next). A consumer that needs a flat (N, K*15) array copies the window
        (reshape); the features kernel (f16_jsb_amd.features) reads it in place.
        fused_features (windowed layout): every step also keeps the policy features of both
        windows (obs_features(), features.py:37-67 per frame) in its own epilogue -- the step's
        feature-window build (f16env_window_step_ex, F16_STEP_FEATURE_WINDOW), no second launch;
        obs_features() is then a view. Off by default: the plain step's instance carries none of
        that code.
        fused_poses (windowed layout): every step also writes the render/telemetry pose of the
        returned observation's newest frame (poses(), telemetry.poses of obs[:, -1], the same
        bits) in its epilogue (f16env_window_step_ex, F16_STEP_POSES): no second launch."""
        import torch

        if not torch.cuda.is_available():
            raise F16EnvError("F16Envs needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.torch = torch
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise F16EnvError("device must be a cuda (ROCm) device, got %s" % self.device)
        self.n = int(n_envs)
        self.k = int(stack_k)
        self._dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        self._raw_stream = raw if raw is not None else (lambda i: torch.cuda.current_stream(i).cuda_stream)
        flags = int(cfg_kw.pop("flags", 0)) | (0 if autoreset else F16_FLAG_NO_AUTORESET) \
            | (F16_FLAG_NAN_GUARD if nan_guard else 0) | (F16_FLAG_OBS_CHECK if obs_check else 0)
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
        if obs_layout not in ("contiguous", "window"):
            raise ValueError("obs_layout must be 'contiguous' or 'window'")
        self.window = obs_layout == "window"
        if self.window:
            T = int(history) if history else _default_history(k)
            if T < 2 * k:
                raise ValueError("history must be >= 2 * stack_k")
            self.T = T
            if window_order not in ("position", "env"):
                raise ValueError("window_order must be 'position' or 'env'")
            self._env_major = window_order == "env"
            check(L.f16env_set_window_order(h, 1 if self._env_major else 0), "f16env_set_window_order")
            # [parity][position][env][16] (64-B frame slots, position-major) or [parity][env][position][16]
            self._hist = torch.zeros((2, n, T, 16) if self._env_major else (2, T, n, 16), dtype=f32, device=dev)
            self._hist_ptr = (self._hist[0].data_ptr(), self._hist[1].data_ptr())
            self._views = [[None] * T for _ in range(2)]
            self._p = k - 1   # newest frame position of the current observation's window
            self._obs = None
            # feature window (obs_features): feature histories beside the frame histories, made
            # at the first call; op counters tell whether they describe the current windows
            self._fh = None
            self._op = 0          # ops that changed the windows (steps, resets, state / obs writes)
            self._step_op = -1    # the last op that was a step
            self._feat_op = -1    # the op the feature windows describe
            self._feat_prev_ok = False  # the feature windows hold the last step's ahead fills
            self.feature_window_calls = {"incremental": 0, "full": 0, "fused": 0}
        else:
            if fused_features or fused_poses:
                raise ValueError("fused_features / fused_poses need obs_layout='window'")
            self._obs = [torch.zeros((n, k, F16_OBS_DIM), dtype=f32, device=dev) for _ in range(2)]
        self.fused_features = bool(fused_features)
        self.fused_poses = bool(fused_poses)
        self._poses = None    # (N, 10) pose export; _poses_op: the op it describes
        self._poses_op = -1
        self._cur = 0
        # rewards (f32), terminated, truncated (u8) in ONE allocation, so a host-side consumer
        # (F16VecEnv's numpy mode) moves the three with a single device-to-host copy
        nb = (4 * n + 2 * n + 15) // 16 * 16
        self.step_flags = torch.zeros(nb, dtype=torch.uint8, device=dev)
        self.rew = self.step_flags[:4 * n].view(f32)
        self.term = self.step_flags[4 * n:5 * n]
        self.trunc = self.step_flags[5 * n:6 * n]
        # window layout: terminal_obs is re-pointed at the other history's window every step
        self.terminal_obs = None if self.window else torch.zeros((n, k, F16_OBS_DIM), dtype=f32, device=dev)
        self.ep_return = torch.zeros(n, dtype=torch.float64, device=dev)
        self.ep_len = torch.zeros(n, dtype=torch.int32, device=dev)
        self._act = torch.zeros((n, 4), dtype=f32, device=dev)
        # the handle's own buffers never move: their addresses are taken once, not per step
        if self.window:
            self._win_ptr = (self.rew.data_ptr(), self.term.data_ptr(), self.trunc.data_ptr(),
                             self.ep_return.data_ptr(), self.ep_len.data_ptr())
            self._step_win_fn = L.f16env_step_window
            check(L.f16env_window_bind(self._h, self._hist_ptr[0], self._hist_ptr[1], self.T, *self._win_ptr),
                  "f16env_window_bind")
            self._step_bound = L.f16env_window_step_bound
            self._step_ex = L.f16env_window_step_ex
            self.terminal_obs = self._window(1)
            if (self.fused_features or self.fused_poses) and L.f16env_window_resets_deferred(h):
                # the deferred-reset step (cfg5 with F16ENV_ICC_PERIOD=0): the epilogue extras
                # would describe the pre-reset window, and f16env_window_step_ex refuses them --
                # refused here instead of at the first step
                self.close()
                raise ValueError("fused_features / fused_poses are not available with the deferred-reset "
                                 "windowed step (cfg5 with F16ENV_ICC_PERIOD=0)")
            if self.fused_features:
                self._feature_hist()
            if self.fused_poses:
                self._poses = torch.zeros((n, 10), dtype=f32, device=dev)
                check(L.f16env_window_poses_bind(self._h, self._poses.data_ptr()), "f16env_window_poses_bind")
        else:
            self._obs_ptr = [o.data_ptr() for o in self._obs]
            self._out_ptr = (self.rew.data_ptr(), self.term.data_ptr(), self.trunc.data_ptr(),
                             self.terminal_obs.data_ptr(), self.ep_return.data_ptr(), self.ep_len.data_ptr())
        self._step_fn = L.f16env_step

    # --------------------------------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(self._stream_int())

    def _stream_int(self) -> int:
        """The caller's current stream on this device (the raw handle: 0.03 us, where
        torch.cuda.current_stream() builds a Stream object per call, ~1.7 us)."""
        return self._raw_stream(self._dev_index)

    def _window(self, other: int = 0):
        """(N, K, 15) view of the current (other=0) or other-parity history's window (views are
        made once per (parity, position) and reused: a step's host cost stays one ctypes call)."""
        b, p = self._cur ^ other, self._p
        v = self._views[b][p]
        if v is None:
            v = self._views[b][p] = self._make_window(b, p)
        return v

    def _make_window(self, b: int, p: int):
        if self._env_major:
            return self._hist[b, :, p - self.k + 1:p + 1, :F16_OBS_DIM]
        return self._hist[b, p - self.k + 1:p + 1, :, :F16_OBS_DIM].transpose(0, 1)

    @property
    def obs(self):
        return self._window() if self.window else self._obs[self._cur]

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
        if self.window:
            return int(lib().f16env_step_window_waves_per_simd(self._h))
        return int(lib().f16env_step_waves_per_simd(self._h))

    @property
    def step_kernel_name(self) -> str:
        """The step kernel instance this handle launches (the symbol rocprofv3 reports)."""
        return lib().f16env_step_kernel_name(self._h).decode()

    @property
    def state_bytes_per_env(self) -> int:
        return int(lib().f16env_state_bytes_per_env())

    def algorithmic_bytes_per_env_step(self) -> int:
        """Bytes per env step of this handle's layout (abi.algorithmic_bytes_per_env_step)."""
        return algorithmic_bytes_per_env_step(self.k, self.state_bytes_per_env,
                                              "window" if self.window else "contiguous")

    def stack_bytes_per_env_step(self) -> int:
        """SURVEY.md 8(d)'s B(K): the bytes of the same step with the stack materialised."""
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
        if self.window:
            check(lib().f16env_reset_window(self._h, self._stream(), _ptr(m), _ptr(g), _ptr(c),
                                            self._hist_ptr[self._cur], self.T, self._p), "f16env_reset_window")
            self._op += 1
            return self._window()
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

    def step(self, actions, done_idx=None, n_done=None, features=None, seed=None, step=None) -> StepOut:
        """One env step for all lanes; ``actions`` (N,4) float32 device tensor (or host
        array, copied). Returns device tensors; obs alternates between two buffers.
        done_idx (N,) / n_done (1,) int32 device tensors receive the compacted list of lanes
        that finished (optional). features: an (N, K, 17) float32 device tensor that receives
        the policy features of the returned obs (features.py:37-67) in the same call.
        actions None with seed / step: the actions are drawn inside the step kernel from the
        sample_actions(seed, step) stream (bit-identical to step(sample_actions(seed, step)),
        without the sampling launch and the action read; windowed layout: f16env_window_step_ex,
        contiguous: the rollout-slot step with an empty slot)."""
        if actions is None:
            if seed is None or step is None:
                raise ValueError("actions=None needs seed and step (the in-kernel sample_actions stream)")
            if done_idx is not None or n_done is not None or features is not None:
                raise ValueError("in-kernel actions: no done list / features argument")
            if self.window:
                return self._step_window_ex(None, int(seed), int(step))
            return self.step_rollout(seed, step)
        if features is not None:
            return self.step_rollout(0, 0, features=features, policy_actions=actions)
        if self.window:
            if (self.fused_features or self.fused_poses) and done_idx is None and n_done is None:
                return self._step_window_ex(self._as_act(actions), 0, 0)
            return self._step_window(actions, done_idx, n_done)
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

    def _as_act(self, actions):
        """actions as an aligned contiguous (N, 4) float32 tensor on the device (copied if not)."""
        t = self.torch
        if isinstance(actions, t.Tensor) and actions.device == self.device and actions.dtype == t.float32 \
                and actions.is_contiguous() and actions.data_ptr() % 16 == 0:
            act = actions
        else:
            self._act.copy_(t.as_tensor(actions, dtype=t.float32).reshape(self.n, 4), non_blocking=True)
            act = self._act
        if act.shape != (self.n, 4):
            raise ValueError("actions must be (N, 4), got %s" % (tuple(act.shape),))
        return act

    def _step_window_ex(self, act, seed: int, step: int) -> StepOut:
        """f16env_window_step_ex: act None draws the actions in the kernel (sample_actions(seed,
        step)); a fused_features handle also keeps its feature windows in the step's epilogue
        whenever they are current before it, and catches them up after a step that could not."""
        fw = self.fused_features and self._fh is not None and self._feat_prev_ok and self._feat_op == self._op
        s, cur, p = self._advance()
        flags = (F16_STEP_FEATURE_WINDOW if fw else 0) | (F16_STEP_POSES if self.fused_poses else 0)
        check(self._step_ex(self._h, s, None if act is None else act.data_ptr(), cur, p,
                            flags, seed & 0xFFFFFFFFFFFFFFFF, step & 0xFFFFFFFFFFFFFFFF), "f16env_window_step_ex")
        out = self._fused_done(fw, self._advanced(cur, p))
        if self.fused_poses:
            self._poses_op = self._op
        if self.fused_features and not fw:
            self.obs_features()  # whole windows + the step's ahead fills: the next step fuses
        return out

    def _step_window(self, actions, done_idx, n_done) -> StepOut:
        """f16env_step_window: the new frame goes to position p+1 of both histories, the
        observation is the window ending there in the history of the new parity."""
        t = self.torch
        act = self._as_act(actions)
        if done_idx is not None or n_done is not None:
            if (done_idx is None) != (n_done is None):
                raise ValueError("done_idx and n_done go together")
            self._need(done_idx, (self.n,), t.int32, "done_idx")
            self._need(n_done, (1,), t.int32, "n_done")
        s, cur, p = self._advance()
        if done_idx is None:  # the common case: five arguments, the rest bound at creation
            check(self._step_bound(self._h, s, act.data_ptr(), cur, p), "f16env_window_step_bound")
        else:
            check(self._step_win_fn(self._h, s, act.data_ptr(), self._hist_ptr[cur], self._hist_ptr[cur ^ 1], self.T,
                                    p, *self._win_ptr, _ptr(done_idx), _ptr(n_done)), "f16env_step_window")
        return self._advanced(cur, p)

    def _advance(self):
        """(stream, parity, position) of the next windowed step: the new frame goes to position
        p+1 of both histories (after a restart when p+1 reaches T)."""
        s = self._stream_int()
        p = self._p + 1
        if p >= self.T:  # move the last K-1 frames to the front of both histories
            check(lib().f16env_window_restart(self._h, s, self._hist_ptr[0], self._hist_ptr[1], self.T, self._p),
                  "f16env_window_restart")
            if self._fh is not None and self._feat_op == self._op:  # the feature windows move along
                k = self.k   # (K-1 whole rows: one contiguous device-to-device copy per parity)
                for b in (0, 1):
                    self._fh[b, :k - 1].copy_(self._fh[b, self._p - k + 2:self._p + 1])
            p = self.k - 1
        return s, self._cur ^ 1, p

    def _advanced(self, cur, p) -> StepOut:
        self._cur, self._p = cur, p
        self._op += 1
        self._step_op = self._op
        self.terminal_obs = self._window(1)
        return StepOut(self._window(), self.rew, self.term, self.trunc, self.terminal_obs, self.ep_return,
                       self.ep_len)

    def step_rollout(self, seed: int, step: int, frame=None, actions=None, rewards=None, next_start=None,
                     policy_actions=None, features=None, next_frame=None, clip: bool = False) -> StepOut:
        """One env step that also writes one rollout-buffer slot, with no extra launch
        (f16env_step_rollout / f16env_window_step_rollout): the actions, the rewards and the next
        slot's episode starts, and one frame of the frame-deduplicated log -- the contiguous
        layout writes `frame` (the newest frame of the observation acted on), the windowed layout
        `next_frame` (the newest frame of the returned observation, i.e. the next slot's frame).
        policy_actions None: actions drawn in-kernel from the sample_actions(seed, step) stream
        (bit-identical). clip: the env steps np.clip(policy_actions, low, high) over the action
        Box (on_policy_algorithm.py:216) while `actions` receives policy_actions unclipped
        (:247-254)."""
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
        if self.window and frame is not None:
            raise ValueError("the windowed layout writes next_frame (the returned observation's newest frame), not frame")
        if not self.window and next_frame is not None:
            raise ValueError("the contiguous layout writes frame (the acted-on observation's newest frame), not next_frame")
        self._need(frame, (self.n, F16_OBS_DIM), t.float32, "frame")
        self._need(next_frame, (self.n, F16_OBS_DIM), t.float32, "next_frame")
        self._need(actions, (self.n, 4), t.float32, "actions")
        self._need(rewards, (self.n,), t.float32, "rewards")
        self._need(next_start, (self.n,), t.float32, "next_start")
        if features is not None and (tuple(features.shape) != (self.n, self.k, 17) or features.dtype != t.float32
                                     or not features.is_contiguous()):
            raise ValueError("features must be a contiguous float32 (N, K, 17) tensor")
        slot = RolloutSlot(int(seed) & 0xFFFFFFFFFFFFFFFF, int(step) & 0xFFFFFFFFFFFFFFFF, _ptr(frame),
                           _ptr(actions), _ptr(rewards), _ptr(next_start), _ptr(features), _ptr(next_frame),
                           F16_SLOT_CLIP if clip else 0, 0)
        if self.window:
            fw = self._fused_features(slot)
            s, cur, p = self._advance()
            check(lib().f16env_window_step_rollout(self._h, s, ctypes.byref(slot), _ptr(act), cur, p),
                  "f16env_window_step_rollout")
            return self._fused_done(fw, self._advanced(cur, p))
        prev = self._obs[self._cur]
        nxt = self._obs[self._cur ^ 1]
        check(lib().f16env_step_rollout(self._h, self._stream(), ctypes.byref(slot), _ptr(act), _ptr(prev), _ptr(nxt),
                                        _ptr(self.rew), _ptr(self.term), _ptr(self.trunc), _ptr(self.terminal_obs),
                                        _ptr(self.ep_return), _ptr(self.ep_len), None, None), "f16env_step_rollout")
        self._cur ^= 1
        return StepOut(nxt, self.rew, self.term, self.trunc, self.terminal_obs, self.ep_return, self.ep_len)

    def _step_rollout_raw(self, slot, act_ptr) -> StepOut:
        """step_rollout with a prepared RolloutSlot and action address and no argument checks:
        collect_rollout validates its buffers once per rollout and moves the slot's row
        addresses itself (the per-step host cost is then the launch, not the checks)."""
        if self.window:
            fw = self._fused_features(slot)
            s, cur, p = self._advance()
            check(lib().f16env_window_step_rollout(self._h, s, ctypes.byref(slot), act_ptr, cur, p),
                  "f16env_window_step_rollout")
            return self._fused_done(fw, self._advanced(cur, p))
        cur = self._cur
        nxt = self._obs[cur ^ 1]
        check(lib().f16env_step_rollout(self._h, self._stream_int(), ctypes.byref(slot), act_ptr, self._obs_ptr[cur],
                                        self._obs_ptr[cur ^ 1], *self._out_ptr, None, None), "f16env_step_rollout")
        self._cur = cur ^ 1
        return StepOut(nxt, self.rew, self.term, self.trunc, self.terminal_obs, self.ep_return, self.ep_len)

    def _fused_features(self, slot) -> bool:
        """Whether this rollout-slot step keeps the feature window itself (F16_SLOT_FEATURE_WINDOW:
        the windows are current, so the step's epilogue brings them to its new position)."""
        fw = self._fh is not None and self._feat_prev_ok and self._feat_op == self._op
        slot.flags = (slot.flags | F16_SLOT_FEATURE_WINDOW) if fw else (slot.flags & ~F16_SLOT_FEATURE_WINDOW)
        return fw

    def _fused_done(self, fw: bool, out: StepOut) -> StepOut:
        if fw:
            self._feat_op = self._op
            self.feature_window_calls["fused"] += 1
        return out

    def rollout_random(self, seed: int, step0: int, n_steps: int, frames, actions, rewards, next_start,
                       last_start) -> None:
        """n_steps env steps in ONE launch under the uniform random policy (f16env_rollout_random /
        f16env_window_rollout_random: actions from the sample_actions(seed, step0 + t) stream,
        state kept on-chip): writes the rollout slots frames (T, N, 15) (frames[t] = newest frame
        of the observation step t acts on), actions (T, N, 4), rewards (T, N), next_start (T-1, N)
        (episode starts of slots 1..T-1) and last_start (N,), and leaves the env at its
        observation after the last step (self.obs). Bit-identical to n_steps step_rollout calls.
        Any stack_k and mode (cfg5: random ICs + gusts). Windowed layout: the final observation
        is written into both histories at a window beside the current one (when no such window
        fits in the history, the current windows are first moved to its front); no terminal
        observation is kept for the last step's finished lanes."""
        T = int(n_steps)
        n = self.n
        for name, x, shape in (("frames", frames, (T, n, F16_OBS_DIM)), ("actions", actions, (T, n, 4)),
                               ("rewards", rewards, (T, n)), ("last_start", last_start, (n,))):
            if x is None or tuple(x.shape) != shape or x.dtype != self.torch.float32 or not x.is_contiguous() \
                    or x.device != self.device:
                raise ValueError("%s must be a contiguous float32 %s tensor on %s" % (name, shape, self.device))
        if T > 1 and (next_start is None or tuple(next_start.shape) != (T - 1, n) or not next_start.is_contiguous()
                      or next_start.dtype != self.torch.float32 or next_start.device != self.device):
            raise ValueError("next_start must be a contiguous float32 (T-1, N) tensor")
        sd, st = int(seed) & 0xFFFFFFFFFFFFFFFF, int(step0) & 0xFFFFFFFFFFFFFFFF
        if self.window:
            k, p = self.k, self._p
            q = p + k if p + k < self.T else k - 1  # the output window: beside the input one
            if q - k + 1 <= p and p - k + 1 <= q:
                # (T < 3K - 1 and the window near the front): move the current windows
                # of both histories to positions 0 .. K-1 first; the output window K .. 2K-1 then
                # fits whenever T >= 2K (window_check's bound). The lanes' FRESH marks describe
                # window-relative positions, so they stay valid.
                for b in (0, 1):
                    if self._env_major:
                        self._hist[b, :, :k].copy_(self._hist[b, :, p - k + 1:p + 1].clone())
                    else:
                        self._hist[b, :k].copy_(self._hist[b, p - k + 1:p + 1].clone())
                p = self._p = k - 1
                q = 2 * k - 1
            check(lib().f16env_window_rollout_random(self._h, self._stream(), sd, st, T, self._cur, p, q, _ptr(frames),
                                                     _ptr(actions), _ptr(rewards), _ptr(next_start), _ptr(last_start)),
                  "f16env_window_rollout_random")
            self._p = q
            self._op += 1
            self.terminal_obs = self._window(1)
            return
        prev = self._obs[self._cur]
        nxt = self._obs[self._cur ^ 1]
        check(lib().f16env_rollout_random(self._h, self._stream(), sd, st, T, _ptr(prev), _ptr(nxt), _ptr(frames),
                                          _ptr(actions), _ptr(rewards), _ptr(next_start), _ptr(last_start)),
              "f16env_rollout_random")
        self._cur ^= 1

    def profile_kernel(self, fn, launches: int, times: Optional[list] = None):
        """Run fn() (which issues `launches` steps) with the step kernel's own dispatch events
        recording each launch; returns (avg_ms, min_ms, launches timed). `times`, a list,
        receives each launch's (start, stop) in ms from the first launch's start."""
        L = lib()
        check(L.f16env_profile_begin(self._h, int(launches)), "f16env_profile_begin")
        fn()
        if times is not None:
            buf = (ctypes.c_double * (2 * int(launches)))()
            got = L.f16env_profile_times(self._h, buf, int(launches))
            if got < 0:
                check(got, "f16env_profile_times")
            times.extend((buf[2 * i], buf[2 * i + 1]) for i in range(got))
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

    @property
    def obs_bounds_count(self) -> int:
        """Lane-steps since creation whose new observation frame had a finite value outside the
        observation space (obs_check=True; jsbsim_gym.py:268-285's warning, counted on the
        device). Waits for the handle's stream."""
        c = ctypes.c_uint64()
        check(lib().f16env_obs_bounds_count(self._h, self._stream(), ctypes.byref(c)), "f16env_obs_bounds_count")
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
        if self.window:
            self._op += 1
        self.torch.cuda.current_stream(self.device).synchronize()

    def set_obs(self, obs):
        """Overwrite the current observation (window layout: both histories' windows, so the
        next step continues from it)."""
        o = self.torch.as_tensor(obs, dtype=self.torch.float32)
        if self.window:
            self._window(0).copy_(o)
            self._window(1).copy_(o)
            # both windows are whole now: lanes reset before this need no refill at the next step
            check(lib().f16env_window_clear_fresh(self._h, self._stream()), "f16env_window_clear_fresh")
            self._op += 1
        else:
            self._obs[self._cur].copy_(o)

    def poses(self):
        """(N, 10) float32 render/telemetry poses of the current observation's newest frame
        (telemetry.poses(self.obs[:, -1]), JSBSimEnv.render, jsbsim_gym.py:381-415). A
        fused_poses handle's step writes them in its epilogue, so after such a step this is the
        bound buffer with no launch; otherwise (or after any other op) f16env_poses computes them.
        The result is a view valid until the next op."""
        from .telemetry import poses as _poses
        if self._poses is not None and self._poses_op == getattr(self, "_op", None):
            return self._poses
        out = _poses(self.obs, out=self._poses)  # (the newest frame of each stack, read in place)
        if self._poses is not None:
            self._poses_op = getattr(self, "_op", None)
        return out

    def obs_features(self):
        """(N, K, 17) float32 policy features of the current observation (features.py:37-67 per
        frame; LMA_features.py:757-765 over the stack), equal bit for bit to
        features.features(self.obs). Windowed layout: kept in two feature histories beside the
        frame histories ([T][N][17] per parity, position-major; the result is a view, valid
        until the first call after the next step, which writes the other parity's rows), so a
        call after each step transforms one frame per
        env (f16env_features_window_step) instead of K, and a rollout-slot step (step_rollout,
        collect_rollout) keeps them in its own epilogue (F16_SLOT_FEATURE_WINDOW: no launch
        here at all). The first call, a call after a reset,
        set_state, set_obs or rollout_random, the call after the step that follows one of
        those, and a call after a step not followed by a call transform both whole windows.
        Contiguous layout: features(self.obs)."""
        from .features import FEATURES_DIM, features
        if not self.window:
            return features(self.obs)
        n, k, L = self.n, self.k, lib()
        self._feature_hist()
        cur, p = self._cur, self._p
        if self._feat_op != self._op:
            wrow, wenv = (16, self.T * 16) if self._env_major else (n * 16, 16)
            autoreset = 0 if int(self.cfg.flags) & F16_FLAG_NO_AUTORESET else 1
            s = self._stream()
            after_step = self._step_op == self._op
            hc, fc, fo = self._hist_ptr[cur], self._fh_ptr[cur], self._fh_ptr[cur ^ 1]
            if self._feat_prev_ok and self._feat_op == self._op - 1 and after_step:
                check(L.f16env_features_window_step(s, n, k, p, hc, wrow, wenv, fc, fo, self.term.data_ptr(),
                                                    self.trunc.data_ptr(), autoreset, 1),
                      "f16env_features_window_step")
                self.feature_window_calls["incremental"] += 1
            else:
                self.feature_window_calls["full"] += 1
                for b in (cur, cur ^ 1):  # positions p-K+1 .. p of history b: K "rows" of N frames
                    check(L.f16env_features_strided(s, k, n, self._hist_ptr[b] + 4 * (p - k + 1) * wrow, wrow, wenv,
                                                    self._fh_ptr[b] + 4 * (p - k + 1) * n * FEATURES_DIM),
                          "f16env_features_strided")
                # the next step's window fills of the lanes this state's step reset, applied ahead
                # (f16env_features_window_step's invariant); after any other op the lanes due a
                # fill are not known here, so the call after the next step transforms whole
                # windows again
                self._feat_prev_ok = after_step
                if after_step:
                    check(L.f16env_features_window_step(s, n, k, p, hc, wrow, wenv, fc, fo, self.term.data_ptr(),
                                                        self.trunc.data_ptr(), autoreset, 0),
                          "f16env_features_window_step")
            self._feat_op = self._op
        v = self._fviews[cur][p]
        if v is None:
            v = self._fviews[cur][p] = self._fh[cur, p - k + 1:p + 1].transpose(0, 1)
        return v

    def _feature_hist(self):
        """The two feature histories [T][N][17] beside the frame histories, allocated and bound
        once (rollout-slot steps with F16_SLOT_FEATURE_WINDOW and fused_features steps update them
        in their epilogue); positions outside the window are written before they are read."""
        if self._fh is None:
            from .features import FEATURES_DIM
            t = self.torch
            self._fh = t.empty((2, self.T, self.n, FEATURES_DIM), dtype=t.float32, device=self.device)
            self._fh_ptr = (self._fh[0].data_ptr(), self._fh[1].data_ptr())
            check(lib().f16env_window_feature_bind(self._h, *self._fh_ptr), "f16env_window_feature_bind")
            self._fviews = [[None] * self.T for _ in range(2)]

    def trim(self, ic):
        t = self.torch
        c = t.as_tensor(ic, dtype=t.float64, device=self.device).contiguous()
        out = t.zeros_like(c)
        res = t.zeros((self.n, 3), dtype=t.float64, device=self.device)
        check(lib().f16env_trim(self._h, self._stream(), _ptr(c), _ptr(out), _ptr(res)), "f16env_trim")
        return out, res

    def sample_actions(self, seed: int, step: int, out=None, steps: int | None = None):
        """Uniform Box actions from the device Philox stream keyed by (seed, env id, step)
        (action_space.sample() per env, jsbsim_gym.py:143-148): (N, 4) for `step`, or with
        `steps` = T the (T, N, 4) batches of steps step .. step+T-1 in ONE launch
        (f16env_sample_actions_steps, bit-identical to T single calls)."""
        t = self.torch
        if steps is None:
            if out is None:
                out = t.empty((self.n, 4), dtype=t.float32, device=self.device)
            if tuple(out.shape) != (self.n, 4) or not out.is_contiguous():
                raise ValueError("out must be a contiguous (N, 4) float32 tensor")
            check(lib().f16env_sample_actions(self._h, self._stream(), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                              int(step) & 0xFFFFFFFFFFFFFFFF, _ptr(out)), "f16env_sample_actions")
            return out
        T = int(steps)
        if out is None:
            out = t.empty((T, self.n, 4), dtype=t.float32, device=self.device)
        if tuple(out.shape) != (T, self.n, 4) or not out.is_contiguous():
            raise ValueError("out must be a contiguous (steps, N, 4) float32 tensor")
        check(lib().f16env_sample_actions_steps(self._h, self._stream(), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                                int(step) & 0xFFFFFFFFFFFFFFFF, T, _ptr(out)),
              "f16env_sample_actions_steps")
        return out


def _optional_class(module: str, name: str):
    """A base class from an optional dependency (stable_baselines3 / gymnasium), or None."""
    try:
        mod = __import__(module, fromlist=[name])
        return getattr(mod, name)
    except Exception:  # noqa: BLE001 - absent or broken: the duck-typed surface is used
        return None


# stable_baselines3/common/base_class.py:215 accepts an env as-is only when
# isinstance(env, VecEnv); gymnasium learners check gymnasium.Env / gymnasium.vector.VectorEnv.
# When those libraries are importable the facades below ARE subclasses of their ABCs.
SB3VecEnv = _optional_class("stable_baselines3.common.vec_env.base_vec_env", "VecEnv")
GymEnv = _optional_class("gymnasium", "Env")
GymVectorEnv = _optional_class("gymnasium.vector", "VectorEnv")


def _bases(*classes):
    return tuple(c for c in classes if c is not None) or (object,)


class _ReadOnlyInfo(dict):
    """The info dict of every lane that did not finish its step: {"TimeLimit.truncated": False}
    (dummy_vec_env.py:56-73 through TimeLimit + Monitor). ONE shared, immutable instance per
    step instead of N fresh dicts; lanes that finished get fresh dicts of their own."""

    def _ro(self, *a, **k):
        raise TypeError("info of a lane that did not finish is shared and read-only")

    __setitem__ = __delitem__ = update = pop = popitem = clear = setdefault = _ro  # type: ignore[assignment]

    def copy(self):
        return dict(self)

    def __deepcopy__(self, memo):
        return dict(self)


_NOT_DONE_INFO = _ReadOnlyInfo({"TimeLimit.truncated": False})


class _HostStaging:
    """Numpy mode of the facades: pinned host buffers the step's outputs land in, with one
    stream sync per step. obs goes to a ring of `ring` pinned (N, K, 15) buffers -- the arrays a
    step returns stay valid for `ring` - 1 further steps (SB3 copies obs into its buffers one step
    later: on_policy_algorithm.py:250-257, off_policy_algorithm.py _store_transition); rewards /
    terminated / truncated arrive by ONE copy of the handle's packed step_flags buffer."""

    def __init__(self, envs: "F16Envs", ring: int = 3):
        t = envs.torch
        self.t, self.envs = t, envs
        pin = envs.device.type == "cuda"
        n, k = envs.n, envs.k
        self.obs = [t.empty((n, k, F16_OBS_DIM), dtype=t.float32, pin_memory=pin) for _ in range(ring)]
        self.flags = t.empty(envs.step_flags.shape, dtype=t.uint8, pin_memory=pin)
        self.act = t.empty((n, 4), dtype=t.float32, pin_memory=pin)
        self.i = 0

    def actions_to_device(self, actions):
        """Host actions -> the handle's device action buffer through pinned staging; device
        float32 (N, 4) tensors pass through untouched."""
        t, e = self.t, self.envs
        if isinstance(actions, t.Tensor):
            if actions.device == e.device and actions.dtype == t.float32 and actions.is_contiguous() \
                    and tuple(actions.shape) == (e.n, 4):
                return actions
            actions = actions.detach().to("cpu", t.float32).numpy()
        a = np.asarray(actions, dtype=np.float32)
        if a.size != e.n * 4:
            raise ValueError("actions must hold (N, 4) = (%d, 4) values, got shape %s" % (e.n, a.shape))
        self.act.numpy()[...] = a.reshape(e.n, 4)
        e._act.copy_(self.act, non_blocking=True)
        return e._act

    def fetch(self, obs_dev, with_flags: bool = True):
        """Copy obs (and rew/term/trunc) to pinned memory, wait once; numpy views."""
        o = self.obs[self.i]
        self.i = (self.i + 1) % len(self.obs)
        o.copy_(obs_dev, non_blocking=True)
        if with_flags:
            self.flags.copy_(self.envs.step_flags, non_blocking=True)
        if self.envs.device.type == "cuda":
            self.t.cuda.current_stream(self.envs.device).synchronize()
        n = self.envs.n
        f = self.flags.numpy()
        return o.numpy(), f[:4 * n].view(np.float32), f[4 * n:5 * n], f[5 * n:6 * n]

    def done_rows(self, idx: np.ndarray):
        """terminal obs, episode return / length of the lanes in idx (small device gathers)."""
        e, t = self.envs, self.t
        i = t.as_tensor(idx, dtype=t.int64).to(e.device, non_blocking=True)
        return (e.terminal_obs.index_select(0, i).cpu().numpy(), e.ep_return.index_select(0, i).cpu().numpy(),
                e.ep_len.index_select(0, i).cpu().numpy())


class _HostWindow:
    """Numpy mode over a windowed handle (obs_layout="window", position-major): the host keeps
    a pinned mirror of the device's two frame histories, [2][Th][N][16], and per step copies
    only the step's new 64-B slot block of each (position p of both device histories: 2 x N x 64
    B, contiguous) instead of the whole (N, K, 15) observation (N x K x 60 B: 39 MB per step at
    65 536 envs, K = 10). The host then repeats what the windowed step kernel does to the
    windows of reset lanes (f16env.hip WIN block): lanes reset by this step get K-1 copies of
    their reset frame in the current history's window, lanes reset by the previous step get
    the same fill from the other history (the kernel's FRESH fill). The observation returned is
    a strided numpy view (N, K, 15) of the current host history's window (strides 64 B, N x 64 B,
    4 B), valid until the step after next -- the device layout's guarantee, which SB3 needs
    (it stores obs one step later, on_policy_algorithm.py:247-254); the terminal observation is
    the other history's window, as on the device. The host ring has its own Th positions and
    moves its last K-1 to the front when full."""

    def __init__(self, envs: "F16Envs", th: int = 0):
        t = envs.torch
        self.t, self.envs = t, envs
        n, k = envs.n, envs.k
        self.Th = int(th) if th else max(128, 4 * k)
        pin = envs.device.type == "cuda"
        self.H = t.zeros((2, self.Th, n, 16), dtype=t.float32, pin_memory=pin)
        self.Hn = self.H.numpy()
        self.flags = t.empty(envs.step_flags.shape, dtype=t.uint8, pin_memory=pin)
        self.act = t.empty((n, 4), dtype=t.float32, pin_memory=pin)
        self.par = 0
        self.q = k - 1
        self.prev_reset = None
        self.autoreset = not (int(envs.cfg.flags) & F16_FLAG_NO_AUTORESET)

    actions_to_device = _HostStaging.actions_to_device

    def _view(self, par: int) -> np.ndarray:
        k, q = self.envs.k, self.q
        return self.Hn[par, q - k + 1:q + 1, :, :F16_OBS_DIM].transpose(1, 0, 2)

    def fetch(self, obs_dev, with_flags: bool = True):
        e, k, n = self.envs, self.envs.k, self.envs.n
        if not with_flags:  # after a reset: the whole current window, into both host histories
            self.q, self.prev_reset = k - 1, None
            w = obs_dev.transpose(0, 1)
            for b in (0, 1):
                self.H[b, :k, :, :F16_OBS_DIM].copy_(w, non_blocking=True)
            if e.device.type == "cuda":
                self.t.cuda.current_stream(e.device).synchronize()
            return self._view(self.par), None, None, None
        q = self.q + 1
        if q >= self.Th:  # host restart: the last K-1 positions to the front of both histories
            for b in (0, 1):
                self.Hn[b, :k - 1] = self.Hn[b, q - k + 1:q]
            q = k - 1
        par = self.par ^ 1
        cur, p = e._cur, e._p
        self.H[par, q].copy_(e._hist[cur, p], non_blocking=True)
        self.H[par ^ 1, q].copy_(e._hist[cur ^ 1, p], non_blocking=True)
        self.flags.copy_(e.step_flags, non_blocking=True)
        self.t.cuda.current_stream(e.device).synchronize()
        f = self.flags.numpy()
        rew, term, trunc = f[:4 * n].view(np.float32), f[4 * n:5 * n], f[5 * n:6 * n]
        Hc = self.Hn[par]
        if k > 1 and self.prev_reset is not None and self.prev_reset.size:  # the kernel's FRESH fill
            idx = self.prev_reset
            Hc[q - k + 1:q, idx] = self.Hn[par ^ 1, q - 1, idx][None]
        self.prev_reset = None
        if self.autoreset:
            idx = np.flatnonzero(term | trunc)
            if idx.size:
                if k > 1:  # lanes reset by this step: K-1 copies of their reset frame
                    Hc[q - k + 1:q, idx] = Hc[q, idx][None]
                self.prev_reset = idx
        self.q, self.par = q, par
        return self._view(par), rew, term, trunc

    def done_rows(self, idx: np.ndarray):
        """terminal obs (the other host history's window), episode return / length."""
        e, t = self.envs, self.t
        tobs = np.ascontiguousarray(self._view(self.par ^ 1)[idx])
        i = t.as_tensor(idx, dtype=t.int64).to(e.device, non_blocking=True)
        return tobs, e.ep_return.index_select(0, i).cpu().numpy(), e.ep_len.index_select(0, i).cpu().numpy()


def _staging(envs, copy_obs: bool = False):
    """The numpy-mode staging for a handle: the host window mirror for position-major windowed
    handles (only the new slots cross PCIe), else whole-observation copies."""
    if getattr(envs, "window", False) and not getattr(envs, "_env_major", True) and hasattr(envs, "_hist") \
            and not copy_obs:
        return _HostWindow(envs)
    return _HostStaging(envs)


class F16VecEnv(*_bases(SB3VecEnv)):
    """Vectorised drop-in for ``DummyVecEnv([lambda: Monitor(gym.make("JSBSim-v0"))] * N)``.

    Honours the SB3 VecEnv contract (base_vec_env.py:50-357): ``reset() -> obs``,
    ``step_async/step_wait -> (obs, rews, dones, infos)``, auto-reset with
    ``infos[i]["terminal_observation"]`` and ``infos[i]["TimeLimit.truncated"]``
    (dummy_vec_env.py:56-73), Monitor's ``infos[i]["episode"] = {r, l, t}``
    (monitor.py:96-109), ``seed()`` applied at the next reset (:292-309). When
    stable_baselines3 is importable this class IS a ``VecEnv`` subclass, so
    ``BaseAlgorithm._wrap_env`` (base_class.py:215) takes it as-is.

    Numpy mode (default, what SB3 consumes): the handle steps in the windowed layout and the
    host keeps a pinned mirror of its frame histories, so per step only the new frame slots
    (2 x N x 64 B) and the packed rewards/flags cross PCIe, one stream sync (_HostWindow); the
    obs returned is a strided (N, K, 15) numpy view of that mirror, valid until the step after
    next (SB3 stores it one step later). ``copy_obs=True`` returns contiguous copies instead
    (whole-observation D2H per step, _HostStaging), for consumers that keep observations
    longer. Infos of lanes that did not finish share one read-only dict.
    ``return_numpy=False`` keeps everything on the GPU (infos is then None: the caller reads the
    ``last_step`` device tensors). ``envs=`` wraps an existing handle instead of creating one.
    The handle it creates steps in the windowed observation layout in numpy mode and in the
    contiguous one in device mode (``obs_layout=`` overrides)."""

    metadata = {"render_modes": []}

    def __init__(self, num_envs: int = 1, stack_k: int = 10, device=None, seed: int = 0,
                 return_numpy: bool = True, env_id_base: int = 0, envs=None, copy_obs: bool = False, **kw):
        if envs is None:
            # numpy mode copies every observation to the host anyway, so the env steps in the
            # windowed layout (no per-step stack rewrite: 16.9 vs 27.8 us at K = 10, 65 536 envs);
            # device mode keeps dense (N, K, 15) buffers unless asked otherwise
            kw.setdefault("obs_layout", "window" if return_numpy else "contiguous")
            envs = F16Envs(num_envs, stack_k=stack_k, device=device, seed=seed, env_id_base=env_id_base, **kw)
        self.envs = envs
        n = self.envs.n
        self.render_mode = None
        self._attrs: dict = {}
        obs_space, act_space = spaces.observation_space(self.envs.k), spaces.action_space()
        if SB3VecEnv is not None:
            SB3VecEnv.__init__(self, n, obs_space, act_space)  # base_vec_env.py:59-94
        else:
            self.num_envs = n
            self.observation_space, self.action_space = obs_space, act_space
            self.reset_infos: list = [{} for _ in range(n)]
            self._seeds: list = [None for _ in range(n)]
            self._options: list = [{} for _ in range(n)]
        self.return_numpy = bool(return_numpy)
        self.copy_obs = bool(copy_obs)
        self._host = _staging(self.envs, self.copy_obs) if self.return_numpy else None
        self._actions = None
        self._t_start = time.time()
        self.last_step: Optional[StepOut] = None

    # -- VecEnv API -------------------------------------------------------------------------
    def reset(self):
        goals = None
        if any(s is not None for s in self._seeds):
            # seeded lanes follow the reference's numpy stream (jsbsim_gym.py:312-323); NaN rows
            # draw the device goal, all in ONE reset (each lane's episode counter advances once)
            goals = np.full((self.num_envs, 3), np.nan, np.float32)
            for i, s in enumerate(self._seeds):
                if s is not None:
                    goals[i] = reference_goal(s)
        obs = self.envs.reset(goals=goals)
        self._seeds = [None for _ in range(self.num_envs)]
        self._options = [{} for _ in range(self.num_envs)]
        self.reset_infos = [{} for _ in range(self.num_envs)]
        self._t_start = time.time()
        if not self.return_numpy:
            return obs
        return self._host.fetch(obs, with_flags=False)[0]

    def step_async(self, actions) -> None:
        self._actions = actions

    def step_wait(self):
        if not self.return_numpy:
            out = self.envs.step(self._actions)
            self.last_step = out
            return out.obs, out.rew, (out.terminated | out.truncated).bool(), None
        out = self.envs.step(self._host.actions_to_device(self._actions))
        self.last_step = out
        obs, rew, term_u8, trunc_u8 = self._host.fetch(out.obs)
        dones = (term_u8 | trunc_u8).astype(bool)
        infos = [_NOT_DONE_INFO] * self.num_envs
        idx = np.flatnonzero(dones)
        if idx.size:
            tobs, eret, elen = self._host.done_rows(idx)
            t = round(time.time() - self._t_start, 6)
            for j, i in enumerate(idx.tolist()):
                info = {"TimeLimit.truncated": bool(trunc_u8[i] and not term_u8[i]),
                        "terminal_observation": tobs[j],
                        "episode": {"r": round(float(eret[j]), 6), "l": int(elen[j]), "t": t}}
                if term_u8[i] & 2:  # NaN guard quarantine (nan_guard=True)
                    info["nonfinite"] = True
                infos[i] = info
        if self.copy_obs:
            obs = np.array(obs)
        return obs, rew.copy(), dones, infos

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

    # per-lane attributes of the reference env (jsbsim_gym.py:103-118), read from the device state
    _LANE_ATTRS = ("current_step", "goal", "state")
    _CONST_ATTRS = {"num_stacked_frames": "k", "max_episode_steps": None, "down_sample": None, "dg": None}

    def get_attr(self, attr_name: str, indices=None) -> list:
        idx = list(self._indices(indices))
        if attr_name in self._attrs:
            return [self._attrs[attr_name] for _ in idx]
        if attr_name in ("render_mode", "observation_space", "action_space", "metadata"):
            return [getattr(self, attr_name) for _ in idx]
        if attr_name == "spec":
            return [None for _ in idx]
        c = self.envs.cfg
        const = {"num_stacked_frames": self.envs.k, "max_episode_steps": int(c.max_steps),
                 "down_sample": int(c.down_sample), "dg": float(c.dg_m)}
        if attr_name in const:
            return [const[attr_name] for _ in idx]
        if attr_name in self._LANE_ATTRS:
            from .abi import F16C_GOAL, F16C_STEP
            if attr_name == "state":  # jsbsim_gym.py:181-193: newest frame's 12 state values
                rows = self.envs.obs[:, -1, :12].index_select(0, self.envs.torch.as_tensor(idx, device=self.envs.device))
                return list(rows.cpu().numpy())
            st = self.envs.get_state().cpu().numpy()
            if attr_name == "current_step":
                return [int(st[i, F16C_STEP]) for i in idx]
            return [st[i, F16C_GOAL:F16C_GOAL + 3].astype(np.float32) for i in idx]
        raise AttributeError(attr_name)

    def set_attr(self, attr_name: str, value: Any, indices=None) -> None:
        self._attrs[attr_name] = value

    def env_method(self, method_name: str, *method_args, indices=None, **method_kwargs) -> list:
        """The single-env methods that make sense on device lanes: render (no renderer: None,
        like an env without render_mode), get_wrapper_attr (gymnasium >= 1.0 attribute access),
        reset (the indexed lanes, new goals from the device stream)."""
        idx = list(self._indices(indices))
        if method_name == "render":
            return [None for _ in idx]
        if method_name == "get_wrapper_attr":
            return self.get_attr(method_args[0], idx)
        if method_name == "reset":
            mask = np.zeros(self.num_envs, np.uint8)
            mask[idx] = 1
            full = self.envs.reset(mask=mask)
            if self._host is not None:  # the host mirror takes the new windows
                self._host.fetch(full, with_flags=False)
            obs = full[self.envs.torch.as_tensor(idx, device=self.envs.device)]
            return [(o, {}) for o in obs.cpu().numpy()]
        raise AttributeError("F16VecEnv lanes have no per-env method %r" % method_name)

    def env_is_wrapped(self, wrapper_class, indices=None) -> list:
        name = getattr(wrapper_class, "__name__", str(wrapper_class))
        # Monitor / TimeLimit / PositionReward semantics are built into the kernel
        wrapped = name in ("Monitor", "TimeLimit", "PositionReward")
        return [wrapped for _ in self._indices(indices)]

    def has_attr(self, attr_name: str) -> bool:
        try:
            self.get_attr(attr_name, 0)
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


class F16GymVectorEnv(*_bases(GymVectorEnv)):
    """gymnasium.vector.VectorEnv surface over the same kernel (the north star's "Gymnasium
    VectorEnv step()/reset()"), for gymnasium-native learners; a VectorEnv subclass when
    gymnasium is importable (registered as "JSBSim-v0"'s vector entry point,
    f16_jsb_amd/__init__.py). Autoreset mode SAME_STEP -- what the kernel does: a lane that
    terminates or truncates returns its reset observation in the same step, and

      infos["final_obs"] / infos["_final_obs"]   final (K,15) observation / mask
      infos["episode"] = {"r", "l", "t"}, infos["_episode"]   (RecordEpisodeStatistics keys)

    are filled for the finished lanes (gymnasium's vector-info convention: a value array plus a
    "_key" boolean mask). ``reset(seed=s)`` seeds env i with s + i (the reference's
    default_rng(seed) goal, jsbsim_gym.py:312-323). Single-env semantics are jsbsim_gym.py's
    JSBSimEnv wrapped in TimeLimit(1200) and PositionReward(1e-2) (jsbsim_gym.py:537-545).

    Numpy mode returns observations as strided views of a pinned host mirror of the windowed
    handle's frame histories (_HostWindow): an obs array stays valid until the step after next
    (the next step leaves it intact, the one after overwrites it). A consumer that keeps
    observations longer passes ``copy_obs=True`` (contiguous copies; whole-observation
    device-to-host copies per step). ``infos["final_obs"]`` is always a copy."""

    metadata = {"autoreset_mode": "SameStep", "render_modes": []}

    def __init__(self, num_envs: int = 1, stack_k: int = 10, device=None, seed: int = 0,
                 return_numpy: bool = True, envs=None, copy_obs: bool = False, **kw):
        if envs is None:  # as F16VecEnv: the windowed layout when observations go to the host
            kw.setdefault("obs_layout", "window" if return_numpy else "contiguous")
            envs = F16Envs(num_envs, stack_k=stack_k, device=device, seed=seed, **kw)
        self.envs = envs
        self.num_envs = self.envs.n
        self.single_observation_space = spaces.observation_space(self.envs.k)
        self.single_action_space = spaces.action_space()
        self.observation_space = spaces.batch_space(self.single_observation_space, self.num_envs)
        self.action_space = spaces.batch_space(self.single_action_space, self.num_envs)
        self.render_mode = None
        self.spec = None
        self.closed = False
        self.return_numpy = bool(return_numpy)
        self.copy_obs = bool(copy_obs)
        self._host = _staging(self.envs, self.copy_obs) if self.return_numpy else None
        self._t_start = time.time()

    def reset(self, *, seed=None, options=None):
        goals = None
        if seed is not None:
            seeds = [seed + i for i in range(self.num_envs)] if isinstance(seed, int) else list(seed)
            if len(seeds) != self.num_envs:
                raise ValueError("need one seed per env")
            goals = np.full((self.num_envs, 3), np.nan, np.float32)  # NaN rows: device goal
            for i, s in enumerate(seeds):
                if s is not None:
                    goals[i] = reference_goal(s)
        obs = self.envs.reset(goals=goals)
        self._t_start = time.time()
        if not self.return_numpy:
            return obs, {}
        o = self._host.fetch(obs, with_flags=False)[0]
        return (np.array(o) if self.copy_obs else o), {}

    def step(self, actions):
        if not self.return_numpy:
            out = self.envs.step(actions)
            term, trunc = out.terminated.bool(), out.truncated.bool()
            done = term | trunc
            infos = {}
            if bool(done.any()):
                t = round(time.time() - self._t_start, 6)
                infos["final_obs"] = out.terminal_obs.clone()
                infos["_final_obs"] = done
                infos["episode"] = {"r": t_where(done, out.ep_return, 0.0), "l": t_where(done, out.ep_len, 0),
                                    "t": t_where(done, t, 0.0)}
                infos["_episode"] = done
            return out.obs, out.rew, term, trunc, infos
        out = self.envs.step(self._host.actions_to_device(actions))
        obs, rew, term_u8, trunc_u8 = self._host.fetch(out.obs)
        term, trunc = term_u8.astype(bool), trunc_u8.astype(bool)
        done = term | trunc
        infos = {}
        idx = np.flatnonzero(done)
        if idx.size:
            t = round(time.time() - self._t_start, 6)
            tobs, eret, elen = self._host.done_rows(idx)
            final = np.zeros_like(obs)
            final[idx] = tobs
            r = np.zeros(self.num_envs)
            r[idx] = np.round(eret, 6)
            ln = np.zeros(self.num_envs, np.int32)
            ln[idx] = elen
            infos["final_obs"] = final
            infos["_final_obs"] = done
            infos["episode"] = {"r": r, "l": ln, "t": np.where(done, t, 0.0)}
            infos["_episode"] = done
        if self.copy_obs:
            obs = np.array(obs)
        return obs, rew.copy(), term, trunc, infos

    def close(self, **kwargs):
        if not self.closed:
            self.envs.close()
            self.closed = True

    def render(self):
        return None

    @property
    def unwrapped(self):
        return self


def t_where(mask, x, other):
    import torch
    if not isinstance(x, torch.Tensor):
        x = torch.full(mask.shape, float(x), device=mask.device)
    return torch.where(mask, x, torch.as_tensor(other, dtype=x.dtype, device=x.device))


class F16GymEnv(*_bases(GymEnv)):
    """ONE env with the single-env gymnasium surface of ``gym.make("JSBSim-v0")``
    (jsbsim_gym.py:537-545: JSBSimEnv wrapped in PositionReward(1e-2), TimeLimit(1200)) over a
    one-lane handle: ``reset(seed, options) -> (obs (K,15), {})`` with the default_rng(seed)
    goal of jsbsim_gym.py:312-323 (seed None: the device goal stream), ``step(action) ->
    (obs, reward, terminated, truncated, {})``, no auto-reset (the caller resets, as with the
    reference). A gymnasium.Env subclass when gymnasium is importable; the entry point
    "JSBSim-v0" is registered to (f16_jsb_amd/__init__.py), so an unchanged train.py gets a
    GPU-backed env from gym.make -- one env, SB3 then wraps it in Monitor + DummyVecEnv as it
    does the reference's. For throughput use F16VecEnv."""

    metadata = {"render_modes": []}

    def __init__(self, stack_k: int = 10, device=None, seed: int = 0, envs=None, **kw):
        self.envs = envs if envs is not None else F16Envs(1, stack_k=stack_k, device=device, seed=seed,
                                                          autoreset=False, **kw)
        self.observation_space = spaces.observation_space(self.envs.k)
        self.action_space = spaces.action_space()
        self.render_mode = None
        self._host = _HostStaging(self.envs, ring=2)

    def reset(self, *, seed=None, options=None):
        if GymEnv is not None:
            GymEnv.reset(self, seed=seed)  # gymnasium's np_random seeding (jsbsim_gym.py:302)
        goals = None if seed is None else reference_goal(seed)[None]
        obs = self.envs.reset(goals=goals)
        return self._host.fetch(obs, with_flags=False)[0][0].copy(), {}

    def step(self, action):
        out = self.envs.step(self._host.actions_to_device(np.asarray(action, np.float32).reshape(1, 4)))
        obs, rew, term, trunc = self._host.fetch(out.obs)
        return obs[0].copy(), float(rew[0]), bool(term[0]), bool(trunc[0]), {}

    def render(self):
        return None

    def close(self):
        self.envs.close()

    @property
    def unwrapped(self):
        return self


def make_gym_env(**kw) -> F16GymEnv:
    """gymnasium entry point of "JSBSim-v0" (jsbsim_gym.py:537-545 wrap_jsbsim counterpart)."""
    kw.pop("root", None)  # JSBSimEnv(root=...) names a JSBSim data directory: nothing to load here
    return F16GymEnv(**kw)


def make_gym_vector_env(num_envs: int = 1, **kw) -> F16GymVectorEnv:
    """gymnasium vector entry point of "JSBSim-v0" (gymnasium.make_vec)."""
    kw.pop("root", None)
    return F16GymVectorEnv(num_envs=num_envs, **kw)
