"""A CPU stand-in for F16Envs (TEST INFRASTRUCTURE): the same buffers and call surface, with
trivial deterministic "dynamics", so the host logic of the VecEnv / gymnasium facades
(f16_jsb_amd/env.py) can be tested without a GPU. Lane i terminates at step 2 + i % 3 when i is
even and truncates at max_steps when odd; frame = [lane, step, episode, act0..3, 0.., goal]."""
from __future__ import annotations

import numpy as np
import torch

from f16_jsb_amd.abi import F16C_EP_COUNT, F16C_GOAL, F16C_N, F16C_STEP, config_default
from f16_jsb_amd.env import StepOut


class FakeEnvs:
    def __init__(self, n, k=4, max_steps=6):
        self.torch, self.n, self.k = torch, n, k
        self.device = torch.device("cpu")
        self.cfg = config_default(n_envs=n, stack_k=k, max_steps=max_steps)
        nb = (6 * n + 15) // 16 * 16
        self.step_flags = torch.zeros(nb, dtype=torch.uint8)
        self.rew = self.step_flags[:4 * n].view(torch.float32)
        self.term = self.step_flags[4 * n:5 * n]
        self.trunc = self.step_flags[5 * n:6 * n]
        self.terminal_obs = torch.zeros((n, k, 15))
        self.ep_return = torch.zeros(n, dtype=torch.float64)
        self.ep_len = torch.zeros(n, dtype=torch.int32)
        self._act = torch.zeros((n, 4))
        self._obs = torch.zeros((n, k, 15))
        self.steps = np.zeros(n, np.int64)
        self.eps = np.zeros(n, np.int64)
        self.goals = np.zeros((n, 3), np.float32)
        self.ret = np.zeros(n)
        self.closed = False

    @property
    def obs(self):
        return self._obs

    def _frame(self, i, extra=(0, 0, 0, 0)):
        f = np.zeros(15, np.float32)
        f[0], f[1], f[2] = i, self.steps[i], self.eps[i]
        f[3:7] = extra
        f[12:15] = self.goals[i]
        return f

    def _reset_lane(self, i, goal=None):
        self.goals[i] = goal if goal is not None else (i, self.eps[i], -1.0)  # "device" goal
        self.eps[i] += 1
        self.steps[i] = 0
        self.ret[i] = 0.0
        self._obs[i] = torch.as_tensor(np.tile(self._frame(i), (self.k, 1)))

    def reset(self, mask=None, goals=None, ic=None):
        for i in range(self.n):
            if mask is not None and not mask[i]:
                continue
            g = None if goals is None else np.asarray(goals[i], np.float32)
            if g is not None and np.isnan(g[0]):
                g = None
            self._reset_lane(i, g)
        return self._obs

    def step(self, actions):
        a = actions.cpu().numpy()
        for i in range(self.n):
            self.steps[i] += 1
            f = self._frame(i, a[i])
            term = i % 2 == 0 and self.steps[i] == 2 + i % 3
            trunc = not term and self.steps[i] >= self.cfg.max_steps
            r = -10.0 if term else 0.5
            self.ret[i] += r
            self.rew[i], self.term[i], self.trunc[i] = r, int(term), int(trunc)
            row = torch.cat([self._obs[i, 1:], torch.as_tensor(f)[None]])
            if term or trunc:
                self.terminal_obs[i] = row
                self.ep_return[i], self.ep_len[i] = self.ret[i], int(self.steps[i])
                self._reset_lane(i)
            else:
                self._obs[i] = row
        return StepOut(self._obs, self.rew, self.term, self.trunc, self.terminal_obs, self.ep_return, self.ep_len)

    def get_state(self):
        s = torch.zeros((self.n, F16C_N), dtype=torch.float64)
        s[:, F16C_STEP] = torch.as_tensor(self.steps, dtype=torch.float64)
        s[:, F16C_EP_COUNT] = torch.as_tensor(self.eps, dtype=torch.float64)
        s[:, F16C_GOAL:F16C_GOAL + 3] = torch.as_tensor(self.goals, dtype=torch.float64)
        return s

    def close(self):
        self.closed = True
