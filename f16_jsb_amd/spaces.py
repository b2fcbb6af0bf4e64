"""Observation / action spaces of jsbsim_gym.JSBSimEnv (jsbsim_gym.py:28-53,135-148).

Uses gymnasium.spaces.Box when gymnasium is importable; otherwise a minimal Box with the
same attributes (low, high, shape, dtype, contains, sample) so SB3-style callers work.
"""
from __future__ import annotations

import numpy as np

EPSILON = 1e-5
# jsbsim_gym.py:32-41
SINGLE_OBS_LOW = np.array([
    -np.inf, -np.inf, -np.inf,
    0,
    -np.pi - EPSILON, -np.pi - EPSILON,
    -np.inf, -np.inf, -np.inf,
    -np.pi - EPSILON,
    -np.pi / 2 - EPSILON,
    -np.pi - EPSILON,
    -np.inf, -np.inf, 0,
], dtype=np.float32)
# jsbsim_gym.py:44-53
SINGLE_OBS_HIGH = np.array([
    np.inf, np.inf, np.inf,
    np.inf,
    np.pi + EPSILON, np.pi + EPSILON,
    np.inf, np.inf, np.inf,
    np.pi + EPSILON,
    np.pi / 2 + EPSILON,
    np.pi + EPSILON,
    np.inf, np.inf, np.inf,
], dtype=np.float32)
ACT_LOW = np.array([-1, -1, -1, 0], dtype=np.float32)   # jsbsim_gym.py:144
ACT_HIGH = np.array([1, 1, 1, 1], dtype=np.float32)     # jsbsim_gym.py:145

try:  # pragma: no cover - gymnasium is not installed in the build image
    from gymnasium.spaces import Box  # type: ignore
except Exception:  # noqa: BLE001
    class Box:  # minimal stand-in with gymnasium.spaces.Box's surface used by SB3
        def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
            self.dtype = np.dtype(dtype)
            low = np.asarray(low, dtype=self.dtype)
            high = np.asarray(high, dtype=self.dtype)
            if shape is None:
                shape = low.shape
            self.shape = tuple(shape)
            self.low = np.broadcast_to(low, self.shape).astype(self.dtype)
            self.high = np.broadcast_to(high, self.shape).astype(self.dtype)
            self._rng = np.random.default_rng(seed)

        def seed(self, seed=None):
            self._rng = np.random.default_rng(seed)
            return [seed]

        def contains(self, x) -> bool:
            x = np.asarray(x)
            return bool(x.shape == self.shape and np.can_cast(x.dtype, self.dtype)
                        and np.all(x >= self.low) and np.all(x <= self.high))

        def sample(self):
            lo = np.where(np.isfinite(self.low), self.low, -1e6)
            hi = np.where(np.isfinite(self.high), self.high, 1e6)
            return self._rng.uniform(lo, hi).astype(self.dtype)

        def __repr__(self):
            return "Box(%s, %s, %s, %s)" % (self.low.min(), self.high.max(), self.shape, self.dtype)

        def __eq__(self, other):
            return (isinstance(other, Box) and self.shape == other.shape
                    and np.array_equal(self.low, other.low) and np.array_equal(self.high, other.high))


def observation_space(stack_k: int = 10) -> "Box":
    return Box(low=np.tile(SINGLE_OBS_LOW, (stack_k, 1)), high=np.tile(SINGLE_OBS_HIGH, (stack_k, 1)),
               shape=(stack_k, len(SINGLE_OBS_LOW)), dtype=np.float32)


def action_space() -> "Box":
    return Box(low=ACT_LOW, high=ACT_HIGH, shape=(4,), dtype=np.float32)


def batch_space(space: "Box", n: int) -> "Box":
    """gymnasium.vector.utils.batch_space for a Box: the (n, *shape) Box of n copies."""
    return Box(low=np.broadcast_to(space.low, (n,) + space.shape), high=np.broadcast_to(space.high, (n,) + space.shape),
               shape=(n,) + space.shape, dtype=space.dtype)
