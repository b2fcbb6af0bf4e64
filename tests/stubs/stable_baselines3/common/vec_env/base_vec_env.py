"""Test stub: the VecEnv ABC's interface as stable_baselines3/common/vec_env/base_vec_env.py:50-357
defines it -- the same eight abstract methods, the same constructor side effects, the concrete
helpers callers use. Written for the test, not copied."""
from abc import ABC, abstractmethod

import numpy as np


class VecEnv(ABC):
    def __init__(self, num_envs, observation_space, action_space):
        self.num_envs = num_envs
        self.observation_space = observation_space
        self.action_space = action_space
        self.reset_infos = [{} for _ in range(num_envs)]
        self._seeds = [None for _ in range(num_envs)]
        self._options = [{} for _ in range(num_envs)]
        try:
            modes = self.get_attr("render_mode")
        except AttributeError:
            modes = [None for _ in range(num_envs)]
        assert all(m == modes[0] for m in modes)
        self.render_mode = modes[0]
        self.metadata = {"render_modes": [] if self.render_mode is None else [self.render_mode]}
        self.base_init_ran = True

    @abstractmethod
    def reset(self): ...

    @abstractmethod
    def step_async(self, actions): ...

    @abstractmethod
    def step_wait(self): ...

    @abstractmethod
    def close(self): ...

    @abstractmethod
    def get_attr(self, attr_name, indices=None): ...

    @abstractmethod
    def set_attr(self, attr_name, value, indices=None): ...

    @abstractmethod
    def env_method(self, method_name, *method_args, indices=None, **method_kwargs): ...

    @abstractmethod
    def env_is_wrapped(self, wrapper_class, indices=None): ...

    def has_attr(self, attr_name):
        try:
            self.get_attr(attr_name, 0)
            return True
        except AttributeError:
            return False

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def seed(self, seed=None):
        if seed is None:
            seed = int(np.random.randint(0, np.iinfo(np.uint32).max, dtype=np.uint32))
        self._seeds = [seed + i for i in range(self.num_envs)]
        return self._seeds

    def _get_indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        return [indices] if isinstance(indices, int) else indices
