"""Test stub of gymnasium (see tests/stubs/README.md): Env, register/registry/make/make_vec with
entry points given as "module:attr" strings, vector.VectorEnv, spaces.Box."""
import importlib

from . import spaces, vector  # noqa: F401


class Env:
    def reset(self, *, seed=None, options=None):
        self.np_random_seed = seed


class EnvSpec:
    def __init__(self, id, entry_point, max_episode_steps=None, vector_entry_point=None, **kw):
        self.id, self.entry_point, self.max_episode_steps = id, entry_point, max_episode_steps
        self.vector_entry_point = vector_entry_point
        self.kwargs = kw.get("kwargs") or {}


registry = {}


def register(id, entry_point=None, max_episode_steps=None, vector_entry_point=None, **kw):
    registry[id] = EnvSpec(id, entry_point, max_episode_steps, vector_entry_point, **kw)


def _load(ep):
    mod, attr = ep.split(":")
    return getattr(importlib.import_module(mod), attr)


def make(id, **kw):
    return _load(registry[id].entry_point)(**kw)


def make_vec(id, num_envs=1, **kw):
    return _load(registry[id].vector_entry_point)(num_envs=num_envs, **kw)
