"""Test stub: the env-wrapping gate of BaseAlgorithm (base_class.py:204-222): an env that is not
a VecEnv instance is patched, Monitor-wrapped and put in a DummyVecEnv."""
from .vec_env.base_vec_env import VecEnv


class WouldRewrap(Exception):
    pass


def wrap_env(env):
    if not isinstance(env, VecEnv):
        raise WouldRewrap(type(env).__name__)
    return env
