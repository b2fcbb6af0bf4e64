"""f16_jsb_amd -- MI355X-native vectorised F-16 environment (drop-in for the hot path of
Soham4001A/F16_JSB: jsbsim_gym.JSBSimEnv.step()/reset() behind the SB3 VecEnv boundary).

    from f16_jsb_amd import F16VecEnv
    env = F16VecEnv(num_envs=65536, stack_k=4)      # train.py:34 drop-in
"""
from .abi import (F16C_N, F16_IC_N, F16_OBS_DIM, EnvConfig, config_default)  # noqa: F401
from .spaces import action_space, observation_space  # noqa: F401

__all__ = ["F16Envs", "F16VecEnv", "F16GymVectorEnv", "make", "make_vec", "reference_goal", "config_default"]


def __getattr__(name):  # lazy: importing the package must not require torch / a GPU
    if name in ("F16Envs", "F16VecEnv", "F16GymVectorEnv", "reference_goal", "StepOut"):
        from . import env
        return getattr(env, name)
    raise AttributeError(name)


def make(env_id: str = "JSBSim-v0", num_envs: int = 1, **kw):
    """Registry hook mirroring gym.make("JSBSim-v0") (jsbsim_gym.py:537-545): returns the
    vectorised env (TimeLimit(1200), PositionReward(gain=1e-2) and Monitor built in)."""
    if env_id != "JSBSim-v0":
        raise KeyError("unknown env id %r (only 'JSBSim-v0')" % env_id)
    from .env import F16VecEnv
    return F16VecEnv(num_envs=num_envs, **kw)


def make_vec(env_id: str = "JSBSim-v0", num_envs: int = 1, **kw):
    """gymnasium.make_vec("JSBSim-v0", num_envs) counterpart: the gymnasium VectorEnv surface
    (F16GymVectorEnv, autoreset SAME_STEP) over the same kernel."""
    if env_id != "JSBSim-v0":
        raise KeyError("unknown env id %r (only 'JSBSim-v0')" % env_id)
    from .env import F16GymVectorEnv
    return F16GymVectorEnv(num_envs=num_envs, **kw)
