"""f16_jsb_amd -- MI355X-native vectorised F-16 environment (drop-in for the hot path of
Soham4001A/F16_JSB: jsbsim_gym.JSBSimEnv.step()/reset() behind the SB3 VecEnv boundary).

    import f16_jsb_amd
    env = f16_jsb_amd.make("JSBSim-v0", num_envs=65536, stack_k=4)   # train.py:34 drop-in

Importing the package registers "JSBSim-v0" with gymnasium when gymnasium is importable
(jsbsim_gym.py:537-545 counterpart: gym.make -> one env, gym.make_vec -> the vector env).
"""
from .abi import (F16C_N, F16_IC_N, F16_OBS_DIM, EnvConfig, config_default)  # noqa: F401
from .spaces import action_space, observation_space  # noqa: F401

__all__ = ["F16Envs", "F16VecEnv", "F16GymVectorEnv", "F16GymEnv", "make", "make_vec", "reference_goal",
           "config_default", "register_gymnasium"]

ENV_ID = "JSBSim-v0"


def __getattr__(name):  # lazy: importing the package must not require torch / a GPU
    if name in ("F16Envs", "F16VecEnv", "F16GymVectorEnv", "F16GymEnv", "reference_goal", "StepOut"):
        from . import env
        return getattr(env, name)
    raise AttributeError(name)


def make(env_id: str = ENV_ID, num_envs: int = 1, **kw):
    """The vectorised env for SB3 (TimeLimit(1200), PositionReward(gain=1e-2), Monitor and the
    DummyVecEnv auto-reset built in): ``PPO(policy, f16_jsb_amd.make("JSBSim-v0", num_envs=N))``
    replaces ``gym.make("JSBSim-v0")`` at train.py:34. A stable_baselines3 VecEnv subclass when
    SB3 is importable, so base_class.py:215 does not re-wrap it."""
    if env_id != ENV_ID:
        raise KeyError("unknown env id %r (only %r)" % (env_id, ENV_ID))
    from .env import F16VecEnv
    return F16VecEnv(num_envs=num_envs, **kw)


def make_vec(env_id: str = ENV_ID, num_envs: int = 1, **kw):
    """gymnasium.make_vec("JSBSim-v0", num_envs) counterpart: the gymnasium VectorEnv surface
    (F16GymVectorEnv, autoreset SAME_STEP) over the same kernel."""
    if env_id != ENV_ID:
        raise KeyError("unknown env id %r (only %r)" % (env_id, ENV_ID))
    from .env import F16GymVectorEnv
    return F16GymVectorEnv(num_envs=num_envs, **kw)


def register_gymnasium() -> bool:
    """Register "JSBSim-v0" with gymnasium (jsbsim_gym.py:537-545): entry point = one GPU-backed
    env (F16GymEnv, what gym.make returns), vector entry point = F16GymVectorEnv (what
    gym.make_vec returns), max_episode_steps 1200. A no-op returning False when gymnasium is not
    importable or the id is already registered (e.g. by the reference's own module)."""
    try:
        import gymnasium
    except Exception:  # noqa: BLE001
        return False
    registry = getattr(gymnasium, "registry", getattr(getattr(gymnasium, "envs", None), "registry", {}))
    if ENV_ID in registry:
        return False
    kw = dict(id=ENV_ID, entry_point="f16_jsb_amd.env:make_gym_env", max_episode_steps=1200)
    try:
        gymnasium.register(vector_entry_point="f16_jsb_amd.env:make_gym_vector_env", **kw)
    except TypeError:  # gymnasium < 1.0: no vector entry points
        gymnasium.register(**kw)
    return True


register_gymnasium()
