from .base_vec_env import VecEnv  # noqa: F401
