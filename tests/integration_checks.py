"""Checks of the SB3 / gymnasium boundary on CPU (TEST INFRASTRUCTURE), run by
tests/test_integration.py twice: in-process (neither library installed: duck-typed facades)
and in a subprocess with tests/stubs on sys.path (the libraries "installed": the facades must
then subclass their ABCs and "JSBSim-v0" must be registered). The facades wrap the CPU
FakeEnvs (tests/fake_envs.py) through their envs= argument."""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def check_vecenv_contract():
    import f16_jsb_amd
    from f16_jsb_amd.env import F16VecEnv, _ReadOnlyInfo, reference_goal
    from fake_envs import FakeEnvs

    n, k = 6, 4
    fake = FakeEnvs(n, k, max_steps=6)
    venv = f16_jsb_amd.make("JSBSim-v0", envs=fake)
    assert isinstance(venv, F16VecEnv) and venv.num_envs == n
    assert venv.observation_space.shape == (k, 15) and venv.action_space.shape == (4,)
    # seed() applies at the next reset (base_vec_env.py:292-309); mixed seeded / unseeded lanes in
    # ONE reset: every lane's episode counter advances exactly once
    seeds = venv.seed(100)
    assert seeds == [100 + i for i in range(n)]
    venv._seeds[1] = None
    venv._seeds[4] = None
    obs = venv.reset()
    assert obs.shape == (n, k, 15) and obs.dtype == np.float32
    assert (fake.eps == 1).all(), fake.eps
    for i in range(n):
        want = (np.array([i, 0, -1], np.float32) if i in (1, 4) else reference_goal(100 + i))
        np.testing.assert_array_equal(obs[i, 0, 12:], want)
    assert venv._seeds == [None] * n
    kept = []
    ended = 0
    for t in range(12):
        act = np.full((n, 4), 0.25 * (t % 4), np.float32)
        obs, rew, dones, infos = venv.step(act)
        kept.append((obs, obs.copy()))
        assert obs.shape == (n, k, 15) and rew.dtype == np.float32 and dones.dtype == bool
        assert len(infos) == n
        for i in range(n):
            if not dones[i]:
                assert infos[i] == {"TimeLimit.truncated": False} and isinstance(infos[i], dict)
                assert isinstance(infos[i], _ReadOnlyInfo)
                np.testing.assert_array_equal(obs[i, -1, 3:7], act[i])
                continue
            ended += 1
            info = infos[i]
            assert not isinstance(info, _ReadOnlyInfo)
            term = i % 2 == 0
            assert info["TimeLimit.truncated"] == (not term)
            assert info["terminal_observation"].shape == (k, 15)
            np.testing.assert_array_equal(info["terminal_observation"][-1, 3:7], act[i])
            assert set(info["episode"]) == {"r", "l", "t"}
            assert info["episode"]["l"] == info["terminal_observation"][-1, 1]
            assert np.all(obs[i] == obs[i, :1])  # auto-reset: K copies of the reset frame
        nd = [i for i in range(n) if not dones[i]]
        if len(nd) >= 2:
            assert infos[nd[0]] is infos[nd[1]]
            try:
                infos[nd[0]]["x"] = 1
                raise AssertionError("shared info must be read-only")
            except TypeError:
                pass
        # an obs array returned two steps ago is still intact (pinned ring of 3)
        if len(kept) >= 3:
            a, snap = kept[-3]
            np.testing.assert_array_equal(a, snap)
    assert ended >= n
    # attributes of the reference env (jsbsim_gym.py:103-118) per lane
    assert venv.get_attr("num_stacked_frames") == [k] * n
    assert venv.get_attr("max_episode_steps", 2) == [6]
    assert venv.get_attr("current_step", [0, 3]) == [int(fake.steps[0]), int(fake.steps[3])]
    np.testing.assert_array_equal(venv.get_attr("goal", 5)[0], fake.goals[5])
    assert venv.has_attr("dg") and not venv.has_attr("no_such_attr")
    assert venv.env_method("render") == [None] * n
    assert venv.env_is_wrapped(type("Monitor", (), {})) == [True] * n
    venv.close()
    assert fake.closed


def check_gym_vector_contract():
    import f16_jsb_amd
    from f16_jsb_amd.env import reference_goal
    from fake_envs import FakeEnvs

    n = 5
    fake = FakeEnvs(n, 3, max_steps=4)
    env = f16_jsb_amd.make_vec("JSBSim-v0", num_envs=n, envs=fake)
    obs, info = env.reset(seed=7)
    assert info == {} and obs.shape == (n, 3, 15)
    for i in range(n):
        np.testing.assert_array_equal(obs[i, 0, 12:], reference_goal(7 + i))
    seen = 0
    for t in range(8):
        obs, rew, term, trunc, infos = env.step(np.zeros((n, 4), np.float32))
        done = term | trunc
        if done.any():
            assert set(infos) == {"final_obs", "_final_obs", "episode", "_episode"}
            np.testing.assert_array_equal(infos["_final_obs"], done)
            for i in np.flatnonzero(done):
                assert infos["episode"]["l"][i] == infos["final_obs"][i][-1, 1]
                seen += 1
        else:
            assert infos == {}
    assert seen >= n
    env.close()


def check_registration_and_subclassing():
    """With the libraries importable (tests/stubs): the facades subclass their ABCs, SB3's wrap
    gate (base_class.py:215) accepts F16VecEnv as-is, and "JSBSim-v0" is registered."""
    import gymnasium
    from stable_baselines3.common.base_class import wrap_env
    from stable_baselines3.common.vec_env import VecEnv

    import f16_jsb_amd
    from f16_jsb_amd import env as E
    from fake_envs import FakeEnvs

    assert issubclass(E.F16VecEnv, VecEnv) and not E.F16VecEnv.__abstractmethods__
    assert issubclass(E.F16GymVectorEnv, gymnasium.vector.VectorEnv)
    assert issubclass(E.F16GymEnv, gymnasium.Env)
    spec = gymnasium.registry["JSBSim-v0"]
    assert spec.entry_point == "f16_jsb_amd.env:make_gym_env" and spec.max_episode_steps == 1200
    assert spec.vector_entry_point == "f16_jsb_amd.env:make_gym_vector_env"
    assert f16_jsb_amd.register_gymnasium() is False  # idempotent
    venv = f16_jsb_amd.make("JSBSim-v0", envs=FakeEnvs(4, 4))
    assert isinstance(venv, VecEnv) and wrap_env(venv) is venv
    assert venv.base_init_ran and venv.render_mode is None and venv.metadata == {"render_modes": []}
    # gym.make_vec goes through the registry to the vector entry point
    v = gymnasium.make_vec("JSBSim-v0", num_envs=3, envs=FakeEnvs(3, 2))
    assert isinstance(v, E.F16GymVectorEnv) and isinstance(v, gymnasium.vector.VectorEnv)
    # gym.make's single env over a one-lane handle: reset(seed) goal, step 5-tuple, no autoreset
    g = gymnasium.make("JSBSim-v0", envs=FakeEnvs(1, 4, max_steps=3))
    assert isinstance(g, E.F16GymEnv) and isinstance(g, gymnasium.Env)
    o, info = g.reset(seed=3)
    np.testing.assert_array_equal(o[0, 12:], E.reference_goal(3))
    assert g.np_random_seed == 3
    o, r, te, tr, info = g.step(np.array([0.1, 0.2, 0.3, 0.4], np.float32))
    assert o.shape == (4, 15) and isinstance(r, float) and (te, tr) == (False, False) and info == {}


if __name__ == "__main__":
    sys.path.insert(0, HERE)
    check_registration_and_subclassing()
    check_vecenv_contract()
    check_gym_vector_contract()
    print("integration checks OK")
