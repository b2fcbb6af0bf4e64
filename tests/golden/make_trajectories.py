"""Regenerates tests/golden/trajectories.npz: fixed-input trajectories of the CPU oracle
(oracle/f16ref.c, the fp64 restatement of the JSBSim F-16 path; JSBSim itself is unavailable,
SURVEY.md 8c), committed so that

  * tests/test_golden_trajectories.py pins the oracle against drift (bit-exact re-run on CPU),
    and checks the HIP path against the committed outputs without running the oracle (the
    tolerances of tests/test_gpu_parity.py).

Two cases, inputs stored beside the outputs:
  const   16 envs, K = 4, altitude 3 000-30 000 ft x airspeed 600-1 200 fps ICs, fixed goals,
          one constant action per env, 300 steps: newest frame at steps 1, 10, 100, 300, every
          step's rewards and done flags;
  random  64 envs, K = 4, the reference IC (jsbsim_gym.py:166-170), goals from numpy
          default_rng(7), actions uniform over the Box from default_rng(0), 30 steps: newest
          frame at steps 1, 10, 30, every step's rewards and done flags.

    python tests/golden/make_trajectories.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle_ref import OracleEnvs, build_oracle, default_ic  # noqa: E402

CONST_CHECK = (1, 10, 100, 300)
RANDOM_CHECK = (1, 10, 30)


def const_inputs():
    n = 16
    ic = np.tile(default_ic(), (n, 1))
    ic[:, 2] = np.linspace(3000.0, 30000.0, n)
    ic[:, 3] = np.linspace(600.0, 1200.0, n)[::-1]
    ic[:, 7] = np.linspace(-0.05, 0.08, n)
    goals = np.stack([np.linspace(-8000, 8000, n), np.linspace(6000, -6000, n), np.full(n, 2500.0)], 1)
    act = np.stack([np.linspace(-0.05, 0.05, n), np.linspace(-0.15, 0.1, n), np.linspace(0.03, -0.03, n),
                    np.linspace(0.2, 1.0, n)], 1)
    return ic, goals.astype(np.float32), act.astype(np.float32)


def random_inputs():
    n = 64
    ic = np.tile(default_ic(), (n, 1))
    goals = np.random.default_rng(7).uniform([-5000, -5000, 1000], [5000, 5000, 4000], (n, 3)).astype(np.float32)
    acts = np.random.default_rng(0).uniform([-1, -1, -1, 0], [1, 1, 1, 1], (30, n, 4)).astype(np.float32)
    return ic, goals, acts


def run(ic, goals, acts, steps, check):
    n = len(goals)
    e = OracleEnvs(n, stack_k=4, seed=3)
    e.reset(goals=goals, ic=ic)
    frames, rews, dones = [], [], []
    for t in range(1, steps + 1):
        a = acts if acts.ndim == 2 else acts[t - 1]
        o, r, te, tr, *_ = e.step(a)
        rews.append(r)
        dones.append(te | tr)
        if t in check:
            frames.append(o[:, -1].copy())
    e.close()
    return np.stack(frames), np.stack(rews), np.stack(dones)


def generate():
    build_oracle()
    out = {}
    ic, goals, act = const_inputs()
    f, r, d = run(ic, goals, act, 300, CONST_CHECK)
    out.update(const_ic=ic, const_goals=goals, const_act=act, const_frames=f, const_rew=r, const_done=d)
    ic, goals, acts = random_inputs()
    f, r, d = run(ic, goals, acts, 30, RANDOM_CHECK)
    out.update(random_ic=ic, random_goals=goals, random_act=acts, random_frames=f, random_rew=r, random_done=d)
    return out


if __name__ == "__main__":
    np.savez_compressed(os.path.join(HERE, "trajectories.npz"), **generate())
    print("wrote", os.path.join(HERE, "trajectories.npz"))
