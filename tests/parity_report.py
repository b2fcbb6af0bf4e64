"""HIP (fp32) vs oracle (fp64) divergence report -- run on the GPU box:

    python tests/parity_report.py [--n 64] [--steps 300] [--json out.json]

Prints max per-component error of the obs frame for (a) the IC frame, (b) one env step
from identical injected states, (c) trajectories under constant and random actions at
several horizons. Used to calibrate the tolerances in test_gpu_parity.py.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle_ref import OracleEnvs  # noqa: E402
from parity_tools import frame_err, report, state_err  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import torch
    from f16_jsb_amd.build import build
    from f16_jsb_amd.env import F16Envs

    build()
    n, K = args.n, 4
    out = {}
    rng = np.random.default_rng(0)
    goals = rng.uniform([-5000, -5000, 1000], [5000, 5000, 4000], size=(n, 3)).astype(np.float32)
    ref = OracleEnvs(n, stack_k=K, seed=7)
    g = F16Envs(n, stack_k=K, seed=7)
    o_ref = ref.reset(goals=goals)
    o_gpu = g.reset(goals=torch.as_tensor(goals)).cpu().numpy()
    out.update(report("ic", frame_err(o_gpu[:, -1], o_ref[:, -1])))
    out.update({"ic_state:" + k: v for k, v in state_err(g.get_state().cpu().numpy(), ref.get_state()).items()})

    # constant action trajectory
    act = np.tile(np.array([[0.05, -0.1, 0.02, 0.7]], np.float32), (n, 1))
    horizons = {1, 10, 30, 100, 300, 1000}
    for t in range(1, args.steps + 1):
        o_r = ref.step(act)[0]
        o_g = g.step(torch.as_tensor(act).cuda()).obs.cpu().numpy()
        if t in horizons:
            out.update(report("const@%d" % t, frame_err(o_g[:, -1], o_r[:, -1])))

    # one-step parity from identical injected state (random actions, random states)
    ref2 = OracleEnvs(n, stack_k=K, seed=3)
    ref2.reset(goals=goals)
    g2 = F16Envs(n, stack_k=K, seed=3)
    g2.reset(goals=torch.as_tensor(goals))
    worst = None
    worst_state = None
    for t in range(200):
        a = ref2.sample_actions(11, t)
        if t % 20 == 19:
            s = ref2.get_state()
            obs_prev = ref2_obs
            g2.set_state(s)
            g2.set_obs(torch.as_tensor(obs_prev))
            o_r = ref2.step(a)[0]
            o_g = g2.step(torch.as_tensor(a).cuda()).obs.cpu().numpy()
            e = frame_err(o_g[:, -1], o_r[:, -1])
            worst = e if worst is None else np.maximum(worst, e)
            se = state_err(g2.get_state().cpu().numpy(), ref2.get_state())
            worst_state = se if worst_state is None else {k: max(v, se[k]) for k, v in worst_state.items()}
            ref2_obs = o_r
        else:
            ref2_obs = ref2.step(a)[0]
    out.update(report("onestep", worst))
    out.update({"onestep_state:" + k: v for k, v in worst_state.items()})

    # random-action trajectories, divergence vs horizon
    ref3 = OracleEnvs(n, stack_k=K, seed=5)
    g3 = F16Envs(n, stack_k=K, seed=5)
    ref3.reset(goals=goals)
    g3.reset(goals=torch.as_tensor(goals))
    alive = np.ones(n, bool)
    for t in range(1, 301):
        a = ref3.sample_actions(99, t)
        o_r, _, te, tr, *_ = ref3.step(a)
        o_g = g3.step(g3.sample_actions(99, t)).obs.cpu().numpy()
        alive &= ~(te | tr)
        if t in (1, 3, 10, 30, 100, 300) and alive.any():
            out.update(report("rand@%d" % t, frame_err(o_g[alive, -1], o_r[alive, -1])))
    for k in sorted(out):
        print("%-28s %.3e" % (k, out[k]))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
