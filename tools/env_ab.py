#!/usr/bin/env python3
"""A/B timing of step-kernel variants selected by environment variables at handle creation
(F16ENV_OCC, F16ENV_GT; F16ENV_HALF and F16ENV_SPLIT selected the half-wave and two-wave-frame
layouts measured in profiles/r01_env_ab_half.json / r01_env_ab_split.json, since removed), one process, same library. Run on the GPU box:

    python tools/env_ab.py [--json out.json] [--steps 300] NAME=VAR=VAL[,VAR=VAL] ...

Each case is timed (HIP events, us per step, 16 pre-drawn action batches) at the listed env
counts / stack depths and checked bit-for-bit against the default handle over 20 steps.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
KNOBS = ("F16ENV_OCC", "F16ENV_GT")
SHAPES = [(65536, 4, 4), (65536, 4, 0), (131072, 4, 4), (65536, 10, 4), (4096, 4, 4)]


def make(n, k, ds, env):
    from f16_jsb_amd.env import F16Envs
    saved = {v: os.environ.pop(v, None) for v in KNOBS}
    os.environ.update(env)
    try:
        e = F16Envs(n, stack_k=k, down_sample=ds, seed=1)
    finally:
        for v in KNOBS:
            os.environ.pop(v, None)
            if saved[v] is not None:
                os.environ[v] = saved[v]
    e.reset()
    return e


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("cases", nargs="*")
    args = ap.parse_args()
    import torch
    from kernel_sweep import time_steps
    cases = {"default": {}}
    for c in args.cases:
        name, _, spec = c.partition("=")
        cases[name] = dict(kv.split("=", 1) for kv in spec.split(",") if kv)
    res = {}
    for n, k, ds in SHAPES:
        ref = make(n, k, ds, {})
        acts = [ref.sample_actions(5, t) for t in range(16)]
        key = "n%d_k%d_ds%d" % (n, k, ds)
        for name, env in cases.items():
            e = make(n, k, ds, env)
            same = True
            if name != "default":
                r2 = make(n, k, ds, {})
                for t in range(20):
                    a, b = r2.step(acts[t % 16]), e.step(acts[t % 16])
                    same = same and torch.equal(a.obs, b.obs) and torch.equal(a.rew, b.rew) \
                        and torch.equal(a.terminated, b.terminated) and torch.equal(a.truncated, b.truncated)
                same = same and torch.equal(r2.get_state(), e.get_state())
                r2.close()
            us = time_steps(e, acts, args.steps)
            res.setdefault(key, {})[name] = {"us": round(us, 2), "kernel": e.step_kernel_name, "bit_identical": same}
            print("%-18s %-10s %8.2f us  %-26s identical=%s" % (key, name, us, e.step_kernel_name, same), flush=True)
            e.close()
        ref.close()
        torch.cuda.empty_cache()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
