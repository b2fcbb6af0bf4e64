#!/usr/bin/env python3
"""A/B of the half-populated-wave windowed step (F16ENV_HALF=1, f16env.hip step_body HALF) against
the production windowed kernel, same box, same steady-state episode mix (put
a second wave on every SIMD at 65 536 envs).

HALF puts 32 envs in each wave (lanes 0-31), i.e. 2 048 waves = two per SIMD at 65 536 envs, in
the 256-register build; F16ENV_HALF_DELAY makes the second half of the grid start that many
shader cycles late, so a SIMD's two waves are out of phase (one's prologue / store tail beside the
other's frames). For each variant: kernel time from the launches' own dispatch events (mean and
min over `--launches`), the region time, and bit-identity of the observations / rewards / state
with the production kernel over `--check` steps from the same state.

    python tools/half_ab.py --json gpurun_out/half_ab.json [--delays 0,3000,6000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--stack", type=int, default=4)
    ap.add_argument("--delays", default="0,1500,3000,4500,6000,9000")
    ap.add_argument("--launches", type=int, default=300)
    ap.add_argument("--burn", type=int, default=400)
    ap.add_argument("--check", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import numpy as np
    import torch
    from f16_jsb_amd.abi import F16C_STEP
    from f16_jsb_amd.env import F16Envs

    dev = torch.device("cuda", 0)
    n = args.envs

    def make(half, delay):
        os.environ["F16ENV_HALF"] = "1" if half else "0"
        os.environ["F16ENV_HALF_DELAY"] = str(delay)
        e = F16Envs(n, stack_k=args.stack, seed=0, obs_layout="window", device=dev)
        os.environ.pop("F16ENV_HALF")
        os.environ.pop("F16ENV_HALF_DELAY")
        return e

    # one steady-state start (phase spread + burn-in), copied into every variant's handle
    base = make(False, 0)
    base.reset()
    s = base.get_state()
    s[:, F16C_STEP] = torch.as_tensor(np.random.default_rng(77).integers(0, 1200, n), dtype=torch.float64, device=dev)
    base.set_state(s)
    for t in range(args.burn):
        base.step(base.sample_actions(3000, t))
    state0, obs0 = base.get_state(), base.obs.clone()
    acts = [base.sample_actions(1000, t) for t in range(64)]
    torch.cuda.synchronize()

    def run(e):
        e.set_state(state0)
        e.set_obs(obs0)
        outs = []
        for t in range(args.check):
            o = e.step(acts[t % 64])
            outs.append((o.obs.clone(), o.rew.clone(), o.terminated.clone(), o.truncated.clone()))
        st = e.get_state()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for t in range(args.launches):
            e.step(acts[t % 64])
        ev1.record()
        torch.cuda.synchronize()
        region = ev0.elapsed_time(ev1) / args.launches
        avg, mn, _ = e.profile_kernel(lambda: [e.step(acts[t % 64]) for t in range(args.launches)], args.launches)
        return outs, st, {"kernel_ms": round(avg, 5), "kernel_min_ms": round(mn, 5), "region_ms": round(region, 5),
                          "kernel": e.step_kernel_name, "waves_per_simd": e.waves_per_simd}

    variants = [("production", False, 0)] + [("half_delay%d" % d, True, d) for d in map(int, args.delays.split(","))]
    ref_outs, ref_state = None, None
    res = {"envs": n, "stack_k": args.stack, "launches": args.launches, "rounds": []}
    for rnd in range(args.rounds):
        row = {}
        for name, half, delay in variants:
            e = make(half, delay)
            outs, st, tm = run(e)
            if ref_outs is None:
                ref_outs, ref_state = outs, st
            same = all(all(torch.equal(x, y) for x, y in zip(a, b)) for a, b in zip(outs, ref_outs)) \
                and torch.equal(st, ref_state)
            tm["bit_identical"] = bool(same)
            row[name] = tm
            print(rnd, name, tm, flush=True)
            e.close()
        res["rounds"].append(row)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
