#!/usr/bin/env python3
"""Decompose f16_step_kernel time: T(down_sample) = T_env + down_sample * T_frame, and its
dependence on the env count and stack depth. Run on the GPU box:

    python tools/kernel_sweep.py [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def time_steps(envs, acts, steps):
    import torch
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for t in range(10):
        envs.step(acts[t % len(acts)])
    torch.cuda.synchronize()
    s.record()
    for t in range(steps):
        envs.step(acts[t % len(acts)])
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / steps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    import torch
    from f16_jsb_amd.build import build
    from f16_jsb_amd.env import F16Envs
    build()
    res = {}
    for n, k, ds in [(65536, 4, 0), (65536, 4, 1), (65536, 4, 2), (65536, 4, 4), (65536, 4, 8),
                     (65536, 10, 4), (65536, 1, 4), (131072, 4, 4), (262144, 4, 4), (16384, 4, 4),
                     (32768, 4, 4)]:
        envs = F16Envs(n, stack_k=k, down_sample=ds, seed=1)
        envs.reset()
        acts = [envs.sample_actions(5, t) for t in range(16)]
        us = time_steps(envs, acts, args.steps)
        key = "n%d_k%d_ds%d" % (n, k, ds)
        res[key] = round(us, 2)
        print("%-22s %9.2f us/step  %8.3f ns/env-step" % (key, us, us * 1e3 / n), flush=True)
        envs.close()
        del envs
        torch.cuda.empty_cache()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
