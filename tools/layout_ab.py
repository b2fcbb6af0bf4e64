#!/usr/bin/env python3
"""A/B of the observation layouts on the GPU box: ping-pong contiguous stacks (f16env_step) vs
windowed histories (f16env_step_window), µs per env step over 300 back-to-back steps (HIP events
on the launch stream), same handle config, same 16 reused action batches.

    python tools/layout_ab.py [--json out.json]
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CASES = [(65536, 4), (65536, 10), (131072, 4), (262144, 4), (4096, 4)]


def time_case(n, k, layout, steps=300, history=0):
    import torch
    from f16_jsb_amd.env import F16Envs
    e = F16Envs(n, stack_k=k, seed=1, obs_layout=layout, history=history)
    e.reset()
    acts = [e.sample_actions(5, t) for t in range(16)]
    for t in range(30):
        e.step(acts[t % 16])
    torch.cuda.synchronize()
    s, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for t in range(steps):
        e.step(acts[t % 16])
    en.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(en) / steps * 1e3
    name = e.step_kernel_name
    e.close()
    return round(us, 2), name


def main():
    out = {}
    hist = [int(x) for x in os.environ.get("F16_AB_HISTORY", "0").split(",")]
    for n, k in CASES:
        for layout, T in [("contiguous", 0)] + [("window", h) for h in hist]:
            if T and T < 2 * k:
                continue
            us, name = time_case(n, k, layout, history=T)
            key = "n%d_k%d_%s" % (n, k, layout) + ("_T%d" % T if T else "")
            out[key] = {"us_per_step": us, "kernel": name}
            print("n=%-7d K=%-2d %-10s T=%-4d %7.2f us  %s" % (n, k, layout, T, us, name), flush=True)
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
