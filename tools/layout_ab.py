#!/usr/bin/env python3
"""A/B of the observation layouts on the GPU box: ping-pong contiguous stacks (f16env_step) vs
windowed histories (f16env_step_window), µs per env step over 300 back-to-back steps (HIP events
on the launch stream), same handle config, same 16 reused action batches.

    F16_AB_HISTORY=124,128 F16_AB_ORDERS=position,env F16_AB_DS=4,0 python tools/layout_ab.py [--json out.json]
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CASES = [(65536, 4), (65536, 10), (131072, 4), (262144, 4), (4096, 4)]


def time_case(n, k, layout, steps=300, history=0, order="position", ds=4):
    import torch
    from f16_jsb_amd.env import F16Envs
    kw = dict(history=history, window_order=order) if layout == "window" else {}
    e = F16Envs(n, stack_k=k, seed=1, obs_layout=layout, down_sample=ds, **kw)
    e.reset()
    if os.environ.get("F16_AB_SPREAD"):  # bench.py's steady-state episode mix (phase spread + burn-in)
        import argparse
        from bench import spread_phases
        spread_phases(e, argparse.Namespace(seed=0, burn_in=None), e.device)
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
    orders = os.environ.get("F16_AB_ORDERS", "position").split(",")
    ds_list = [int(x) for x in os.environ.get("F16_AB_DS", "4").split(",")]
    for ds in ds_list:
        for n, k in CASES:
            runs = [("contiguous", 0, "-")] + [("window", h, o) for o in orders for h in hist]
            for layout, T, order in runs:
                if T and T < 2 * k:
                    continue
                us, name = time_case(n, k, layout, history=T, order=order if layout == "window" else "position", ds=ds)
                key = "n%d_k%d_ds%d_%s" % (n, k, ds, layout) + ("_%s_T%d" % (order, T) if layout == "window" else "")
                out[key] = {"us_per_step": us, "kernel": name}
                print("n=%-7d K=%-2d ds=%d %-10s %-8s T=%-4d %7.2f us  %s" % (n, k, ds, layout, order, T, us, name),
                      flush=True)
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
