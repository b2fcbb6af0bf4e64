#!/usr/bin/env python3
"""Latency of the cfg5 per-lane RunIC reset (f16_reset_kernel with a mask of `--lanes` lanes on
a cfg5 handle, the work f16_reset_done_kernel does for a step's finished lanes), HIP events,
median of 50 calls. Run on the GPU box; F16ENV_LIB selects a diagnostic build.

    python tools/reset_time.py [--envs 131072] [--lanes 112]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=131072)
    ap.add_argument("--lanes", type=int, default=112)
    a = ap.parse_args()
    import torch
    from f16_jsb_amd.env import F16Envs
    e = F16Envs(a.envs, stack_k=4, seed=3, cfg5=True, obs_layout="window")
    e.reset()
    g = torch.Generator().manual_seed(0)
    ts = []
    s, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(60):
        m = torch.zeros(a.envs, dtype=torch.uint8)
        m[torch.randperm(a.envs, generator=g)[:a.lanes]] = 1
        m = m.cuda()
        torch.cuda.synchronize()
        s.record()
        e.reset(mask=m)
        en.record()
        torch.cuda.synchronize()
        if i >= 10:
            ts.append(s.elapsed_time(en) * 1e3)
    ts.sort()
    print(json.dumps({"envs": a.envs, "lanes": a.lanes, "reset_us_median": round(ts[len(ts) // 2], 2),
                      "reset_us_min": round(ts[0], 2)}))


if __name__ == "__main__":
    main()
