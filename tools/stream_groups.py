#!/usr/bin/env python3
"""Env groups on separate HIP streams: G handles of N/G envs each, every group stepped once
per iteration on its own stream (no cross-stream dependency inside the loop), vs one handle of
N envs. Measures whether groups whose memory phases drift apart finish N env steps sooner than
one lock-step launch. One process, one GPU:

    python tools/stream_groups.py [--envs 65536] [--steps 1000] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(n, groups, steps, stack=4, offset_steps=0):
    import torch
    from f16_jsb_amd.env import F16Envs
    m = n // groups
    streams = [torch.cuda.Stream() for _ in range(groups)]
    envs, acts = [], []
    for g in range(groups):
        with torch.cuda.stream(streams[g]):
            e = F16Envs(m, stack_k=stack, seed=1, env_id_base=g * m)
            e.reset()
            acts.append([e.sample_actions(5, t) for t in range(16)])
            envs.append(e)
    torch.cuda.synchronize()
    for t in range(20):
        for g in range(groups):
            with torch.cuda.stream(streams[g]):
                envs[g].step(acts[g][t % 16])
    torch.cuda.synchronize()
    # optional stagger: the first group runs ahead by offset_steps before the timed loop
    for t in range(offset_steps):
        with torch.cuda.stream(streams[0]):
            envs[0].step(acts[0][t % 16])
    t0 = time.perf_counter()
    for t in range(steps):
        for g in range(groups):
            with torch.cuda.stream(streams[g]):
                envs[g].step(acts[g][t % 16])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    for e in envs:
        e.close()
    return round(el / steps * 1e6, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    res = {}
    for groups, off in ((1, 0), (2, 0), (2, 1), (4, 0)):
        res["g%d_off%d_us_per_step" % (groups, off)] = run(a.envs, groups, a.steps, offset_steps=off)
        print(json.dumps(res), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
