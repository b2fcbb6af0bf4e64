#!/usr/bin/env python3
"""The step kernel's own floors beside tools/probes/floors, same box:
the windowed step at 65 536 envs, K = 4, in the bench's steady state (phase spread + burn-in),
with its 4 FDM frames (the headline) and with none (down_sample = 0: load, env layer, stores),
per-launch dispatch-event durations over `--launches` steps. Prints one JSON line.
    python tools/floors_step.py [--envs 65536] [--launches 300] [--json out.json]"""
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
    ap.add_argument("--launches", type=int, default=300)
    ap.add_argument("--burn-in", type=int, default=300)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import numpy as np
    import torch
    from f16_jsb_amd.abi import F16C_STEP
    from f16_jsb_amd.env import F16Envs
    dev = torch.device("cuda", 0)
    res = {"envs": args.envs, "stack_k": args.stack, "launches": args.launches}
    for ds in (4, 0, 1, 2):
        e = F16Envs(args.envs, stack_k=args.stack, seed=0, obs_layout="window", down_sample=ds)
        e.reset()
        s = e.get_state()
        s[:, F16C_STEP] = torch.as_tensor(np.random.default_rng(77).integers(0, 1200, args.envs), dtype=torch.float64,
                                          device=dev)
        e.set_state(s)
        acts = [e.sample_actions(1000, t) for t in range(16)]
        for t in range(args.burn_in):
            e.step(acts[t % 16])
        torch.cuda.synchronize()
        st = torch.cuda.current_stream(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for t in range(args.launches):
            e.step(acts[t % 16])
        b.record(st)
        torch.cuda.synchronize()
        region = a.elapsed_time(b) / args.launches
        avg, mn, _ = e.profile_kernel(lambda: [e.step(acts[t % 16]) for t in range(args.launches)], args.launches)
        res["down_sample_%d" % ds] = {"kernel": e.step_kernel_name, "kernel_us": round(avg * 1e3, 3),
                                      "kernel_min_us": round(mn * 1e3, 3), "region_us_per_launch": round(region * 1e3, 3)}
        e.close()
    line = json.dumps(res)
    print(line, flush=True)
    if args.json:
        with open(args.json, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
