#!/usr/bin/env python3
"""Per-frame cost of the step kernel at one vs two waves per SIMD. Run on the GPU box:

    python tools/occ_probe.py [--json out.json]

For each occupancy build (F16ENV_OCC=1|2) and env count, times T(down_sample) at 0, 4 and 8
FDM frames per step; the slope (T8 - T4) / 4 is the cost of one frame for the whole launch.
At 131072 envs the one-wave build runs two rounds of waves, the two-wave build runs them
side by side on each SIMD: equal slopes mean the SIMD's VALU issue doubled with the second
wave, twice the slope means the frame is bound by something the two waves share.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    import torch
    from f16_jsb_amd.env import F16Envs
    from kernel_sweep import time_steps
    res = {}
    for occ in (1, 2):
        os.environ["F16ENV_OCC"] = str(occ)
        for n in (65536, 131072):
            row = {}
            for ds in (0, 4, 8):
                envs = F16Envs(n, stack_k=4, down_sample=ds, seed=1)
                envs.reset()
                acts = [envs.sample_actions(5, t) for t in range(16)]
                row[ds] = round(time_steps(envs, acts, args.steps), 2)
                envs.close()
                del envs
                torch.cuda.empty_cache()
            row["frame_us"] = round((row[8] - row[4]) / 4, 3)
            key = "occ%d_n%d" % (occ, n)
            res[key] = row
            print(key, row, flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
