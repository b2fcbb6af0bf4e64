#!/usr/bin/env python3
"""Step time vs env count at down_sample 0 (no FDM frames: prologue + stack rebuild + stores)
and 4 (the reference's step): is a memory phase bound by bytes (time ~ N) or by per-wave
latency (time flat in N while waves <= SIMDs)? Run on the GPU box: python tools/size_sweep.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import torch
    from f16_jsb_amd.env import F16Envs
    from kernel_sweep import time_steps
    res = {}
    for ds in (0, 4):
        for n in (4096, 16384, 32768, 49152, 65536):
            e = F16Envs(n, stack_k=4, down_sample=ds, seed=1)
            e.reset()
            acts = [e.sample_actions(5, t) for t in range(16)]
            us = time_steps(e, acts, 300)
            res["n%d_ds%d" % (n, ds)] = round(us, 2)
            print("n %6d ds %d  %7.2f us/step" % (n, ds, us), flush=True)
            e.close()
            torch.cuda.empty_cache()
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
