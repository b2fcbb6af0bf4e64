#!/usr/bin/env python3
"""Cost of the in-kernel auto-reset at 65 536 envs: the same step with and without
F16_FLAG_NO_AUTORESET (finished lanes still write their terminal observation). Run on the GPU
box:  python tools/reset_cost.py"""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch
from f16_jsb_amd.env import F16Envs
from kernel_sweep import time_steps
res = {}
for auto in (True, False, True, False):
    e = F16Envs(65536, stack_k=4, seed=1, autoreset=auto)
    e.reset()
    acts = [e.sample_actions(5, t) for t in range(16)]
    us = time_steps(e, acts, 400)
    kern, kmin, _ = e.profile_kernel(lambda: [e.step(acts[t % 16]) for t in range(300)], 300)
    print("autoreset", auto, "region us/step %.2f  kernel avg %.2f min %.2f" % (us, kern * 1e3, kmin * 1e3), flush=True)
    e.close()
