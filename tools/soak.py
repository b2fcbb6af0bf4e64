#!/usr/bin/env python3
"""Soak run of the bench's own configurations: many thousands of steps at BASELINE sizes,
window restarts and reset-cache refills included, with the NaN guard and the observation-bounds
diagnostic on; with F16ENV_LIB pointing at libf16env_debug.so the kernels also record every
index / range invariant they find violated (f16env_debug_checks). Prints one JSON line.

    python tools/soak.py [--steps3 N] [--steps5 N]
    F16ENV_LIB=f16_jsb_amd/libf16env_debug.so python tools/soak.py ...
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def soak(n, steps, cfg5, seed):
    import torch
    from bench import spread_phases
    from f16_jsb_amd._lib import lib
    from f16_jsb_amd.abi import F16C_EP_COUNT
    from f16_jsb_amd.env import F16Envs

    e = F16Envs(n, stack_k=4, seed=seed, obs_layout="window", cfg5=cfg5, nan_guard=True, obs_check=True)
    e.reset()
    spread_phases(e, argparse.Namespace(seed=seed, burn_in=None), e.device)
    ep0 = float(e.get_state()[:, F16C_EP_COUNT].sum())
    a = torch.empty((n, 4), dtype=torch.float32, device=e.device)
    t0 = time.time()
    for t in range(steps):
        e.sample_actions(seed + 11, t, out=a)
        out = e.step(a)
    torch.cuda.synchronize()
    wall = time.time() - t0
    finite = bool(torch.isfinite(out.obs).all())
    resets = float(e.get_state()[:, F16C_EP_COUNT].sum()) - ep0
    v = ctypes.c_uint32()
    is_debug = lib().f16env_debug_checks(e._h, None, ctypes.byref(v))
    r = {"envs": n, "steps": steps, "cfg5": cfg5, "kernel": e.step_kernel_name, "auto_resets": int(resets),
         "nonfinite_quarantined": e.nonfinite_count, "obs_out_of_bounds": e.obs_bounds_count,
         "final_obs_finite": finite, "debug_build": bool(is_debug), "violations": int(v.value),
         "wall_s": round(wall, 2)}
    e.close()
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps3", type=int, default=20000)
    ap.add_argument("--steps5", type=int, default=10000)
    a = ap.parse_args()
    res = [soak(65536, a.steps3, False, 1), soak(131072, a.steps5, True, 2)]
    print(json.dumps({"lib": os.environ.get("F16ENV_LIB", "f16_jsb_amd/libf16env.so"), "runs": res}), flush=True)


if __name__ == "__main__":
    main()
