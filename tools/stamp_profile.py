#!/usr/bin/env python3
"""Per-section cycle breakdown of f16_step_kernel from the diagnostic build (-DF16_STAMPS).
Run on the GPU box:  python tools/stamp_profile.py [--envs 65536] [--stack 4]
Builds f16_jsb_amd/libf16env_diag.so and loads it through F16ENV_LIB. The section SHARES
are meaningful; the diagnostic build's total time is not (stamps serialise the wave)."""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIAG = os.path.join(ROOT, "f16_jsb_amd", "libf16env_diag.so")
NAMES = ["load+stage", "propagate", "derive", "atmosphere", "fcs", "aux", "engine", "aero", "accel",
         "make_frame", "reward", "reset", "sync/compact", "obs copy", "state store", "earth angle + alt_ref (+gust)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--stack", type=int, default=4)
    ap.add_argument("--layout", default="window", choices=("window", "contiguous"))
    ap.add_argument("--build-only", action="store_true")
    args = ap.parse_args()
    src = os.path.join(ROOT, "f16_jsb_amd", "csrc")
    fresh = os.path.exists(DIAG) and all(os.path.getmtime(os.path.join(src, f)) <= os.path.getmtime(DIAG)
                                         for f in os.listdir(src))
    if not fresh:  # build here (CPU container) beforehand; the box then reuses it
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I",
                        os.path.join(ROOT, "include"), "-DF16_STAMPS", "-shared", "-fPIC", "-Wno-unused-value",
                        "-fno-slp-vectorize", os.path.join(src, "f16env.hip"), "-o", DIAG], check=True)
    if "--build-only" in sys.argv:
        return
    os.environ["F16ENV_LIB"] = DIAG
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    from f16_jsb_amd import _lib
    from f16_jsb_amd.env import F16Envs
    L = _lib.lib()
    L.f16env_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    e = F16Envs(args.envs, stack_k=args.stack, seed=1, obs_layout=args.layout)
    print("kernel", e.step_kernel_name)
    e.reset()
    for t in range(30):
        e.step(e.sample_actions(3, t))
    torch.cuda.synchronize()
    waves = args.envs // 64
    buf = np.zeros((waves, len(NAMES)), np.uint64)
    n = L.f16env_diag_stamps(buf.ctypes.data_as(ctypes.c_void_p), waves)
    assert n == len(NAMES), n
    per = buf.astype(np.float64)
    tot = per.sum(axis=1)
    print("waves %d, cycles per wave step: median %.0f (min %.0f max %.0f)" % (waves, np.median(tot), tot.min(), tot.max()))
    for i, nm in enumerate(NAMES):
        col = per[:, i]
        print("  %-14s %9.0f cycles  %5.1f%%" % (nm, np.median(col), 100 * np.median(col) / np.median(tot)))


if __name__ == "__main__":
    main()
