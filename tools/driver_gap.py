#!/usr/bin/env python3
"""Where does the driver's short bench region lose time?

Replays bench.py's headline sequence (65 536 envs, K = 4, window layout, phase spread +
1 200-step burn-in, W warm-up steps, then K timed steps behind a sync) and times the
timed region several ways:

  region   -- bench.py's own measure: HIP events around K step() calls on the stream
  host     -- perf_counter after every step() call (host cost per call, no sync)
  kernels  -- each launch's dispatch-packet start/stop events (f16env_profile_times):
              kernel durations and the gaps between consecutive kernels
  busy     -- the same K steps issued while the stream is held by a 300 us spin kernel, so
              the host is far ahead when the first step starts: the GPU's back-to-back rate

    python tools/driver_gap.py [--steps 20] [--warmup 5] [--trials 5] [--json out.json]
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--trials", type=int, default=5)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import numpy as np
    import torch
    from bench import spread_phases
    from f16_jsb_amd.env import F16VecEnv

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = args.envs
    venv = F16VecEnv(num_envs=n, stack_k=4, device=dev, seed=0, return_numpy=False, obs_layout="window")
    e = venv.envs
    venv.reset()

    class A:
        seed, burn_in = 0, None
    spread_phases(e, A, dev)
    K = args.steps
    acts = torch.empty((K, n, 4), dtype=torch.float32, device=dev)
    for t in range(K):
        e.sample_actions(1000, t, out=acts[t])
    for t in range(args.warmup):
        e.step(e.sample_actions(2000, t))
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    res = {"envs": n, "steps": K, "warmup": args.warmup, "kernel": e.step_kernel_name, "trials": []}

    from f16_jsb_amd.abi import F16C_EP_COUNT

    def region(pre_spin_cycles=0, preface=None):
        s, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        if preface == "bench":  # bench.py's episode-counter read in front of its timed region
            e.get_state()[:, F16C_EP_COUNT].sum()
            torch.cuda.synchronize()
        elif preface == "bench_spin":  # ... then 2 ms of host busy-wait before the region
            e.get_state()[:, F16C_EP_COUNT].sum()
            torch.cuda.synchronize()
            tb = time.perf_counter()
            while time.perf_counter() - tb < 2e-3:
                pass
        elif preface == "torch_op":  # a small torch launch + sync first
            torch.zeros(1, device=dev).add_(1)
            torch.cuda.synchronize()
        elif preface == "gc":  # bench.py r03b: gc.collect() right before the region
            gc.collect()
        elif preface == "noop":  # one tiny launch after the sync, before t0 (host launch path warm)
            noop()
        elif preface == "gc_noop":
            gc.collect()
            noop()
        hs = []
        t0 = time.perf_counter()
        if pre_spin_cycles:
            torch.cuda._sleep(pre_spin_cycles)
        s.record(stream)
        for t in range(K):
            e.step(acts[t])
            hs.append(time.perf_counter())
        en.record(stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        host = np.diff(np.array([t0] + hs)) * 1e6
        return s.elapsed_time(en) * 1e3 / K, wall * 1e6 / K, host

    # the launch call alone inside step(): its host time on the region's first call
    real_bound = e._step_bound
    launch_us = []

    def timed_bound(*a):
        tb = time.perf_counter()
        r = real_bound(*a)
        launch_us.append((time.perf_counter() - tb) * 1e6)
        return r
    e._step_bound = timed_bound
    zero = torch.zeros(1, device=dev)

    def noop():
        zero.add_(0)
    variants = {}
    for pre in ("plain", "bench", "gc", "noop", "gc_noop", "bench_spin", "torch_op", "plain"):
        rs = []
        for tr in range(3):
            launch_us.clear()
            r_us, wall_us, host = region(preface=pre)
            rs.append((round(r_us, 3), round(wall_us, 3), round(float(host[0]), 2), round(launch_us[0], 2)))
        variants.setdefault(pre, []).extend(rs)
        print(pre, "(region us/step, wall us/step, first call us, its launch us)", rs, flush=True)
    e._step_bound = real_bound
    res["preface_variants"] = variants
    for tr in range(args.trials):
        r_us, wall_us, host = region()
        b_us, bwall_us, bhost = region(pre_spin_cycles=600000)  # ~250-300 us of spin first
        times = []
        torch.cuda.synchronize()
        e.profile_kernel(lambda: [e.step(acts[t]) for t in range(K)], K, times=times)
        ts = np.array(times)
        dur = (ts[:, 1] - ts[:, 0]) * 1e3
        gaps = (ts[1:, 0] - ts[:-1, 1]) * 1e3
        row = {"region_us_per_step": round(r_us, 3), "wall_us_per_step": round(wall_us, 3),
               "host_us_per_call": [round(float(x), 2) for x in host],
               "busy_region_us_per_step": round(b_us, 3), "busy_host_us_per_call_median": round(float(np.median(bhost)), 2),
               "kernel_us": [round(float(x), 2) for x in dur], "gap_us": [round(float(x), 2) for x in gaps],
               "span_us": round(float(ts[-1, 1] - ts[0, 0]) * 1e3, 2)}
        res["trials"].append(row)
        print(json.dumps({k: (v if not isinstance(v, list) else v[:8]) for k, v in row.items()}), flush=True)
    # host cost of the pieces of a step() call
    L = []
    from f16_jsb_amd._lib import lib
    lb = lib()
    N = 2000
    t0 = time.perf_counter()
    for _ in range(N):
        torch.cuda.current_stream(dev).cuda_stream
    L.append(("torch.cuda.current_stream().cuda_stream", (time.perf_counter() - t0) / N * 1e6))
    get_raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    if get_raw is not None:
        t0 = time.perf_counter()
        for _ in range(N):
            get_raw(0)
        L.append(("torch._C._cuda_getCurrentRawStream", (time.perf_counter() - t0) / N * 1e6))
    t0 = time.perf_counter()
    for _ in range(N):
        lb.f16env_step_mode(e._h)
    L.append(("ctypes call, 1 arg", (time.perf_counter() - t0) / N * 1e6))
    a0 = acts[0]
    t0 = time.perf_counter()
    for _ in range(N):
        (a0.device == e.device, a0.dtype, a0.is_contiguous(), a0.data_ptr(), a0.shape == (n, 4))
    L.append(("tensor checks", (time.perf_counter() - t0) / N * 1e6))
    res["host_pieces_us"] = {k: round(v, 3) for k, v in L}
    print(json.dumps(res["host_pieces_us"]), flush=True)
    try:
        with open("/proc/cpuinfo") as f:
            res["cpu_model"] = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
    except OSError:
        pass
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)
    venv.close()


if __name__ == "__main__":
    main()
