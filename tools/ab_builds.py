#!/usr/bin/env python3
"""Same-box A/B of step-kernel builds: bit identity and time, each library in its own process
(F16ENV_LIB), interleaved A B A B so clock drift hits every build alike.

    python tools/ab_builds.py build NAME [-DFLAG ...]   # here: f16_jsb_amd/libf16env_ab_NAME.so
    python tools/ab_builds.py run [--rounds 2] [--json out.json] [--dump-dir gpurun_out/ab]

Per library and round: the bench headline's workload (65 536 envs, K = 4, windowed layout,
steady-state episode mix: phase spread + 300 burn-in steps), then 300 timed steps: the step
kernel's dispatch-event mean and min (profile_kernel) and the HIP-event region per launch;
cfg5's 131 072 envs likewise (fewer steps). The state, observation, rewards and flags after a
fixed 64-step sequence (with auto-resets) are hashed: builds that must round alike must hash
alike (sha256 of the raw bytes)."""
from __future__ import annotations

import glob
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PAT = os.path.join(ROOT, "f16_jsb_amd", "libf16env_ab_%s.so")


def build(name, flags):
    from f16_jsb_amd.build import build as b
    out = PAT % name
    b(force=True, extra=tuple(flags), out=out)  # (the product library is left alone)
    print("built", out, flags)


def run_one(cases):
    import argparse
    import numpy as np
    import torch
    from bench import spread_phases
    from f16_jsb_amd.env import F16Envs
    res = {}
    for name, n, cfg5, steps, *opt in cases:
        inkernel = bool(opt and opt[0])  # F16Envs.step(None, seed=, step=): in-kernel actions (winx build)
        e = F16Envs(n, stack_k=4, seed=1, obs_layout="window", cfg5=cfg5)
        e.reset()
        spread_phases(e, argparse.Namespace(seed=0, burn_in=300), e.device)
        acts = [e.sample_actions(5, t) for t in range(16)]
        if inkernel:
            class _InKernel:  # the same draws as acts, made by the step kernel itself
                def __getitem__(self, t):
                    return t
            acts, plain_step = _InKernel(), e.step
            e.step = lambda t: plain_step(None, seed=5, step=t)
        h = hashlib.sha256()
        for t in range(64):
            o = e.step(acts[t % 16])
        torch.cuda.synchronize()
        for x in (e.get_state(), o.obs.contiguous(), o.rew, o.terminated, o.truncated):
            h.update(x.detach().cpu().numpy().tobytes())
        st = torch.cuda.current_stream()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for t in range(steps):
            e.step(acts[t % 16])
        b.record(st)
        torch.cuda.synchronize()
        region = a.elapsed_time(b) / steps
        if inkernel:  # (the dispatch-event profile instruments the plain launch only)
            avg = mn = region
        else:
            avg, mn, _ = e.profile_kernel(lambda: [e.step(acts[t % 16]) for t in range(steps)], steps)
        res[name] = {"kernel": "winx (in-kernel actions)" if inkernel else e.step_kernel_name,
                     "kernel_us": round(avg * 1e3, 3), "kernel_min_us": round(mn * 1e3, 3),
                     "region_us": round(region * 1e3, 3), "sha256": h.hexdigest()[:16]}
        e.close()
    print(json.dumps(res), flush=True)


CASES = [("cfg3_65536", 65536, False, 300), ("cfg5_131072", 131072, True, 200),
         ("cfg3_inkernel_actions", 65536, False, 300, True)]


def run(rounds, json_out):
    libs = [("base", os.path.join(ROOT, "f16_jsb_amd", "libf16env.so"))]
    libs += [(os.path.basename(p)[len("libf16env_ab_"):-3], p) for p in sorted(glob.glob(PAT % "*"))]
    out = {name: [] for name, _ in libs}
    for r in range(rounds):
        for name, lib in libs:
            env = dict(os.environ, F16ENV_LIB=lib)
            p = subprocess.run([sys.executable, __file__, "one"], env=env, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(name, "FAILED rc", p.returncode, p.stderr[-2000:], flush=True)
                if p.returncode < 0 or p.returncode in (134, 139):
                    return
                continue
            d = json.loads(p.stdout.strip().splitlines()[-1])
            out[name].append(d)
            print("round %d %-14s %s" % (r, name, json.dumps(d)), flush=True)
    summary = {}
    for name, runs in out.items():
        if not runs:
            continue
        s = {}
        for case in runs[0]:
            s[case] = {"kernel": runs[0][case]["kernel"], "sha256": sorted({x[case]["sha256"] for x in runs}),
                       "kernel_us": [x[case]["kernel_us"] for x in runs], "region_us": [x[case]["region_us"] for x in runs],
                       "kernel_us_best": min(x[case]["kernel_us"] for x in runs)}
        summary[name] = s
    base = summary.get("base", {})
    for name, s in summary.items():
        for case, v in s.items():
            b = base.get(case)
            if b is not None:
                v["bit_identical_to_base"] = v["sha256"] == b["sha256"]
                v["kernel_us_best_delta_vs_base"] = round(v["kernel_us_best"] - b["kernel_us_best"], 3)
    print(json.dumps(summary, indent=1), flush=True)
    if json_out:
        with open(json_out, "w") as f:
            json.dump({"runs": out, "summary": summary}, f, indent=1)


if __name__ == "__main__":
    cmd = sys.argv[1]
    if cmd == "build":
        build(sys.argv[2], sys.argv[3:])
    elif cmd == "one":
        run_one(CASES)
    else:
        rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 2
        run(rounds, sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None)
