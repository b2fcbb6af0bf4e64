#!/usr/bin/env python3
"""A/B timing of step-kernel build variants (-D flags), each in its own process through
F16ENV_LIB. Build here (cross-compile), run on the GPU box:

    python tools/variant_sweep.py build NAME=-DFLAG[,-DFLAG2] ...
    python tools/variant_sweep.py run [--json out.json]
"""
from __future__ import annotations

import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PAT = os.path.join(ROOT, "f16_jsb_amd", "libf16env_var_%s.so")
CASES = [(65536, 4, 4), (65536, 4, 0), (131072, 4, 4), (262144, 4, 4), (65536, 10, 4), (4096, 4, 4)]
# the same cases in the windowed observation layout (the bench headline's)
WCASES = [(65536, 4, 4), (65536, 4, 0), (131072, 4, 4), (262144, 4, 4), (4096, 4, 4)]
# cfg5 mode (random ICs + gusts: MODE 3 kernels), window layout
C5CASES = [(131072, 4, 4), (65536, 4, 4)]
# the bench headline's steady-state episode mix (bench.spread_phases: phase spread + burn-in),
# window layout -- what a change must not lose (fresh episodes have no auto-resets)
SCASES = [(65536, 4, 4)]


def build(specs):
    from f16_jsb_amd.build import OUT, build as b
    for spec in specs:
        name, _, flags = spec.partition("=")
        extra = [f for f in flags.split(",") if f]
        out = PAT % name
        b(force=True, extra=extra)
        os.replace(OUT, out)
        print("built", out, extra)
    b(force=True)


def run_one():
    import torch
    from f16_jsb_amd.env import F16Envs
    res = {}
    runs = ([("c", *c) for c in CASES] + [("w", *c) for c in WCASES] + [("w5", *c) for c in C5CASES]
            + [("ws", *c) for c in SCASES])
    for lay, n, k, ds in runs:
        e = F16Envs(n, stack_k=k, down_sample=ds, seed=1, obs_layout="contiguous" if lay == "c" else "window",
                    cfg5=lay == "w5")
        e.reset()
        if lay == "ws":
            import argparse
            from bench import spread_phases
            spread_phases(e, argparse.Namespace(seed=0, burn_in=None), e.device)
        acts = [e.sample_actions(5, t) for t in range(16)]
        for t in range(20):
            e.step(acts[t % 16])
        torch.cuda.synchronize()
        s, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for t in range(300):
            e.step(acts[t % 16])
        en.record()
        torch.cuda.synchronize()
        res[("" if lay == "c" else lay + "_") + "n%d_k%d_ds%d" % (n, k, ds)] = round(s.elapsed_time(en) / 300 * 1e3, 2)
        e.close()
    print(json.dumps(res))


def run(json_out):
    out = {}
    libs = sorted(glob.glob(PAT % "*"))
    for lib in [os.path.join(ROOT, "f16_jsb_amd", "libf16env.so")] + libs:
        name = "baseline" if lib.endswith("libf16env.so") else os.path.basename(lib)[len("libf16env_var_"):-3]
        env = dict(os.environ, F16ENV_LIB=lib)
        r = subprocess.run([sys.executable, __file__, "one"], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(name, "FAILED rc", r.returncode, r.stderr[-2000:], flush=True)
            if r.returncode < 0 or r.returncode in (134, 139):
                break
            continue
        out[name] = json.loads(r.stdout.strip().splitlines()[-1])
        print("%-16s %s" % (name, out[name]), flush=True)
    if json_out:
        with open(json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    cmd = sys.argv[1]
    if cmd == "build":
        build(sys.argv[2:])
    elif cmd == "one":
        run_one()
    else:
        run(sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None)
