"""BASELINE cfg5 divergence report: fp32 HIP kernel vs fp64 CPU oracle under randomised
initial conditions and wind gusts (F16_FLAG_RANDOM_IC | F16_FLAG_GUSTS), random actions.

    python tests/cfg5_divergence.py [--n 4096] [--steps 1200] [--json out.json]

The GPU runs the same global env ids, seed and Philox action stream as the oracle (both
draw their own random ICs and gusts: the IC difference is the fp32-vs-fp64 RunIC, so the
report starts at the IC). No auto-reset: a lane leaves the comparison when either side ends
its episode. Per horizon and frame component: percentiles (50/90/99/max) of |gpu - oracle|
over lanes alive on both sides, plus the done-flag agreement. Test infrastructure (imports
the oracle); the committed summary lives in profiles/.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle_ref import OracleEnvs  # noqa: E402
from parity_tools import FRAME_NAMES, frame_err  # noqa: E402

from f16_jsb_amd.abi import F16_FLAG_NO_AUTORESET  # noqa: E402

HORIZONS = (0, 1, 3, 10, 30, 100, 300, 600, 1000, 1199)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=1199)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--json", default=None)
    ap.add_argument("--obs-layout", default="window", choices=("window", "contiguous"),
                    help="the GPU handle's layout (window: the bench's cfg5 kernels)")
    args = ap.parse_args()
    import torch
    from f16_jsb_amd.build import build
    from f16_jsb_amd.env import F16Envs

    build()
    n, K = args.n, 4
    kw = dict(stack_k=K, seed=args.seed, cfg5=True, flags=F16_FLAG_NO_AUTORESET)
    ref = OracleEnvs(n, **kw)
    g = F16Envs(n, obs_layout=args.obs_layout, **kw)
    o_r = ref.reset()
    o_g = g.reset().cpu().numpy()
    alive = np.ones(n, bool)
    done_mismatch = 0  # read by record() at each horizon
    first_mismatch = None
    rows = []
    t0 = time.time()

    def record(t):
        if not alive.any():
            return
        e = frame_err(o_g[alive, -1], o_r[alive, -1])[:, :12]
        pct = np.percentile(e, [50, 90, 99, 100], axis=0)
        rows.append({"step": t, "alive": int(alive.sum()), "done_mismatches_so_far": done_mismatch,
                     **{"%s:p%s" % (FRAME_NAMES[c], q): float(pct[i, c])
                        for c in range(12) for i, q in enumerate(("50", "90", "99", "max"))}})

    record(0)
    for t in range(1, args.steps + 1):
        a = ref.sample_actions(args.seed + 1, t)
        o_r, _, te_r, tr_r, *_ = ref.step(a)
        out = g.step(g.sample_actions(args.seed + 1, t))
        o_g = out.obs.cpu().numpy()
        d_g = (out.terminated | out.truncated).cpu().numpy().astype(bool)
        d_r = te_r | tr_r
        mm = int((alive & (d_g != d_r)).sum())
        if mm and first_mismatch is None:
            first_mismatch = t
        done_mismatch += mm
        alive &= ~(d_g | d_r)
        if t in HORIZONS:
            record(t)
            print("step %5d alive %5d  h_m p99 %.3e  alpha p99 %.3e  (%.0f s)" % (
                t, alive.sum(), rows[-1]["h_m:p99"] if rows else -1, rows[-1]["alpha:p99"] if rows else -1,
                time.time() - t0), flush=True)
    res = {"n_envs": n, "stack_k": K, "seed": args.seed, "steps": args.steps,
           "obs_layout": args.obs_layout, "kernel": g.step_kernel_name,
           "model": "cfg5: random IC box + Gauss-Markov gusts (include/f16env.h), random actions (Philox)",
           "done_flag_mismatches_while_alive": done_mismatch, "first_done_mismatch_step": first_mismatch,
           "horizons": rows}
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "horizons"}))


if __name__ == "__main__":
    main()
