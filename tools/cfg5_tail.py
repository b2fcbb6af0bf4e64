"""Diagnose the worst lanes of the cfg5 production parity run (131 072 envs, the two-wave
f16_step_var_kernel<3, 2> build) against the oracle: per-step error history of the worst lanes,
whether they were reset during the run, and the same lanes on the one-wave build
(F16ENV_OCC=1) and on a second handle of the two-wave build (determinism).

    python tools/cfg5_tail.py [--n 131072] [--steps 30] [--json out.json]

Test tooling: imports the oracle (tests/oracle_ref.py) as the checker.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle_ref import OracleEnvs  # noqa: E402
from parity_tools import FRAME_NAMES, frame_err  # noqa: E402

from f16_jsb_amd.abi import F16C_STEP  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=131072)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--seed", type=int, default=41)
    ap.add_argument("--aseed", type=int, default=23)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import torch
    from f16_jsb_amd.env import F16Envs

    n = a.n
    ref = OracleEnvs(n, stack_k=4, seed=a.seed, cfg5=True)
    handles = {}
    for name, occ in (("occ2", None), ("occ2b", None), ("occ1", "1")):
        if occ:
            os.environ["F16ENV_OCC"] = occ
        else:
            os.environ.pop("F16ENV_OCC", None)
        handles[name] = F16Envs(n, stack_k=4, seed=a.seed, cfg5=True)
    os.environ.pop("F16ENV_OCC", None)
    print({k: h.step_kernel_name for k, h in handles.items()})
    o = ref.reset()
    for h in handles.values():
        h.reset()
    s = ref.get_state()
    k = np.arange(n)
    sel = k % 3 == 0
    s[sel, F16C_STEP] = ref.cfg.max_steps - 1 - (k[sel] // 3) % 30
    ref.set_state(s)
    for h in handles.values():
        h.set_state(s)
        h.set_obs(torch.as_tensor(o))
    hist = {name: np.zeros((a.steps, n, 15), np.float32) for name in handles}
    hist_r = np.zeros((a.steps, n, 15), np.float32)
    done_any = np.zeros(n, bool)
    for t in range(1, a.steps + 1):
        act = ref.sample_actions(a.aseed, t)
        o_r, r_r, te_r, tr_r, *_ = ref.step(act)
        done_any |= te_r | tr_r
        hist_r[t - 1] = o_r[:, -1]
        for name, h in handles.items():
            out = h.step(h.sample_actions(a.aseed, t))
            hist[name][t - 1] = out.obs[:, -1].cpu().numpy()
    res = {"kernels": {k: h.step_kernel_name for k, h in handles.items()}}
    res["occ2_deterministic"] = bool(np.array_equal(hist["occ2"], hist["occ2b"]))
    res["occ2_vs_occ1_bit_identical"] = bool(np.array_equal(hist["occ2"], hist["occ1"]))
    for name in ("occ2", "occ1"):
        err = frame_err(hist[name], hist_r)  # (T, N, 15)
        fin = err[-1]
        summ = {}
        for c in range(12):
            order = np.argsort(fin[:, c])[::-1][:5]
            summ[FRAME_NAMES[c]] = {
                "max": float(fin[:, c].max()),
                "p999": float(np.percentile(fin[:, c], 99.9)),
                "worst": [{"lane": int(l), "reset_in_run": bool(done_any[l]),
                           "err_t1_3_10_20_30": [float(err[i, l, c]) for i in (0, 2, 9, 19, a.steps - 1)],
                           "h_m": float(hist_r[-1, l, 2]), "mach": float(hist_r[-1, l, 3])} for l in order[:3]],
            }
        res[name] = summ
    d = frame_err(hist["occ2"][-1], hist["occ1"][-1])
    res["occ2_vs_occ1_max"] = {FRAME_NAMES[c]: float(d[:, c].max()) for c in range(12)}
    print(json.dumps(res, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
