"""The fp64 oracle against itself: how fast does a perturbation at fp32 storage precision grow
on the reference task under random actions? (BASELINE.json north_star:
"state trajectories match ... within a stated fp32 tolerance".)

TEST INFRASTRUCTURE (runs the CPU oracle only): the envelope the HIP-vs-oracle divergence is
judged against (tests/test_gpu_fp32_envelope.py).

    python tests/fp32_envelope.py [--n 256] [--steps 1199] [--json profiles/r06_fp32_envelope.json]

The workload is tests/parity_report.py's random-action trajectories: OracleEnvs(n, K=4,
seed=5), goals default_rng(0) uniform over [-5000, 5000]^2 x [1000, 4000] m, actions
sample_actions(99, t) (the same Philox stream the HIP path draws), the reference IC
(jsbsim_gym.py:166-170). Runs, every one bit-deterministic:

  ref      the oracle as it runs (the trajectory the HIP path is compared with);
  control  its state passed through get_state / set_state at every step and nothing else
           (set_state recomputes the Earth angle from its cosine / sine): what the mechanism
           of the `round` variant costs by itself;
  round1   the state's fp32-stored fields rounded to fp32 once, after the reset (the HIP
           kernel's storage: f16_device.h keeps the ECI position / velocity and the Earth
           angle in fp64, everything else -- attitude, rates, AB histories as velocity deltas,
           FCS, engine, latch -- in fp32);
  ulp1     the same fields moved by one fp32 ulp once (random sign per field and lane);
  round    the fp32-stored fields rounded to fp32 after EVERY step (fp32 storage, fp64
           arithmetic: the part of the kernel's error that storage alone causes);
  hip      (with --gpu / run(hip=True)) the HIP path, F16Envs with the same seed, goals and
           in-kernel-identical Philox actions: the divergence the envelope is for.

Per variant and horizon: p50 / p99 / max over the lanes still running on both sides of
|variant - ref| per frame component (angles wrapped), plus the lane count. A lane leaves the
comparison at its first done on either side (as parity_report.py)."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from f16_jsb_amd.abi import (F16C_AI, F16C_AIP, F16C_BA, F16C_GUST, F16C_LX, F16C_Q,  # noqa: E402
                             F16C_TEF, F16C_VI, F16C_VIH1, F16C_VIH2, F16C_WI, F16C_WID, F16C_WIND, F16L_N)
from parity_tools import FRAME_NAMES, frame_err  # noqa: E402

HORIZONS = (1, 3, 10, 30, 100, 300, 1199)
VARIANTS = ("control", "round1", "ulp1", "round")
# fields the HIP kernel holds in fp32: attitude, rates and their derivatives, the
# AB2 acceleration history, FCS actuators + PID states, engine, the auxiliary latch
F32_FIELDS = np.r_[F16C_AI:F16C_AI + 3, F16C_AIP:F16C_AIP + 3, F16C_Q:F16C_Q + 4, F16C_WI:F16C_WI + 3,
                   F16C_WID:F16C_WID + 3, F16C_BA:F16C_BA + 3, F16C_TEF:F16C_LX + F16L_N,
                   F16C_WIND:F16C_GUST + 3]  # (cfg5: steady wind and gust, fp32 columns of the wind kernels)


def workload(n):
    rng = np.random.default_rng(0)
    goals = rng.uniform([-5000, -5000, 1000], [5000, 5000, 4000], size=(n, 3)).astype(np.float32)
    return goals


def to_f32_storage(s):
    """The canonical state as the kernel stores it: fp32 fields rounded; the AB3 velocity
    history kept as fp32 deltas from the fp64 velocity (vI - vIh1, vIh1 - vIh2)."""
    s = s.copy()
    s[:, F32_FIELDS] = s[:, F32_FIELDS].astype(np.float32).astype(np.float64)
    vi, h1, h2 = s[:, F16C_VI:F16C_VI + 3], s[:, F16C_VIH1:F16C_VIH1 + 3], s[:, F16C_VIH2:F16C_VIH2 + 3]
    d1 = (vi - h1).astype(np.float32).astype(np.float64)
    d2 = (h1 - h2).astype(np.float32).astype(np.float64)
    s[:, F16C_VIH1:F16C_VIH1 + 3] = vi - d1
    s[:, F16C_VIH2:F16C_VIH2 + 3] = vi - d1 - d2
    return s


def one_ulp(s, rng):
    """Every fp32-stored field moved by one fp32 ulp (random sign)."""
    s = s.copy()
    f = s[:, F32_FIELDS].astype(np.float32)
    sign = rng.choice([-1.0, 1.0], size=f.shape)
    up = np.nextafter(f, np.float32(np.inf))
    dn = np.nextafter(f, np.float32(-np.inf))
    s[:, F32_FIELDS] = np.where(sign > 0, up, dn).astype(np.float64)
    return s


def run(n=256, steps=1199, horizons=HORIZONS, variants=VARIANTS, seed=5, act_seed=99, hip=False, cfg5=False):
    """{variant: {horizon: {"lanes": m, component: [p50, p99, max]}}} -- see the module doc.
    cfg5: BASELINE cfg5's randomised ICs + Gauss-Markov gusts (the same goals)."""
    from oracle_ref import OracleEnvs
    goals = workload(n)
    envs = {"ref": OracleEnvs(n, stack_k=4, seed=seed, cfg5=cfg5)}
    for v in variants:
        envs[v] = OracleEnvs(n, stack_k=4, seed=seed, cfg5=cfg5)
    for e in envs.values():
        e.reset(goals=goals)
    g = None
    if hip:
        import torch
        from f16_jsb_amd.env import F16Envs
        g = F16Envs(n, stack_k=4, seed=seed, obs_layout="window", cfg5=cfg5)
        g.reset(goals=torch.as_tensor(goals))
        variants = tuple(variants) + ("hip",)
    rng = np.random.default_rng(1234)
    if "round1" in envs:
        envs["round1"].set_state(to_f32_storage(envs["round1"].get_state()))
    if "ulp1" in envs:
        envs["ulp1"].set_state(one_ulp(envs["ulp1"].get_state(), rng))
    alive = {v: np.ones(n, bool) for v in variants}
    out = {v: {} for v in variants}
    hz = set(horizons)
    for t in range(1, steps + 1):
        a = envs["ref"].sample_actions(act_seed, t)
        res = {}
        for name, e in envs.items():
            if name in ("control", "round"):
                s = e.get_state()
                e.set_state(to_f32_storage(s) if name == "round" else s)
            o, _, te, tr, *_ = e.step(a)
            res[name] = (o[:, -1], te | tr)
        if g is not None:
            out_g = g.step(g.sample_actions(act_seed, t))
            res["hip"] = (out_g.obs[:, -1].cpu().numpy(),
                          (out_g.terminated.cpu().numpy() != 0) | (out_g.truncated.cpu().numpy() != 0))
        for v in variants:
            alive[v] &= ~(res["ref"][1] | res[v][1])
            if t in hz and alive[v].any():
                err = frame_err(res[v][0][alive[v]], res["ref"][0][alive[v]])
                d = {"lanes": int(alive[v].sum())}
                for c, nm in enumerate(FRAME_NAMES[:12]):
                    col = err[:, c]
                    d[nm] = [float(np.percentile(col, 50)), float(np.percentile(col, 99)), float(col.max())]
                out[v][t] = d
    for e in envs.values():
        e.close()
    if g is not None:
        g.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--steps", type=int, default=1199)
    ap.add_argument("--json", default=None)
    ap.add_argument("--gpu", action="store_true", help="also the HIP path on cuda:0 (the GPU box)")
    ap.add_argument("--cfg5", action="store_true", help="BASELINE cfg5: random ICs + gusts")
    args = ap.parse_args()
    out = run(args.n, args.steps, hip=args.gpu, cfg5=args.cfg5)
    for v, per in out.items():
        for t, d in per.items():
            print("%-7s t=%-5d lanes=%-4d h_m p99 %.3e max %.3e | alpha p99 %.3e | phi p99 %.3e | lat*R p99 %.3e"
                  % (v, t, d["lanes"], d["h_m"][1], d["h_m"][2], d["alpha"][1], d["phi"][1], d["lat*R"][1]))
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"workload": "tests/fp32_envelope.py: %d lanes, OracleEnvs(K=4, seed=5), goals default_rng(0), "
                                   "actions sample_actions(99, t), the reference IC" % args.n,
                       "stats": "per frame component [p50, p99, max] of |variant - ref| over lanes running on both sides",
                       "variants": {"control": "get_state / set_state every step, nothing else",
                                    "hip": "the HIP path (F16Envs, windowed layout) against the same oracle run",
                                    "round1": "fp32-stored fields rounded to fp32 once after the reset",
                                    "ulp1": "fp32-stored fields moved by one fp32 ulp once after the reset",
                                    "round": "fp32-stored fields rounded to fp32 after every step"},
                       "envelope": {v: {str(t): d for t, d in per.items()} for v, per in out.items()}}, f, indent=1)


if __name__ == "__main__":
    main()
