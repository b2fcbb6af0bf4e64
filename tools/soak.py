#!/usr/bin/env python3
"""Soak run of the bench's own configurations: many thousands of steps at BASELINE sizes,
window restarts and reset-cache refills included, with the NaN guard and the observation-bounds
diagnostic on, the feature window (F16Envs.obs_features) after every step; with F16ENV_LIB pointing at libf16env_debug.so the kernels also record every
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
    from f16_jsb_amd.features import features
    fw_checks = fw_mismatch = 0
    t0 = time.time()
    for t in range(steps):
        e.sample_actions(seed + 11, t, out=a)
        out = e.step(a)
        # the feature window after every step (window restarts and resets included), checked
        # against the whole-window transform every 997 steps
        fv = e.obs_features()
        if t % 997 == 996:
            fw_checks += 1
            fw_mismatch += int(not torch.equal(fv, features(out.obs)))
    torch.cuda.synchronize()
    wall = time.time() - t0
    finite = bool(torch.isfinite(out.obs).all())
    resets = float(e.get_state()[:, F16C_EP_COUNT].sum()) - ep0
    v = ctypes.c_uint32()
    is_debug = lib().f16env_debug_checks(e._h, None, ctypes.byref(v))
    r = {"envs": n, "steps": steps, "cfg5": cfg5, "kernel": e.step_kernel_name, "auto_resets": int(resets),
         "nonfinite_quarantined": e.nonfinite_count, "obs_out_of_bounds": e.obs_bounds_count,
         "final_obs_finite": finite, "debug_build": bool(is_debug), "violations": int(v.value),
         "feature_window": {"checks": fw_checks, "mismatches": fw_mismatch, "calls": dict(e.feature_window_calls)},
         "wall_s": round(wall, 2)}
    e.close()
    return r


def soak_rollout(n, T, rollouts, k, cfg5, policy, seed):
    """Device rollouts back to back on one handle (the cfg4 collector, rollout.collect_rollout):
    the persistent random-policy launch (f16_rollout_kernel, windowed output) or, with `policy`,
    one windowed rollout-step launch per step with a torch policy in the loop (clip, unclipped
    actions stored, timeout bootstrap), then GAE. Checks every buffer value is finite, every
    episode start is one episode-counter increment, and the handle's counters."""
    import torch
    from f16_jsb_amd._lib import lib
    from f16_jsb_amd.abi import F16C_EP_COUNT
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout

    e = F16Envs(n, stack_k=k, seed=seed, obs_layout="window", cfg5=cfg5, nan_guard=True, obs_check=True)
    e.reset()
    dev = e.device
    pf = vf = None
    if policy:
        g = torch.Generator(device="cpu").manual_seed(seed)
        W = (torch.randn(k * 15, 4, generator=g) * 0.02).to(dev)
        Wv = (torch.randn(k * 15, 1, generator=g) * 0.01).to(dev)

        def feats(obs):  # a fixed linear map of the whole (normalised) stack: ~1/3 of actions leave the Box
            x = obs.reshape(obs.shape[0], -1)
            return torch.tanh(x / torch.tensor([1e4, 1e4, 3e3] + [1.0] * 12, device=dev).repeat(k))

        def pf(obs):
            z = feats(obs)
            a = z @ W * 40.0 + torch.tensor([0.0, 0.0, 0.0, 0.6], device=dev)
            return a.contiguous(), (z @ Wv).reshape(-1), -(a * a).sum(1)

        def vf(obs):
            return (feats(obs) @ Wv).reshape(-1)
    buf = DeviceRolloutBuffer(T, n, k, dev)
    ep0 = e.get_state()[:, F16C_EP_COUNT].clone()
    starts = torch.zeros(n, dtype=torch.float64, device=dev)
    finite = True
    t0 = time.time()
    for r in range(rollouts):
        last_v, last_d = collect_rollout(e, buf, seed + 100 + r, step0=r * T, policy_fn=pf, value_fn=vf)
        buf.compute_returns_and_advantage(last_v, last_d)
        for f in ("frames", "actions", "rewards", "values", "log_probs", "advantages", "returns"):
            finite = finite and bool(torch.isfinite(getattr(buf, f)).all())
        starts += buf.episode_starts[1:].sum(0, dtype=torch.float64) + last_d.to(torch.float64)
    torch.cuda.synchronize()
    wall = time.time() - t0
    eps = (e.get_state()[:, F16C_EP_COUNT] - ep0).to(torch.float64)
    v = ctypes.c_uint32()
    is_debug = lib().f16env_debug_checks(e._h, None, ctypes.byref(v))
    r = {"envs": n, "rollouts": rollouts, "n_steps": T, "stack_k": k, "cfg5": cfg5,
         "collector": "policy in the loop (f16env_window_step_rollout per step)" if policy
         else "persistent random policy (f16_rollout_kernel, one launch per rollout)",
         "auto_resets": int(eps.sum()), "starts_equal_resets": bool(torch.equal(starts, eps)),
         "buffers_finite": finite, "nonfinite_quarantined": e.nonfinite_count, "obs_out_of_bounds": e.obs_bounds_count,
         "debug_build": bool(is_debug), "violations": int(v.value), "wall_s": round(wall, 2)}
    e.close()
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps3", type=int, default=20000)
    ap.add_argument("--steps5", type=int, default=10000)
    ap.add_argument("--rollouts", type=int, default=4, help="cfg4-share rollouts per collector (0 = none)")
    a = ap.parse_args()
    res = [soak(65536, a.steps3, False, 1), soak(131072, a.steps5, True, 2)]
    if a.rollouts:
        res += [soak_rollout(32768, 2048, a.rollouts, 10, False, False, 3),
                soak_rollout(32768, 2048, a.rollouts, 4, True, False, 4),
                soak_rollout(32768, 2048, max(1, a.rollouts // 2), 4, False, True, 5)]
    print(json.dumps({"lib": os.environ.get("F16ENV_LIB", "f16_jsb_amd/libf16env.so"), "runs": res}), flush=True)


if __name__ == "__main__":
    main()
