"""Fixed workload for the miscompile guard (TEST INFRASTRUCTURE, run by
tests/test_gpu_o1_differential.py in a subprocess with F16ENV_LIB naming the library under test).

Every kernel family runs on identical inputs: the windowed and contiguous step (one- and
two-waves-per-SIMD builds, F16ENV_OCC), the K = 10 global-table build, cfg5 modes with the
reset cache and in-step RunICs, the fused rollout step with clipped policy actions, the
persistent rollout, GAE, the timeout bootstrap, features, poses, trim. The outputs are saved to
an .npz; two libraries built from the same source with different optimisation (the product at
-O3, libf16env_o1.so at -O1, the bounds-checked debug build) must produce them bit for bit:
the source fixes every rounding (-ffp-contract=on, explicit FMAs), so any difference is the
compiler's -- round 3 found a register-allocation miscompile (all-zero rewards) that only the
ISA showed.

    F16ENV_LIB=f16_jsb_amd/libf16env_o1.so python tests/o1_diff_run.py out.npz
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def crash_ics(n):
    from f16_jsb_amd.abi import config_default, F16_IC_N
    ic = np.tile(np.array(config_default().ic[:F16_IC_N], np.float64), (n, 1))
    ic[:, 2] = np.linspace(150.0, 9000.0, n)
    ic[:, 7] = -0.35
    ic[:, 9:12] = np.linspace(-0.3, 0.3, n)[:, None]
    return ic


def main(path):
    import torch
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.features import features
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout
    from f16_jsb_amd.telemetry import poses
    out = {}
    dev = torch.device("cuda", 0)

    def steps(tag, e, n_steps, seed):
        print("phase", tag, flush=True)  # (the last phase printed names the section of a failure)
        rew, fl = [], []
        for t in range(n_steps):
            o = e.step(e.sample_actions(seed, t))
            rew.append(o.rew.clone())
            fl.append((o.terminated * 2 + o.truncated).clone())
        out[tag + "_rew"] = torch.stack(rew).cpu().numpy()
        out[tag + "_flags"] = torch.stack(fl).cpu().numpy()
        out[tag + "_obs"] = e.obs.contiguous().cpu().numpy()
        out[tag + "_state"] = e.get_state().cpu().numpy()

    n = 2048
    for occ in ("1", "2"):
        os.environ["F16ENV_OCC"] = occ
        for layout in ("window", "contiguous"):
            e = F16Envs(n, stack_k=4, seed=5, max_steps=30, obs_layout=layout)
            e.reset(ic=crash_ics(n))
            steps("ref_%s_occ%s" % (layout, occ), e, 40, 3)
            e.close()
            e = F16Envs(n, stack_k=4, seed=6, max_steps=8, cfg5=True, obs_layout=layout)
            e.reset()
            steps("cfg5_%s_occ%s" % (layout, occ), e, 40, 4)
            e.close()
    del os.environ["F16ENV_OCC"]
    e = F16Envs(1000, stack_k=10, seed=7, max_steps=25)  # K = 10: the global-table build
    e.reset(ic=crash_ics(1000))
    steps("k10", e, 40, 5)
    e.close()
    # fused rollout steps with a clipping policy, the bootstrap and GAE; the persistent rollout
    g = torch.Generator(device="cpu").manual_seed(1)
    W = (torch.randn(15, 4, generator=g) * 0.6).to(dev)

    def policy(obs):
        x = obs[:, -1, :]
        a = torch.tanh(x * 1e-3) @ W * 3.0
        return a.contiguous(), x[:, 2] * 1e-3, -(a * a).sum(1)

    for layout in ("window", "contiguous"):
        for cfg5 in (False, True):
            print("phase roll_%s%s" % (layout, "_cfg5" if cfg5 else ""), flush=True)
            e = F16Envs(n, stack_k=4, seed=8, max_steps=12, cfg5=cfg5, obs_layout=layout)
            e.reset() if cfg5 else e.reset(ic=crash_ics(n))
            b = DeviceRolloutBuffer(24, n, 4, dev)
            lv, ld = collect_rollout(e, b, 9, policy_fn=policy)
            b.compute_returns_and_advantage(lv, ld)
            tag = "roll_%s%s" % (layout, "_cfg5" if cfg5 else "")
            for f in ("frames", "actions", "rewards", "episode_starts", "advantages", "returns"):
                out[tag + "_" + f] = getattr(b, f).cpu().numpy()
            b2 = DeviceRolloutBuffer(24, n, 4, dev)
            collect_rollout(e, b2, 10)  # persistent
            for f in ("frames", "rewards", "episode_starts"):
                out[tag + "_persistent_" + f] = getattr(b2, f).cpu().numpy()
            out[tag + "_obs"] = e.obs.contiguous().cpu().numpy()
            out[tag + "_features"] = features(e.obs).cpu().numpy()
            out[tag + "_poses"] = poses(e.obs).cpu().numpy()
            e.close()
    print("phase trim", flush=True)
    e = F16Envs(256, stack_k=4, seed=9)
    ic = crash_ics(256)
    ic[:, 2] = np.linspace(3000, 30000, 256)
    ic[:, 3] = np.linspace(600, 1200, 256)
    t_ic, res = e.trim(torch.as_tensor(ic, device=dev))
    out["trim_ic"] = t_ic.cpu().numpy()
    out["trim_res"] = res.cpu().numpy()
    e.close()
    np.savez(path, **out)
    print("saved %d arrays to %s" % (len(out), path))


if __name__ == "__main__":
    main(sys.argv[1])
