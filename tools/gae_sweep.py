#!/usr/bin/env python3
"""GAE kernel A/B (f16env_gae, cfg4's per-GPU share 2 048 x 32 768 by default): the software-
pipelining depth U (F16ENV_GAE_U: steps of loads in flight per block) and the envs per wave
(F16ENV_GAE_LPW), each configuration in its own process (the library reads both once); HIP
events over 20 launches after 3. Run on the GPU box:

    python tools/gae_sweep.py [--T 2048] [--N 32768] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(T, N):
    sys.path.insert(0, ROOT)
    import torch
    from f16_jsb_amd.rollout import DeviceRolloutBuffer
    dev = torch.device("cuda", 0)
    buf = DeviceRolloutBuffer(T, N, 1, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    buf.rewards.normal_(generator=g)
    buf.values.normal_(generator=g)
    buf.episode_starts.copy_((torch.rand(T, N, device=dev, generator=g) < 0.01).float())
    lv = torch.randn(N, device=dev, generator=g)
    ld = torch.zeros(N, dtype=torch.float32, device=dev)
    for _ in range(3):
        buf.compute_returns_and_advantage(lv, ld)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(20):
        buf.compute_returns_and_advantage(lv, ld)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 20
    ck = float(buf.advantages.double().sum())
    print(json.dumps({"ms": round(ms, 4), "TBps": round((T * N * 20 + N * 5) / ms / 1e9, 3), "checksum": ck}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=2048)
    ap.add_argument("--N", type=int, default=32768)
    ap.add_argument("--json", default=None)
    ap.add_argument("--one", action="store_true")
    a = ap.parse_args()
    if a.one:
        return one(a.T, a.N)
    res = {}
    for u in (8, 16, 32):
        for lpw in (16, 32, 64):
            env = dict(os.environ, F16ENV_GAE_U=str(u), F16ENV_GAE_LPW=str(lpw))
            key = "U%d_LPW%d" % (u, lpw)
            r = subprocess.run([sys.executable, __file__, "--one", "--T", str(a.T), "--N", str(a.N)], env=env,
                               capture_output=True, text=True, timeout=120)
            line = [l for l in r.stdout.splitlines() if l.startswith("{")]
            res[key] = json.loads(line[-1]) if line else {"error": r.stderr[-500:]}
            print(key, res[key], flush=True)
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
