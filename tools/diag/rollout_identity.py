"""Diagnostic: persistent rollout kernel vs fused per-step rollout launches -- bit-identical?
(tests/test_gpu_rollout.py test_persistent_rollout_matches_fused_steps setup)"""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from oracle_ref import default_ic
from f16_jsb_amd.env import F16Envs
from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout

dev = torch.device("cuda", 0)
for n, k, T in ((4096, 4, 64), (777, 3, 33)):
    ic = np.tile(default_ic(), (n, 1))
    ic[:, 2] = np.linspace(150.0, 9000.0, n)
    ic[:, 7] = -0.35
    bufs, envs = [], []
    for persistent in (False, True):
        e = F16Envs(n, stack_k=k, seed=4, max_steps=40)
        e.reset(ic=ic)
        b = DeviceRolloutBuffer(T, n, k, dev)
        collect_rollout(e, DeviceRolloutBuffer(3, n, k, dev), 17, persistent=persistent)
        collect_rollout(e, b, 21, step0=100, persistent=persistent)
        bufs.append(b)
        envs.append(e)
    b0, b1 = bufs
    for name in ("frames", "obs0", "rewards", "actions", "episode_starts"):
        x, y = getattr(b0, name), getattr(b1, name)
        ne = (x != y)
        print(n, k, T, name, "equal", bool(torch.equal(x, y)), "differing", int(ne.sum()),
              "max", float((x.float() - y.float()).abs().max()), flush=True)
    print(n, "final obs equal", torch.equal(envs[0].obs, envs[1].obs), "state equal",
          torch.equal(envs[0].get_state(), envs[1].get_state()), flush=True)
