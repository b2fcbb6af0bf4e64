"""Child process of tests/test_gpu_debug_build.py: drives every kernel family of the DEBUG
build (libf16env_debug.so, F16ENV_LIB) through edge cases -- short episodes (auto-resets every
few steps), window restarts, cfg5 in-step and deferred resets, the reference stack K = 10
(global-table kernel), ragged N, the persistent rollout, the strided features, the trim --
and prints the invariant-violation bits the kernels recorded (f16env_debug_checks) as JSON."""
from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from f16_jsb_amd._lib import LIB_PATH, lib
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.features import features
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout

    assert LIB_PATH.endswith("libf16env_debug.so"), LIB_PATH
    ran = []
    cases = [dict(n=4096, stack_k=4, obs_layout="window", history=12, max_steps=7),
             dict(n=1000, stack_k=4, max_steps=5),
             dict(n=777, stack_k=10, max_steps=6),                      # global-table kernel
             dict(n=2049, stack_k=3, obs_layout="window", history=8, max_steps=6),
             dict(n=512, stack_k=4, obs_layout="window", history=8, max_steps=5, cfg5=True),
             dict(n=300, stack_k=4, max_steps=5, cfg5=True)]
    for c in cases:
        n = c.pop("n")
        e = F16Envs(n, seed=3, **c)
        e.reset()
        for t in range(40):
            out = e.step(e.sample_actions(1, t))
        assert bool(torch.isfinite(out.obs).all())
        if e.window:
            f = torch.empty(out.obs.shape[:-1] + (17,), device=out.obs.device)
            features(out.obs, f)
        ran.append("%s n=%d" % (e.step_kernel_name, n))
        e.close()
    os.environ["F16ENV_ICC_PERIOD"] = "0"  # cfg5 window with the deferred reset kernel
    e = F16Envs(512, stack_k=4, seed=3, obs_layout="window", history=8, max_steps=5, cfg5=True)
    e.reset()
    for t in range(30):
        e.step(e.sample_actions(1, t))
    ran.append("deferred resets " + e.step_kernel_name)
    e.close()
    e = F16Envs(1000, stack_k=4, seed=5, max_steps=9)
    e.reset()
    buf = DeviceRolloutBuffer(40, 1000, 4, e.device)
    collect_rollout(e, buf, 7)
    ran.append("f16_rollout_kernel")
    ic = np.tile(np.array(list(e.cfg.ic))[:19], (1000, 1))
    ic[:, 2] = np.linspace(3000, 30000, 1000)
    e.trim(torch.as_tensor(ic, device=e.device))
    ran.append("f16_trim_kernel")
    v = ctypes.c_uint32()
    is_debug = lib().f16env_debug_checks(e._h, None, ctypes.byref(v))
    torch.cuda.synchronize()
    e.close()
    print(json.dumps({"is_debug": int(is_debug), "violations": int(v.value), "ran": ran}))


if __name__ == "__main__":
    main()
