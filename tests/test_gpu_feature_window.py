"""Feature window (F16Envs.obs_features, f16env_features_window_step): the policy features of the
windowed observation kept incrementally beside the frame histories must equal, bit for bit, the
feature transform of the whole observation (features.features(envs.obs), itself checked against
the fp32 restatement of features.py:37-67 in tests/test_features.py) after every op of a seeded
random sequence: steps (in-kernel resets at short TimeLimits, cfg5 cache resets), steps whose
features are not asked for, window restarts (short histories), caller / masked resets, set_state
and set_obs, fused rollout steps and the one-launch rollout, in both window orders, K = 1 .. 10,
with and without auto-reset."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = [
    dict(n=1000, k=4, T=9, order="position", max_steps=5, cfg5=False, autoreset=True),
    dict(n=257, k=10, T=21, order="env", max_steps=7, cfg5=False, autoreset=True),
    dict(n=65, k=1, T=2, order="position", max_steps=3, cfg5=False, autoreset=True),
    dict(n=513, k=3, T=7, order="position", max_steps=4, cfg5=True, autoreset=True),
    dict(n=300, k=5, T=12, order="env", max_steps=6, cfg5=False, autoreset=False),
    dict(n=4096, k=4, T=64, order="position", max_steps=1200, cfg5=False, autoreset=True),
]


@pytest.mark.parametrize("c", CASES, ids=["n%d_k%d_T%d_%s%s%s" % (c["n"], c["k"], c["T"], c["order"],
                                                                  "_cfg5" if c["cfg5"] else "",
                                                                  "" if c["autoreset"] else "_noauto")
                                          for c in CASES])
def test_feature_window_equals_full_transform(gpu, c):
    import torch
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.features import features
    n, k = c["n"], c["k"]
    e = F16Envs(n, stack_k=k, seed=11, max_steps=c["max_steps"], cfg5=c["cfg5"], autoreset=c["autoreset"],
                obs_layout="window", history=c["T"], window_order=c["order"])
    e.reset()
    rng = np.random.default_rng(n * 31 + k)
    checked = 0
    for i in range(60):
        r = rng.random()
        if not c["autoreset"]:  # the caller resets its finished lanes before the next step
            d = (e.term | e.trunc) != 0
            if bool(d.any()):
                e.reset(mask=d)
        if r < 0.06:
            e.reset(mask=torch.as_tensor(rng.random(n) < 0.3))
        elif r < 0.09:
            e.set_state(e.get_state())
        elif r < 0.11:
            e.set_obs(e.obs.clone())
        elif r < 0.16 and c["autoreset"]:
            e.step_rollout(5, i)
        elif r < 0.18 and c["autoreset"]:
            T = 3
            fr = torch.empty((T, n, 15), dtype=torch.float32, device=gpu)
            ac = torch.empty((T, n, 4), dtype=torch.float32, device=gpu)
            rw = torch.empty((T, n), dtype=torch.float32, device=gpu)
            ns = torch.empty((T - 1, n), dtype=torch.float32, device=gpu)
            ls = torch.empty((n,), dtype=torch.float32, device=gpu)
            e.rollout_random(7, 1000 + i, T, fr, ac, rw, ns, ls)
        else:
            e.step(e.sample_actions(3, i))
        if rng.random() < 0.8:  # sometimes a step goes by without its features
            got = e.obs_features()
            want = features(e.obs)
            assert got.shape == (n, k, 17)
            assert torch.equal(got, want), (i, float((got - want).abs().max()))
            checked += 1
    assert checked > 30
    calls = e.feature_window_calls
    # without auto-reset the caller's resets (most steps here) make whole-window transforms
    assert calls["incremental"] > (calls["full"] if c["autoreset"] else 5), calls
    e.close()


@pytest.mark.parametrize("k,order,cfg5", [(4, "position", False), (10, "env", False), (3, "position", True),
                                           (1, "position", False)])
def test_feature_window_fused_in_rollout_steps(gpu, k, order, cfg5):
    """Rollout-slot steps (step_rollout, in-kernel or policy actions, clipped) keep the feature
    window in their epilogue (F16_SLOT_FEATURE_WINDOW): after each, obs_features launches
    nothing and equals the whole-window transform; mixed with plain steps (incremental kernel),
    short TimeLimits (resets every few steps), restarts (T = 2K+1) and a caller reset."""
    import torch
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.features import features
    n = 777
    e = F16Envs(n, stack_k=k, seed=5, max_steps=5, cfg5=cfg5, obs_layout="window", history=2 * k + 1,
                window_order=order)
    e.reset()
    rng = np.random.default_rng(k)
    for i in range(50):
        r = rng.random()
        if i == 25:
            e.reset(mask=torch.as_tensor(rng.random(n) < 0.5))
        elif r < 0.4:
            e.step_rollout(9, i)
        elif r < 0.8:
            act = (torch.randn((n, 4), device=gpu) * 1.5).contiguous()
            e.step_rollout(9, i, policy_actions=act, clip=True)
        else:
            e.step(e.sample_actions(4, i))
        got = e.obs_features()
        assert torch.equal(got, features(e.obs)), i
    calls = e.feature_window_calls
    assert calls["fused"] > 25 and calls["full"] <= 4, calls
    e.close()


def test_feature_window_contiguous_layout(gpu):
    """The contiguous layout has no feature histories: obs_features is the transform of obs."""
    import torch
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.features import features
    e = F16Envs(100, stack_k=4, seed=2)
    e.reset()
    e.step(e.sample_actions(1, 0))
    assert torch.equal(e.obs_features(), features(e.obs))
    e.close()
