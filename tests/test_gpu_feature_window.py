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


@pytest.mark.parametrize("c", CASES, ids=["n%d_k%d_T%d_%s%s%s" % (c["n"], c["k"], c["T"], c["order"],
                                                                  "_cfg5" if c["cfg5"] else "",
                                                                  "" if c["autoreset"] else "_noauto")
                                          for c in CASES])
def test_feature_window_fused_in_plain_steps(gpu, c):
    """a fused_features handle keeps the feature window in the PLAIN step's
    epilogue (f16env_window_step_ex, F16_STEP_FEATURE_WINDOW, the f16_step_winx_kernel build):
    after every op of the seeded sequence -- plain steps with given or in-kernel actions, caller /
    masked resets, set_state / set_obs, rollout-slot steps, one-launch rollouts, restarts --
    obs_features() equals the whole-window transform bit for bit, and the handle's observations,
    rewards and flags stay bit-identical to a plain handle's."""
    import torch
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.features import features
    n, k = c["n"], c["k"]
    kw = dict(stack_k=k, seed=11, max_steps=c["max_steps"], cfg5=c["cfg5"], autoreset=c["autoreset"],
              obs_layout="window", history=c["T"], window_order=c["order"])
    e = F16Envs(n, fused_features=True, **kw)
    ref = F16Envs(n, **kw)
    e.reset(), ref.reset()
    rng = np.random.default_rng(n * 37 + k)
    for i in range(60):
        r = rng.random()
        if not c["autoreset"]:
            d = (e.term | e.trunc) != 0
            if bool(d.any()):
                e.reset(mask=d), ref.reset(mask=d)
        if r < 0.05:
            m = torch.as_tensor(rng.random(n) < 0.3)
            e.reset(mask=m), ref.reset(mask=m)
        elif r < 0.08:
            e.set_state(e.get_state()), ref.set_state(ref.get_state())
        elif r < 0.10:
            e.set_obs(e.obs.clone()), ref.set_obs(ref.obs.clone())
        elif r < 0.14 and c["autoreset"]:
            e.step_rollout(5, i), ref.step_rollout(5, i)
        elif r < 0.16 and c["autoreset"]:
            T = 3
            for x in (e, ref):
                fr = torch.empty((T, n, 15), dtype=torch.float32, device=gpu)
                ac = torch.empty((T, n, 4), dtype=torch.float32, device=gpu)
                rw = torch.empty((T, n), dtype=torch.float32, device=gpu)
                ns = torch.empty((T - 1, n), dtype=torch.float32, device=gpu)
                ls = torch.empty((n,), dtype=torch.float32, device=gpu)
                x.rollout_random(7, 1000 + i, T, fr, ac, rw, ns, ls)
        elif r < 0.5:  # in-kernel actions (the sample_actions stream)
            a, b = e.step(None, seed=3, step=i), ref.step(ref.sample_actions(3, i))
            assert torch.equal(a.rew, b.rew) and torch.equal(a.terminated, b.terminated)
        else:
            act = e.sample_actions(3, i)
            e.step(act), ref.step(act)
        assert torch.equal(e.obs, ref.obs), i
        got = e.obs_features()
        assert torch.equal(got, features(e.obs)), (i, float((got - features(e.obs)).abs().max()))
    calls = e.feature_window_calls
    assert calls["fused"] > 25, calls
    e.close(), ref.close()


@pytest.mark.parametrize("layout", ["window", "contiguous"])
@pytest.mark.parametrize("cfg5", [False, True], ids=["reference_task", "cfg5"])
def test_in_kernel_actions_equal_sample_then_step(gpu, layout, cfg5):
    """step(None, seed=, step=) draws the actions inside the step kernel from
    the sample_actions stream: bit-identical to sample_actions + step (obs, rewards, flags,
    episode bookkeeping, state), across auto-resets; the windowed layout launches the winx build."""
    import torch
    from f16_jsb_amd.env import F16Envs
    n = 3000
    kw = dict(stack_k=4, seed=21, max_steps=6, cfg5=cfg5, obs_layout=layout)
    a, b = F16Envs(n, **kw), F16Envs(n, **kw)
    a.reset(), b.reset()
    for t in range(20):
        sa = a.step(None, seed=77, step=t)
        sb = b.step(b.sample_actions(77, t))
        for f in ("obs", "rew", "terminated", "truncated", "ep_return", "ep_len"):
            assert torch.equal(getattr(sa, f), getattr(sb, f)), (t, f)
    assert torch.equal(a.get_state(), b.get_state())
    a.close(), b.close()


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
