"""Policy feature transform: jsbsim_gym/features.py:37-67.

CPU: the torch restatement (tests/features_ref.py) against known answers, and the ABI shape /
error behaviour. GPU (-m gpu): the HIP kernel f16env_features against the restatement on the
same seeded frames, including ragged sizes, unaligned slices, K-stacks and degenerate inputs.
Tolerances (float32): copied fields bit-exact; dist/dz/alt normalisations within 2 ulp
(3e-7 relative: same IEEE op sequence, torch's CPU reduction/scalar paths differ by an ulp); sin/cos outputs within 1e-6 absolute (OCML vs torch's
vectorised libm differ by 1-2 ulp, and atan2's ulp error of a value near pi feeds cos/sin of
the relative bearing).
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from features_ref import jsbsim_features_ref, stacked_features_ref  # noqa: E402


def _frame(pos, mach, ab, pqr, ptp, goal):
    return torch.tensor([list(pos) + [mach] + list(ab) + list(pqr) + list(ptp) + list(goal)], dtype=torch.float32)


def test_ref_known_answers():
    # goal 1000 m due "north" (+x) of the aircraft, same altitude, heading 0
    o = _frame((0.0, 0.0, 1500.0), 0.8, (0.1, -0.05), (0.01, 0.02, 0.03), (0.2, -0.1, 0.0), (1000.0, 0.0, 1500.0))
    f = jsbsim_features_ref(o)[0].numpy()
    assert f.shape == (17,)
    assert f[0] == pytest.approx(0.5, abs=1e-7)          # 1 / (1 + 1000 * 1e-3)
    assert f[1] == 0.0 and f[2] == pytest.approx(0.1)    # dz, 1500 / 15000
    np.testing.assert_array_equal(f[3:7], np.float32([0.8, 0.01, 0.02, 0.03]))
    np.testing.assert_allclose(f[7:11], np.float32([math.cos(0.1), math.cos(-0.05), math.sin(0.1), math.sin(-0.05)]), atol=1e-7)
    np.testing.assert_allclose(f[11:15], np.float32([math.cos(0.2), math.cos(-0.1), math.sin(0.2), math.sin(-0.1)]), atol=1e-7)
    assert f[15] == pytest.approx(1.0) and f[16] == pytest.approx(0.0, abs=1e-7)  # bearing 0 - psi 0
    # goal due +y, heading pi/2: relative bearing 0; goal 3 km up: dz_norm 0.2
    o = _frame((0.0, 0.0, 0.0), 0.5, (0, 0), (0, 0, 0), (0, 0, math.pi / 2), (0.0, 2000.0, 3000.0))
    f = jsbsim_features_ref(o)[0].numpy()
    assert f[0] == pytest.approx(1.0 / 3.0, rel=1e-6) and f[1] == pytest.approx(0.2)
    assert f[15] == pytest.approx(1.0, abs=1e-6) and f[16] == pytest.approx(0.0, abs=1e-6)
    # on top of the goal: distance 0, atan2(0, 0) = 0
    o = _frame((5.0, 7.0, 100.0), 0.5, (0, 0), (0, 0, 0), (0, 0, 1.0), (5.0, 7.0, 100.0))
    f = jsbsim_features_ref(o)[0].numpy()
    assert f[0] == 1.0 and f[15] == pytest.approx(math.cos(-1.0)) and f[16] == pytest.approx(math.sin(-1.0))


def test_ref_stacked_is_per_frame():
    g = torch.Generator().manual_seed(0)
    obs = torch.randn(5, 4, 15, generator=g) * 100
    s = stacked_features_ref(obs)
    assert s.shape == (5, 4, 17)
    for k in range(4):
        torch.testing.assert_close(s[:, k], jsbsim_features_ref(obs[:, k]), rtol=0, atol=0)


def _random_frames(n, seed):
    rng = np.random.default_rng(seed)
    o = np.empty((n, 15), np.float32)
    o[:, 0:2] = rng.uniform(-2e4, 2e4, (n, 2))
    o[:, 2] = rng.uniform(0, 15000, n)
    o[:, 3] = rng.uniform(0, 2, n)
    o[:, 4:6] = rng.uniform(-0.5, 0.5, (n, 2))
    o[:, 6:9] = rng.uniform(-3, 3, (n, 3))
    o[:, 9:12] = rng.uniform(-math.pi, math.pi, (n, 3))
    o[:, 12:14] = o[:, 0:2] + rng.uniform(-1e4, 1e4, (n, 2))
    o[:, 14] = rng.uniform(1000, 4000, n)
    o[: n // 50, 12:15] = o[: n // 50, 0:3]  # degenerate: at the goal
    return torch.from_numpy(o)


def _check(got, want):
    got, want = got.cpu(), want.cpu()
    torch.testing.assert_close(got[..., 3:7], want[..., 3:7], rtol=0, atol=0)
    torch.testing.assert_close(got[..., 0:3], want[..., 0:3], rtol=3e-7, atol=1e-30)
    torch.testing.assert_close(got[..., 7:], want[..., 7:], rtol=0, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 255, 256, 257, 4096 + 13, 65536 * 4])
def test_gpu_features_match_ref(gpu, n):
    from f16_jsb_amd.features import features
    o = _random_frames(n, n)
    _check(features(o.cuda()), jsbsim_features_ref(o))


@pytest.mark.gpu
def test_gpu_features_stacked_and_unaligned(gpu):
    from f16_jsb_amd.features import JSBSimFeatureExtractor, features, stacked_features
    o = _random_frames(3000 * 4, 7).reshape(3000, 4, 15)
    _check(stacked_features(o.cuda()), stacked_features_ref(o))
    # a slice that starts mid-frame-block (not 16-byte aligned): scalar path
    flat = _random_frames(1001, 8).cuda()
    sub = flat[1:]
    assert (sub.data_ptr() % 16) != 0
    _check(features(sub), jsbsim_features_ref(flat[1:].cpu()))
    ext = JSBSimFeatureExtractor()
    assert ext.features_dim == 17
    _check(ext(o[:, -1].contiguous().cuda()), jsbsim_features_ref(o[:, -1]))


@pytest.mark.gpu
def test_gpu_features_of_env_obs(gpu):
    """The transform on the env's own device obs (the policy-forward use)."""
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.features import stacked_features
    e = F16Envs(2048, stack_k=4, seed=3)
    e.reset()
    for t in range(20):
        out = e.step(e.sample_actions(1, t))
    _check(stacked_features(out.obs), stacked_features_ref(out.obs.cpu()))
    e.close()


@pytest.mark.gpu
def test_gpu_features_of_window_view(gpu):
    """The transform read in place from a windowed observation (strided (N, K, 15) view,
    f16env_features_strided) equals the transform of the same frames made contiguous, and
    the reference transform; plus an odd-stride (unaligned) slice."""
    import torch
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.features import stacked_features
    e = F16Envs(1000, stack_k=4, seed=5, obs_layout="window", history=12)
    e.reset()
    for t in range(20):
        out = e.step(e.sample_actions(2, t))
    assert not out.obs.is_contiguous()
    a = stacked_features(out.obs)
    b = stacked_features(out.obs.contiguous())
    torch.testing.assert_close(a, b, rtol=0, atol=0)
    _check(a, stacked_features_ref(out.obs.cpu()))
    big = torch.randn(300, 7, 19, device="cuda") * 100
    v = big[:, 1:6, 2:17]  # row stride 133, frame stride 19, 8-B-misaligned base
    torch.testing.assert_close(stacked_features(v), stacked_features(v.contiguous()), rtol=0, atol=0)
    w = big.transpose(0, 1)[:, :, 2:17]  # (7, 300, 15): row stride 19 < frame stride 133
    torch.testing.assert_close(stacked_features(w), stacked_features(w.contiguous()), rtol=0, atol=0)
    e.close()


def test_default_history():
    from f16_jsb_amd.env import _default_history
    for k in (1, 4, 10, 63, 100, 200):
        T = _default_history(k)
        assert T >= 2 * k and T >= 256


def test_features_rejects_bad_input():
    from f16_jsb_amd.features import features
    with pytest.raises(ValueError):
        features(torch.zeros(4, 14))
    with pytest.raises(TypeError):
        features(torch.zeros(4, 15))  # CPU tensor: the product path has no CPU fallback


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,cfg5", [(4096, 4, False), (1000, 4, False), (777, 8, False), (2048, 4, True)])
def test_gpu_step_features_equal_separate_kernel(gpu, n, k, cfg5):
    """F16Envs.step(..., features=f): the features of the returned obs computed in the same
    call, bit-identical to f16env_features over the same obs -- including the rows of lanes
    that finished and were reset during the step (cfg5: after the deferred-reset kernel)."""
    from oracle_ref import default_ic
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.features import features
    ic = np.tile(default_ic(), (n, 1))
    ic[:, 2] = np.linspace(150.0, 9000.0, n)
    ic[:, 7] = -0.35
    e = F16Envs(n, stack_k=k, seed=6, cfg5=cfg5)
    e.reset(ic=None if cfg5 else ic)
    f = torch.empty((n, k, 17), dtype=torch.float32, device=gpu)
    done_total = 0
    for t in range(25):
        out = e.step(e.sample_actions(8, t), features=f)
        done_total += int((out.terminated | out.truncated).sum())
        assert torch.equal(f, features(out.obs)), "step %d" % t
    assert cfg5 or done_total > 0
    e.close()
