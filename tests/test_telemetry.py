"""Render/telemetry pose export: jsbsim_gym.py:381-415.

CPU: the numpy restatement (tests/telemetry_ref.py) against known answers. GPU: the HIP kernel
f16env_poses against the restatement on env observations and random frames; positions
bit-exact (same float32 ops), quaternion components within 1e-6 (OCML vs numpy cos/sin ulps).
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from telemetry_ref import from_euler, pose_ref  # noqa: E402


def test_ref_known_answers():
    q = from_euler(np.float32(0), np.float32(0), np.float32(0))
    np.testing.assert_array_equal(q, np.float32([1, 0, 0, 0]))
    # pure yaw psi: q = (cos psi/2, 0, 0, sin psi/2)
    q = from_euler(np.float32(0), np.float32(0), np.float32(1.0))
    np.testing.assert_allclose(q, [math.cos(0.5), 0, 0, math.sin(0.5)], atol=1e-7)
    # the rotation it encodes is R_z(psi) R_y(theta) R_x(phi)
    phi, th, psi = np.float32(0.3), np.float32(-0.2), np.float32(2.0)
    w, x, y, z = from_euler(phi, th, psi).astype(np.float64)
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    c, s = np.cos, np.sin
    Rz = np.array([[c(psi), -s(psi), 0], [s(psi), c(psi), 0], [0, 0, 1]])
    Ry = np.array([[c(th), 0, s(th)], [0, 1, 0], [-s(th), 0, c(th)]])
    Rx = np.array([[1, 0, 0], [0, c(phi), -s(phi)], [0, s(phi), c(phi)]])
    np.testing.assert_allclose(R, Rz @ Ry @ Rx, atol=1e-6)
    frame = np.zeros(15, np.float32)
    frame[:3] = [1000.0, -2000.0, 1500.0]
    frame[12:15] = [3000.0, 4000.0, 2500.0]
    p = pose_ref(frame)
    np.testing.assert_allclose(p[:3], [2.0, 1.5, 1.0], rtol=1e-6)
    np.testing.assert_array_equal(p[3:7], np.float32([1, 0, 0, 0]))
    np.testing.assert_allclose(p[7:], [-4.0, 2.5, 3.0], rtol=1e-6)


@pytest.mark.gpu
def test_gpu_poses_match_ref(gpu):
    import torch
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.telemetry import poses
    e = F16Envs(3000, stack_k=4, seed=12)
    e.reset()
    for t in range(15):
        e.step(e.sample_actions(2, t))
    obs = e.obs
    got = poses(obs).cpu().numpy()
    want = np.stack([pose_ref(f) for f in obs[:, -1].cpu().numpy()])
    np.testing.assert_array_equal(got[:, [0, 1, 2, 7, 8, 9]], want[:, [0, 1, 2, 7, 8, 9]])
    np.testing.assert_allclose(got[:, 3:7], want[:, 3:7], rtol=0, atol=1e-6)
    # (N, 15) input and arbitrary angles
    rng = np.random.default_rng(3)
    fr = rng.uniform(-4, 4, (777, 15)).astype(np.float32) * np.float32(1000.0)
    fr[:, 9:12] = rng.uniform(-math.pi, math.pi, (777, 3))
    got = poses(torch.as_tensor(fr).cuda()).cpu().numpy()
    want = np.stack([pose_ref(f) for f in fr])
    np.testing.assert_array_equal(got[:, [0, 1, 2, 7, 8, 9]], want[:, [0, 1, 2, 7, 8, 9]])
    np.testing.assert_allclose(got[:, 3:7], want[:, 3:7], rtol=0, atol=1e-6)
    e.close()
