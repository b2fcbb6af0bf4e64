"""Test oracle for the render/telemetry pose export (TEST INFRASTRUCTURE ONLY).

numpy float32 restatement of the state -> Viewer transform of jsbsim_gym/jsbsim_gym.py:381-415
with Quaternion.from_euler / __mul__ of jsbsim_gym/visualization/quaternion.py:7-45 (float32
arrays, the reference's operation order). The reference modules are not imported (SURVEY.md
8c: denied); the known answers in tests/test_telemetry.py pin this restatement.
"""
from __future__ import annotations

import numpy as np


def _qmul(a, b):
    """quaternion.py:9-14 on float32 arrays (q3 = np.zeros(4) holds float32 results)."""
    w = a[0] * b[0] - a[1:].dot(b[1:])
    v = a[0] * b[1:] + b[0] * a[1:] + np.cross(a[1:], b[1:])
    return np.array([w, *v], dtype=np.float32)


def from_euler(phi, theta, psi):
    """quaternion.py:38-44, mode 0: q_psi * q_theta * q_phi."""
    q1 = np.array([np.cos(phi / 2), np.sin(phi / 2), 0, 0], dtype=np.float32)
    q2 = np.array([np.cos(theta / 2), 0, np.sin(theta / 2), 0], dtype=np.float32)
    q3 = np.array([np.cos(psi / 2), 0, 0, np.sin(psi / 2)], dtype=np.float32)
    return _qmul(_qmul(q3, q2), q1)


def pose_ref(frame):
    """One float32 frame (15,) -> (10,) pose as JSBSimEnv.render hands it to the Viewer."""
    scale = 1e-3
    f = np.asarray(frame, np.float32)
    pos, eul, goal = f[:3], f[9:12], f[12:15]
    ac = np.array([-pos[1] * scale, pos[2] * scale, pos[0] * scale], dtype=np.float32)   # :392-396
    q = from_euler(*eul)                                                                    # :400
    qd = np.array([q[0], -q[2], -q[3], q[1]], dtype=np.float32)                             # :404-406
    g = np.array([-goal[1] * scale, goal[2] * scale, goal[0] * scale], dtype=np.float32)    # :410-414
    return np.concatenate([ac, qd, g]).astype(np.float32)
