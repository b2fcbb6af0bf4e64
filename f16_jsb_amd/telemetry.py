"""Render / telemetry export from device snapshots.

The reference draws one env with moderngl (jsbsim_gym/jsbsim_gym.py:333-462, Viewer in
visualization/rendering.py); each frame it turns the env state into Viewer poses
(jsbsim_gym.py:381-415): the aircraft position in viewer axes, its attitude quaternion and
the goal position. ``poses`` does that transform for every env at once with one HIP launch
(``f16env_poses``) over the device observations, so a recorder or a renderer on another
process gets poses without stepping the FDM on the CPU. (The OpenGL viewer itself is not part
of the hot path and is not rebuilt: moderngl is absent here and the reference's renderer is
broken, SURVEY.md component #9.)
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import check, lib

POSE_DIM = 10
POSE_FIELDS = ("ac_x", "ac_y", "ac_z", "q_w", "q_x", "q_y", "q_z", "goal_x", "goal_y", "goal_z")


def poses(obs: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """(N, K, 15) stack (newest frame used) or (N, 15) frames, float32 device tensor ->
    (N, 10) poses (see POSE_FIELDS), jsbsim_gym.py:381-415 per env."""
    if obs.dtype != torch.float32 or not obs.is_cuda:
        raise TypeError("obs must be a float32 device tensor")
    if obs.dim() == 3 and obs.shape[-1] == 15:
        if obs.stride(-1) != 1 or obs.shape[0] == 0 or obs.stride(0) < 15:
            obs = obs.contiguous()
        # the newest frame of each stack read in place (contiguous or windowed layout)
        n, k = obs.shape[0], obs.shape[1]
        base, stride = obs.data_ptr() + 4 * obs.stride(1) * (k - 1), obs.stride(0)
    elif obs.dim() == 2 and obs.shape[-1] == 15:
        obs = obs.contiguous()
        n, base, stride = obs.shape[0], obs.data_ptr(), 15
    else:
        raise ValueError("expected (N, K, 15) or (N, 15), got %s" % (tuple(obs.shape),))
    if out is None:
        out = torch.empty((n, POSE_DIM), dtype=torch.float32, device=obs.device)
    stream = ctypes.c_void_p(torch.cuda.current_stream(obs.device).cuda_stream)
    check(lib().f16env_poses(stream, n, ctypes.c_void_p(base), stride, ctypes.c_void_p(out.data_ptr())),
          "f16env_poses")
    return out


def snapshot(envs, path: str = None):
    """Poses of every env of an F16Envs handle as a host numpy array (and optionally a .npy
    file): the telemetry record a viewer replays. (envs.poses(): a fused_poses handle's step has
    already written them, no launch here.)"""
    import numpy as np
    p = (envs.poses() if hasattr(envs, "poses") else poses(envs.obs)).cpu().numpy()
    if path is not None:
        np.save(path, p)
    return p
