"""Policy feature transform on device.

The reference's policies see the observation through
``jsbsim_gym/features.py:37-67 JSBSimFeatureExtractor`` (15 -> 17 per frame: cylindrical goal
coordinates, normalised altitude, sin/cos of every angle), and its stacked variant
``jsbsim_gym/LMA_features.py:744-776 StackedLMAFeaturesExtractor`` applies that per frame to
the (B, K, 15) stack before its attention stage. Here the per-frame transform is one HIP
kernel (``f16env_features``) over any (..., 15) float32 block on the GPU, so a policy forward
can consume ``F16Envs.step``'s device obs without a round trip through PyTorch elementwise ops.

``JSBSimFeatureExtractor`` mirrors the reference class (features_dim 17, ``forward(obs)``);
``stacked_features(obs)`` is the (B, K, 15) -> (B, K, 17) first stage of the stacked extractor.
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import check, lib

FEATURES_DIM = 17
OBS_DIM = 15


def features(obs: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """(..., 15) float32 CUDA tensor -> (..., 17) float32, every frame transformed as
    features.py:37-67. Raises if the HIP library is missing (no CPU fallback)."""
    if obs.shape[-1] != OBS_DIM:
        raise ValueError("last dimension must be %d (jsbsim_gym.py:12-25 + goal), got %s" % (OBS_DIM, tuple(obs.shape)))
    if obs.dtype != torch.float32 or not obs.is_cuda:
        raise TypeError("obs must be a float32 device tensor")
    if (obs.dim() == 3 and not obs.is_contiguous() and obs.stride(-1) == 1 and obs.shape[0] > 0 and obs.shape[1] > 0
            and obs.stride(0) >= 0 and obs.stride(1) >= 0):
        # a strided (B, K, 15) stack -- e.g. F16Envs(obs_layout="window")'s observation view --
        # read in place by f16env_features_strided
        B, K = obs.shape[0], obs.shape[1]
        if out is None:
            out = torch.empty((B, K, FEATURES_DIM), dtype=torch.float32, device=obs.device)
        elif tuple(out.shape) != (B, K, FEATURES_DIM) or not out.is_contiguous() or out.dtype != torch.float32:
            raise ValueError("out must be a contiguous float32 tensor of shape %s" % ((B, K, FEATURES_DIM),))
        stream = ctypes.c_void_p(torch.cuda.current_stream(obs.device).cuda_stream)
        check(lib().f16env_features_strided(stream, B, K, ctypes.c_void_p(obs.data_ptr()), obs.stride(0), obs.stride(1),
                                            ctypes.c_void_p(out.data_ptr())), "f16env_features_strided")
        return out
    obs = obs.contiguous()
    n = obs.numel() // OBS_DIM
    if out is None:
        out = torch.empty(obs.shape[:-1] + (FEATURES_DIM,), dtype=torch.float32, device=obs.device)
    elif out.shape != obs.shape[:-1] + (FEATURES_DIM,) or not out.is_contiguous() or out.dtype != torch.float32:
        raise ValueError("out must be a contiguous float32 tensor of shape %s" % ((obs.shape[:-1] + (FEATURES_DIM,)),))
    stream = ctypes.c_void_p(torch.cuda.current_stream(obs.device).cuda_stream)
    check(lib().f16env_features(stream, n, ctypes.c_void_p(obs.data_ptr()), ctypes.c_void_p(out.data_ptr())),
          "f16env_features")
    return out


def stacked_features(obs: torch.Tensor) -> torch.Tensor:
    """(B, K, 15) -> (B, K, 17): the per-frame stage of StackedLMAFeaturesExtractor
    (LMA_features.py:757-765 reshapes to (B*K, 15), applies JSBSimFeatureExtractor, reshapes back)."""
    if obs.dim() != 3:
        raise ValueError("expected (B, K, 15)")
    return features(obs)


class JSBSimFeatureExtractor(torch.nn.Module):
    """Drop-in for jsbsim_gym/features.py:JSBSimFeatureExtractor (forward on (B, 15) obs,
    features_dim 17), computed by the HIP kernel. The SB3 BaseFeaturesExtractor contract it
    needs is the ``features_dim`` attribute and ``forward``."""

    def __init__(self, observation_space=None):
        super().__init__()
        self.observation_space = observation_space
        self._features_dim = FEATURES_DIM

    @property
    def features_dim(self) -> int:
        return self._features_dim

    def forward(self, observations: torch.Tensor) -> torch.Tensor:
        return features(observations)
