"""Test oracle for the policy feature transform (TEST INFRASTRUCTURE ONLY -- the product path
is the HIP kernel f16env_features; nothing under f16_jsb_amd/ imports this).

A plain PyTorch float32 restatement of jsbsim_gym/features.py:37-67
(JSBSimFeatureExtractor.forward), line by line, on CPU tensors. The reference module itself is
not imported (importing reference Python was denied); parity for this row rests on
this restatement plus the known answers in tests/test_features.py.
"""
from __future__ import annotations

import torch


def jsbsim_features_ref(observations: torch.Tensor) -> torch.Tensor:
    """(B, 15) float32 -> (B, 17) float32, features.py:37-67."""
    th = torch
    position = observations[:, :3]                 # :39
    mach = observations[:, 3:4]                    # :40
    alpha_beta = observations[:, 4:6]              # :41
    angular_rates = observations[:, 6:9]           # :42
    phi_theta = observations[:, 9:11]              # :43
    psi = observations[:, 11:12]                   # :44
    goal = observations[:, 12:]                    # :45
    displacement = goal - position                 # :48
    distance = th.sqrt(th.sum(displacement[:, :2] ** 2, 1, True))  # :49
    dz = displacement[:, 2:3]                      # :50
    altitude = position[:, 2:3]                    # :51
    abs_bearing = th.atan2(displacement[:, 1:2], displacement[:, 0:1])  # :52
    rel_bearing = abs_bearing - psi                # :53
    dist_norm = 1 / (1 + distance * 1e-3)          # :56
    dz_norm = dz / 15000                           # :59
    alt_norm = altitude / 15000                    # :60
    cab, sab = th.cos(alpha_beta), th.sin(alpha_beta)  # :63
    cpt, spt = th.cos(phi_theta), th.sin(phi_theta)    # :64
    cr, sr = th.cos(rel_bearing), th.sin(rel_bearing)  # :65
    return th.concat([dist_norm, dz_norm, alt_norm, mach, angular_rates, cab, sab, cpt, spt, cr, sr], 1)  # :67


def stacked_features_ref(obs: torch.Tensor) -> torch.Tensor:
    """(B, K, 15) -> (B, K, 17): LMA_features.py:757-765 reshape, per-frame transform, reshape."""
    b, k, f = obs.shape
    return jsbsim_features_ref(obs.reshape(b * k, f)).reshape(b, k, 17)
