"""Shared helpers for HIP-vs-oracle parity checks (test infrastructure)."""
from __future__ import annotations

import numpy as np

from f16_jsb_amd.abi import (F16C_AI, F16C_AIP, F16C_BA, F16C_CMD, F16C_EP_COUNT, F16C_EP_RET,
                             F16C_EPA_C, F16C_GOAL, F16C_LX, F16C_N, F16C_Q, F16C_RI, F16C_STEP,
                             F16C_VI, F16C_VIH1, F16C_VIH2, F16C_WI, F16C_WID, F16C_WIND,
                             F16L_N)

FRAME_NAMES = ["lat*R", "lon*R", "h_m", "mach", "alpha", "beta", "p", "q", "r", "phi", "theta", "psi",
               "goal_x", "goal_y", "goal_z"]
ANGLE_COLS = (9, 10, 11)


def frame_err(a, b):
    """|a-b| per frame component (angles wrapped to [-pi, pi))."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    d = np.abs(a - b)
    for c in ANGLE_COLS:
        w = np.abs((a[..., c] - b[..., c] + np.pi) % (2 * np.pi) - np.pi)
        d[..., c] = w
    return d


def report(name, err):
    """Max error per frame component as a dict."""
    err = np.asarray(err)
    flat = err.reshape(-1, err.shape[-1])
    return {name + ":" + FRAME_NAMES[i]: float(flat[:, i].max()) for i in range(flat.shape[-1])}


# Canonical-state fields the two paths are compared on (the HIP path does not keep the last
# command or double-precision AB histories; those are excluded or compared loosely).
def state_err(gpu, ref):
    g = np.asarray(gpu, np.float64)
    r = np.asarray(ref, np.float64)
    out = {}
    out["rI_ft"] = np.abs(g[:, F16C_RI:F16C_RI + 3] - r[:, F16C_RI:F16C_RI + 3]).max()
    out["vI_fps"] = np.abs(g[:, F16C_VI:F16C_VI + 3] - r[:, F16C_VI:F16C_VI + 3]).max()
    out["q"] = np.abs(g[:, F16C_Q:F16C_Q + 4] - r[:, F16C_Q:F16C_Q + 4]).max()
    out["wI"] = np.abs(g[:, F16C_WI:F16C_WI + 3] - r[:, F16C_WI:F16C_WI + 3]).max()
    out["aI"] = np.abs(g[:, F16C_AI:F16C_AI + 3] - r[:, F16C_AI:F16C_AI + 3]).max()
    fcs = [c for c in range(33, 45) if c != 42]  # PID_P_P: not carried by the HIP path (kd = 0)
    out["fcs"] = np.abs(g[:, fcs] - r[:, fcs]).max()
    out["n2"] = np.abs(g[:, 46] - r[:, 46]).max()
    out["lx_alpha"] = np.abs(g[:, F16C_LX] - r[:, F16C_LX]).max()
    out["lx_mach"] = np.abs(g[:, F16C_LX + 2] - r[:, F16C_LX + 2]).max()
    out["lx_vc"] = np.abs(g[:, F16C_LX + 3] - r[:, F16C_LX + 3]).max()
    out["lx_npz"] = np.abs(g[:, F16C_LX + 9] - r[:, F16C_LX + 9]).max()
    return {k: float(v) for k, v in out.items()}
