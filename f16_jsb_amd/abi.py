"""Python mirror of include/f16env.h (constants, config struct, defaults).

Pure ctypes/numpy: no torch, no library load. The defaults are the reference's constants
(jsbsim_gym/jsbsim_gym.py:56-58,157-170,532).
"""
from __future__ import annotations

import ctypes

F16ENV_ABI_VERSION = 1
F16_OBS_DIM = 15
F16_ACT_DIM = 4

(F16_IC_LAT_GEOD_RAD, F16_IC_LON_RAD, F16_IC_H_SL_FT, F16_IC_U_FPS, F16_IC_V_FPS, F16_IC_W_FPS,
 F16_IC_PHI_RAD, F16_IC_THETA_RAD, F16_IC_PSI_RAD, F16_IC_P_RPS, F16_IC_Q_RPS, F16_IC_R_RPS,
 F16_IC_CMD_AIL, F16_IC_CMD_ELE, F16_IC_CMD_RUD, F16_IC_CMD_THR,
 F16_IC_WIND_N_FPS, F16_IC_WIND_E_FPS, F16_IC_WIND_D_FPS, F16_IC_N) = range(20)

F16C_RI, F16C_VI, F16C_VIH1, F16C_VIH2, F16C_AI, F16C_AIP = 0, 3, 6, 9, 12, 15
F16C_Q, F16C_WI, F16C_WID, F16C_BA = 18, 22, 25, 28
F16C_EPA_C, F16C_EPA_S = 31, 32
F16C_TEF, F16C_AIL, F16C_ELE, F16C_RUD, F16C_LEF, F16C_SB = 33, 34, 35, 36, 37, 38
F16C_PID_R_I, F16C_PID_R_P, F16C_PID_P_I, F16C_PID_P_P, F16C_PID_Y_I, F16C_PID_Y_P = range(39, 45)
F16C_N1, F16C_N2, F16C_AUG = 45, 46, 47
F16C_LX = 48
F16C_CMD = 58
F16C_GOAL = 62
F16C_LAST_D, F16C_STEP, F16C_EP_RET, F16C_EP_COUNT = 65, 66, 67, 68
F16C_WIND = 69
F16C_N = 72

(F16L_ALPHA, F16L_BETA, F16L_MACH, F16L_VC_KTS, F16L_VG_FPS, F16L_P_AERO, F16L_Q_AERO,
 F16L_R_AERO, F16L_NPY, F16L_NPZ, F16L_N) = range(11)

F16_FLAG_NO_AUTORESET = 0x1

# jsbsim_gym.py:28-53 observation bounds (per frame)
EPSILON = 1e-5


class EnvConfig(ctypes.Structure):
    _fields_ = [
        ("n_envs", ctypes.c_int32),
        ("stack_k", ctypes.c_int32),
        ("down_sample", ctypes.c_int32),
        ("max_steps", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("reserved0", ctypes.c_int32),
        ("dt", ctypes.c_double),
        ("dg_m", ctypes.c_double),
        ("goal_gain", ctypes.c_double),
        ("crash_alt_m", ctypes.c_double),
        ("seed", ctypes.c_uint64),
        ("env_id_base", ctypes.c_int64),
        ("ic", ctypes.c_double * F16_IC_N),
    ]


def default_ic_values():
    ic = [0.0] * F16_IC_N
    ic[F16_IC_H_SL_FT] = 5000.0  # jsbsim_gym.py:170 ic/h-sl-ft
    ic[F16_IC_U_FPS] = 900.0     # jsbsim_gym.py:169 ic/u-fps
    return ic


def config_default(n_envs=1, stack_k=10, down_sample=4, max_steps=1200, flags=0,
                   dt=1.0 / 120.0, dg_m=100.0, goal_gain=1e-2, crash_alt_m=10.0, seed=0,
                   env_id_base=0, ic=None) -> EnvConfig:
    c = EnvConfig()
    c.n_envs = int(n_envs)
    c.stack_k = int(stack_k)          # NUM_STACKED_FRAMES (:58)
    c.down_sample = int(down_sample)  # (:157)
    c.max_steps = int(max_steps)      # (:159, TimeLimit :541)
    c.flags = int(flags)
    c.dt = float(dt)                  # JSBSim default frame
    c.dg_m = float(dg_m)              # (:163)
    c.goal_gain = float(goal_gain)    # (:532)
    c.crash_alt_m = float(crash_alt_m)  # (:245)
    c.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    c.env_id_base = int(env_id_base)
    vals = default_ic_values() if ic is None else list(ic)
    for i in range(F16_IC_N):
        c.ic[i] = float(vals[i])
    return c


def algorithmic_bytes_per_env_step(stack_k: int, state_bytes: int) -> int:
    """B(K) = 16 + 60K + 60(K-1) + 4 + 2 + 2S."""
    return 16 + 60 * stack_k + 60 * (stack_k - 1) + 4 + 2 + 2 * state_bytes
