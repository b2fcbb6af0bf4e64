"""Python mirror of include/f16env.h (constants, config struct, defaults).

Pure ctypes/numpy: no torch, no library load. The defaults are the reference's constants
(jsbsim_gym/jsbsim_gym.py:56-58,157-170,532).
"""
from __future__ import annotations

import ctypes

F16ENV_ABI_VERSION = 6  # include/f16env.h (checked against f16env_abi_version() at load)
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
F16C_GUST = 72
F16C_N = 75

(F16L_ALPHA, F16L_BETA, F16L_MACH, F16L_VC_KTS, F16L_VG_FPS, F16L_P_AERO, F16L_Q_AERO,
 F16L_R_AERO, F16L_NPY, F16L_NPZ, F16L_N) = range(11)

F16_FLAG_NO_AUTORESET = 0x1
F16_FLAG_RANDOM_IC = 0x2  # cfg5: reset IC drawn from the [ic_lo, ic_hi] box
F16_FLAG_GUSTS = 0x4      # cfg5: Gauss-Markov gusts on top of the steady wind
F16_FLAG_NAN_GUARD = 0x8  # quarantine lanes whose frame goes non-finite (terminated = 3, counted)
F16_FLAG_OBS_CHECK = 0x10  # count lane-steps whose new frame has a finite value outside the obs space

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
        ("ic_lo", ctypes.c_double * F16_IC_N),
        ("ic_hi", ctypes.c_double * F16_IC_N),
        ("gust_sigma_fps", ctypes.c_double),
        ("gust_tau_s", ctypes.c_double),
    ]


def default_ic_values():
    ic = [0.0] * F16_IC_N
    ic[F16_IC_H_SL_FT] = 5000.0  # jsbsim_gym.py:170 ic/h-sl-ft
    ic[F16_IC_U_FPS] = 900.0     # jsbsim_gym.py:169 ic/u-fps
    return ic


def config_default(n_envs=1, stack_k=10, down_sample=4, max_steps=1200, flags=0,
                   dt=1.0 / 120.0, dg_m=100.0, goal_gain=1e-2, crash_alt_m=10.0, seed=0,
                   env_id_base=0, ic=None, cfg5=False) -> EnvConfig:
    """f16env_config_default with overrides; cfg5=True adds the BASELINE cfg5 random-IC box
    and gusts (config_cfg5)."""
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
        c.ic[i] = c.ic_lo[i] = c.ic_hi[i] = float(vals[i])
    c.gust_sigma_fps = 0.0
    c.gust_tau_s = 2.0
    if cfg5:
        config_cfg5(c)
    return c


# BASELINE cfg5 box (include/f16env.h f16env_config_cfg5; SURVEY.md 8c cfg5 ranges)
CFG5_BOX = {
    F16_IC_H_SL_FT: (3000.0, 30000.0),
    F16_IC_U_FPS: (600.0, 1200.0),
    F16_IC_PHI_RAD: (-0.17453292519943295, 0.17453292519943295),
    F16_IC_THETA_RAD: (-0.17453292519943295, 0.17453292519943295),
    F16_IC_PSI_RAD: (0.0, 6.283185307179586),
    F16_IC_CMD_THR: (0.3, 1.0),
    F16_IC_WIND_N_FPS: (-30.0, 30.0),
    F16_IC_WIND_E_FPS: (-30.0, 30.0),
}
CFG5_GUST_SIGMA_FPS = 10.0
CFG5_GUST_TAU_S = 2.0


def config_cfg5(c: EnvConfig) -> EnvConfig:
    """Python twin of f16env_config_cfg5: random-IC box + gusts on top of ``c``."""
    c.flags = int(c.flags) | F16_FLAG_RANDOM_IC | F16_FLAG_GUSTS
    for i in range(F16_IC_N):
        lo, hi = CFG5_BOX.get(i, (c.ic[i], c.ic[i]))
        c.ic_lo[i], c.ic_hi[i] = lo, hi
    c.gust_sigma_fps = CFG5_GUST_SIGMA_FPS
    c.gust_tau_s = CFG5_GUST_TAU_S
    return c


def algorithmic_bytes_per_env_step(stack_k: int, state_bytes: int, layout: str = "contiguous") -> int:
    """Bytes one env step must move. Contiguous stacks, SURVEY.md 8(d):
    B(K) = 16 + 60K + 60(K-1) + 4 + 2 + 2S (action, the new stack written, the previous K-1
    frames read, reward, flags, state read + written). Windowed observations
    (f16env_step_window): B_win = 16 + 2*60 + 4 + 2 + S + (S - 16), independent of K -- the
    new frame written to both histories, no frames read (a reset lane's fresh window aside), the
    state read whole and written back without its per-episode column (goal, episode count),
    which only a lane the step resets rewrites (round 5; ~0.1 % of lanes per step in the bench's
    steady state)."""
    if layout == "window":
        return 16 + 2 * 60 + 4 + 2 + 2 * state_bytes - 16
    if layout != "contiguous":
        raise ValueError("layout must be 'contiguous' or 'window'")
    return 16 + 60 * stack_k + 60 * (stack_k - 1) + 4 + 2 + 2 * state_bytes


F16_SLOT_CLIP = 0x1  # the env steps np.clip(act, low, high); the slot keeps act unclipped
F16_SLOT_FEATURE_WINDOW = 0x2  # the windowed rollout-slot step also updates the bound feature histories
F16_STEP_FEATURE_WINDOW = 0x2  # f16env_window_step_ex: the plain windowed step updates them too (ABI 4)
F16_STEP_POSES = 0x4  # f16env_window_step_ex: the step writes the bound N x 10 pose export (ABI 5)


class RolloutSlot(ctypes.Structure):
    """f16env_rollout_slot (include/f16env.h): one slot of a device rollout buffer filled by
    f16env_step_rollout / f16env_window_step_rollout; NULL pointers are not written."""
    _fields_ = [
        ("act_seed", ctypes.c_uint64),
        ("act_step", ctypes.c_uint64),
        ("frame", ctypes.c_void_p),
        ("actions", ctypes.c_void_p),
        ("rewards", ctypes.c_void_p),
        ("next_start", ctypes.c_void_p),
        ("features", ctypes.c_void_p),
        ("next_frame", ctypes.c_void_p),
        ("flags", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
    ]
