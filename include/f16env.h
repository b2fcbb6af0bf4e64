/*
 * f16env.h -- C ABI of the MI355X-native vectorised F-16 environment (libf16env.so).
 *
 * One handle = one device = N independent F-16 envs held as struct-of-arrays state in
 * HBM. Every array argument is a caller-owned DEVICE pointer (e.g. a PyTorch-ROCm
 * tensor's data_ptr()); `stream` is a hipStream_t (NULL = default stream). Calls are
 * stream-ordered and asynchronous unless documented otherwise. A handle is not
 * thread-safe. Errors: int status (0 ok, <0 error) + f16env_last_error() (thread-local).
 *
 * What each entry point replaces in the reference (Soham4001A/F16_JSB):
 *   f16env_create   <- jsbsim_gym/jsbsim_gym.py:122-164 JSBSimEnv.__init__ (FGFDMExec(root),
 *                      load_model('f16'), _set_initial_conditions :166-170, run_ic :155)
 *                      x N, plus stable_baselines3/common/vec_env/dummy_vec_env.py:30-50
 *   f16env_reset    <- jsbsim_gym.py:289-331 JSBSimEnv.reset + :511-519 PositionReward.reset,
 *                      vectorised as dummy_vec_env.py:75-83 DummyVecEnv.reset
 *   f16env_step     <- jsbsim_gym.py:199-287 JSBSimEnv.step (4x FGFDMExec.run() :225-232),
 *                      :487-509 PositionReward.step, gymnasium TimeLimit(1200) (:537-545),
 *                      common/monitor.py:85-111 Monitor.step and the auto-reset loop of
 *                      dummy_vec_env.py:56-73 DummyVecEnv.step_wait
 *   f16env_get_state/set_state <- FGFDMExec state (no reference equivalent; used for
 *                      parity replay and checkpoint/restore)
 *   f16env_trim     <- no reference equivalent (the reference never trims; BASELINE cfg 2)
 *   f16env_sample_actions <- action_space.sample() (jsbsim_gym.py:575), device Philox
 *   f16env_step_rollout <- f16env_step + buffers.py:440-479 RolloutBuffer.add (8f rank 1)
 *   f16env_window_step_rollout <- the same on windowed observations, with the policy's actions
 *                      clipped to the Box in-kernel (on_policy_algorithm.py:199-218)
 *   f16env_rollout_random / f16env_window_rollout_random <- on_policy_algorithm.py:194-262's
 *                      loop under the uniform random policy, one launch
 *   f16env_bootstrap_timeouts <- on_policy_algorithm.py:236-245 (timeout bootstrap)
 *   f16env_bootstrap_stash / f16env_bootstrap_apply <- the same, deferred to the end of the
 *                      rollout (one value evaluation over the stashed terminal observations)
 *   f16env_gae      <- stable_baselines3/common/buffers.py:403-438 (device rollout, 8f rank 1)
 *   f16env_features <- jsbsim_gym/features.py:37-67 JSBSimFeatureExtractor.forward (8f rank 3)
 *   f16env_features_window_step <- the same per step on a windowed observation, one frame each
 *   f16env_poses    <- jsbsim_gym.py:381-415 JSBSimEnv.render state -> Viewer poses (8f rank 4)
 */
#ifndef F16ENV_H
#define F16ENV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 3 (round 4): f16env_step_kernel_name takes the handle (was (void)); f16env_set_state keeps the
 * windowed layout's FRESH mark; the rollout slot gained next_frame / flags (F16_SLOT_CLIP);
 * f16env_rollout_random has no stack_k / mode limits; new f16env_window_step_rollout,
 * f16env_window_rollout_random, f16env_bootstrap_timeouts, f16env_bootstrap_stash,
 * f16env_bootstrap_apply, f16env_features_window_step, f16env_window_feature_bind
 * (+ F16_SLOT_FEATURE_WINDOW), f16env_abi_version.
 * 4 (round 5): new f16env_window_step_ex (in-step action draws, F16_STEP_FEATURE_WINDOW) and
 * f16env_window_step_ex_kernel_name; nothing else changed.
 * 5 (round 5): new F16_STEP_POSES flag and f16env_window_poses_bind; nothing else changed.
 * 6 (round 6): new f16env_sample_actions_steps and f16env_window_resets_deferred; nothing else
 * changed. */
#define F16ENV_ABI_VERSION 6

/* Frame layout (jsbsim_gym.py:12-25 STATE_FORMAT + goal, :172-197) */
#define F16_OBS_DIM 15
#define F16_ACT_DIM 4

/* Initial condition vector (per env), JSBSim "ic/" semantics (jsbsim_gym.py:166-170). */
enum f16_ic_index {
  F16_IC_LAT_GEOD_RAD = 0, /* geodetic latitude                         (default 0)    */
  F16_IC_LON_RAD,          /* longitude                                 (default 0)    */
  F16_IC_H_SL_FT,          /* altitude above the WGS84 ellipsoid        (5000)         */
  F16_IC_U_FPS,            /* body velocity wrt ECEF: u (ic/u-fps)     (900)          */
  F16_IC_V_FPS,            /*                          v                (0)            */
  F16_IC_W_FPS,            /*                          w                (0)            */
  F16_IC_PHI_RAD,          /* Euler angles wrt local NED                (0)            */
  F16_IC_THETA_RAD,
  F16_IC_PSI_RAD,
  F16_IC_P_RPS,            /* body rates wrt ECEF                       (0)            */
  F16_IC_Q_RPS,
  F16_IC_R_RPS,
  F16_IC_CMD_AIL,          /* FCS command properties held at IC         (0)            */
  F16_IC_CMD_ELE,
  F16_IC_CMD_RUD,
  F16_IC_CMD_THR,
  F16_IC_WIND_N_FPS,       /* steady wind NED (cfg5; the reference has none) (0)       */
  F16_IC_WIND_E_FPS,
  F16_IC_WIND_D_FPS,
  F16_IC_N
};

/* Canonical full per-env state (fp64 vector). Both the HIP path and the CPU oracle can
 * export/import it; the HIP path stores most of it in fp32 SoA. */
enum f16_canon_index {
  F16C_RI = 0,       /* 0-2   inertial position ECI (ft)                                */
  F16C_VI = 3,       /* 3-5   inertial velocity ECI (ft/s)                              */
  F16C_VIH1 = 6,     /* 6-8   AB3 history: inertial velocity one frame back            */
  F16C_VIH2 = 9,     /* 9-11  two frames back                                          */
  F16C_AI = 12,      /* 12-14 latest inertial acceleration (FGAccelerations vUVWidot)   */
  F16C_AIP = 15,     /* 15-17 AB2 history: previous inertial acceleration             */
  F16C_Q = 18,       /* 18-21 attitude quaternion ECI->body (q0 q1 q2 q3)              */
  F16C_WI = 22,      /* 22-24 body rates wrt ECI, body axes (vPQRi)                    */
  F16C_WID = 25,     /* 25-27 latest vPQRidot                                          */
  F16C_BA = 28,      /* 28-30 latest body specific-force acceleration (vBodyAccel); the  */
                     /* HIP path carries y, z (read by the next frame's pilot load      */
                     /* factors) and reports x as 0                                     */
  F16C_EPA_C = 31,   /* cos / sin of the Earth position angle                          */
  F16C_EPA_S = 32,
  F16C_TEF = 33,     /* fcs/tef-control            (kinematic, f16.xml:334-350)        */
  F16C_AIL = 34,     /* fcs/left-aileron-pos-norm  (kinematic, f16.xml:419-432)        */
  F16C_ELE = 35,     /* fcs/elevator-pos-norm      (kinematic, f16.xml:630-643)        */
  F16C_RUD = 36,     /* fcs/rudder-pos-norm        (kinematic, f16.xml:739-752)        */
  F16C_LEF = 37,     /* fcs/lef-control            (kinematic, f16.xml:831-843)        */
  F16C_SB = 38,      /* fcs/speedbrake-pos-deg     (kinematic, f16.xml:909-922)        */
  F16C_PID_R_I = 39, /* roll-rate-pid  (f16.xml:383-389): integrator, previous input   */
  F16C_PID_R_P = 40,
  F16C_PID_P_I = 41, /* g-load-pid     (f16.xml:594-604); kd = 0, so the HIP path does   */
                     /* not carry its previous input (PID_P_P reported as 0)            */
  F16C_PID_P_P = 42,
  F16C_PID_Y_I = 43, /* yaw-load-pid   (f16.xml:716-727)                               */
  F16C_PID_Y_P = 44,
  F16C_N1 = 45,      /* FGTurbine N1, N2 (%), augmentation flag. The HIP path does not   */
                     /* carry N1 (thrust under augmethod 2 reads N2 only; nothing        */
                     /* observes N1): reported as 0, ignored by set_state                */
  F16C_N2 = 46,
  F16C_AUG = 47,
  F16C_LX = 48,      /* 48-57 auxiliary latch read by the next frame's FCS:             */
                     /* alpha, beta, mach, vc_kts, vg_fps, p_aero, q_aero, r_aero,      */
                     /* n_pilot_y, n_pilot_z                                           */
  F16C_CMD = 58,     /* 58-61 fcs/{aileron,elevator,rudder,throttle}-cmd-norm          */
  F16C_GOAL = 62,    /* 62-64 goal (float32 values, jsbsim_gym.py:321-323)             */
  F16C_LAST_D = 65,  /* PositionReward.last_distance (float32)                         */
  F16C_STEP = 66,    /* JSBSimEnv.current_step                                          */
  F16C_EP_RET = 67,  /* Monitor episode return (sum of float64 rewards)                */
  F16C_EP_COUNT = 68,/* resets so far (keys the device goal RNG)                        */
  F16C_WIND = 69,    /* 69-71 steady wind NED (fps)                                     */
  F16C_GUST = 72,    /* 72-74 gust wind NED (fps), F16_FLAG_GUSTS (cfg5)                  */
  F16C_N = 75
};
enum f16_latch_index {
  F16L_ALPHA = 0, F16L_BETA, F16L_MACH, F16L_VC_KTS, F16L_VG_FPS,
  F16L_P_AERO, F16L_Q_AERO, F16L_R_AERO, F16L_NPY, F16L_NPZ, F16L_N
};

/* flags */
#define F16_FLAG_NO_AUTORESET 0x1 /* leave done lanes un-reset (caller resets)          */
/* BASELINE cfg5 (the reference has neither: it always resets to jsbsim_gym.py:166-170 and
 * never enables FGWinds). Build-defined models, documented in DESIGN.md:
 *   RANDOM_IC: every reset that is not given an explicit IC (auto-reset, f16env_reset with
 *     ic == NULL) draws ic[j] = ic_lo[j] + (ic_hi[j] - ic_lo[j]) * u_j, u_j = (w_j + 0.5) 2^-32,
 *     w_j word j of Philox4x32-10 keyed by (seed; gid, gid_hi, episode, 0x52494300 + j/4).
 *   GUSTS: per-lane first-order Gauss-Markov gust g (NED, fps) added to the steady wind:
 *     g_0 = sigma * xi_0 at reset, g_s = a g_{s-1} + sigma sqrt(1 - a^2) xi_s before the FDM
 *     frames of env step s, a = exp(-down_sample dt / tau); xi_s three Box-Muller normals
 *     from Philox keyed by (seed; gid, gid_hi ^ 0x47555354, episode, s). */
#define F16_FLAG_RANDOM_IC 0x2
#define F16_FLAG_GUSTS 0x4
/* Failure detection (the reference has none -- a non-finite JSBSim state just
 * propagates into the observation, jsbsim_gym.py:268-285 only prints): a lane whose new frame
 * has a non-finite position, Mach, alpha, beta or body rate ends that step as terminated with
 * reward 0 and terminated[i] = 3 (bit 1 marks the quarantine), is auto-reset like any finished
 * lane, and is counted (f16env_nonfinite_count). Off by default. */
#define F16_FLAG_NAN_GUARD 0x8
/* Observation-bounds diagnostic (jsbsim_gym.py:268-285: observation_space.contains(obs) and
 * the warning for FINITE values outside SINGLE_OBS_LOW / SINGLE_OBS_HIGH, :28-53): each step
 * checks the lane's new frame (the older K-1 frames were checked when they were new) and counts
 * the lanes with a finite component out of bounds (f16env_obs_bounds_count). Off by default;
 * changes nothing else. */
#define F16_FLAG_OBS_CHECK 0x10

typedef struct f16env_config {
  int32_t n_envs;       /* envs on this device                                          */
  int32_t stack_k;      /* frames per observation (reference NUM_STACKED_FRAMES=10 :58)  */
  int32_t down_sample;  /* FDM frames per env step (reference 4, :157)                   */
  int32_t max_steps;    /* truncation (reference 1200, :159 and TimeLimit :541)          */
  int32_t flags;
  int32_t reserved0;
  double dt;            /* FDM frame (JSBSim default 1/120 s)                           */
  double dg_m;          /* goal cylinder radius (reference 100 m, :163)                  */
  double goal_gain;     /* PositionReward gain (reference 1e-2, :532)                    */
  double crash_alt_m;   /* crash altitude (reference 10 m, :245)                         */
  uint64_t seed;        /* device RNG seed for auto-reset goals                          */
  int64_t env_id_base;  /* global id of local env 0 (multi-GPU shards key the RNG by it) */
  double ic[F16_IC_N];  /* default initial condition                                    */
  double ic_lo[F16_IC_N]; /* F16_FLAG_RANDOM_IC box, per IC component (lo == hi: fixed)    */
  double ic_hi[F16_IC_N];
  double gust_sigma_fps;  /* F16_FLAG_GUSTS: stationary std-dev per NED axis              */
  double gust_tau_s;      /*                 correlation time                              */
} f16env_config;

typedef struct f16env* f16env_t;

/* Fill *cfg with the reference's defaults (n_envs=1, K=10, down_sample=4, ...). */
int f16env_config_default(f16env_config* cfg);
/* BASELINE cfg5 on top of *cfg: sets F16_FLAG_RANDOM_IC | F16_FLAG_GUSTS and the build's
 * box (u 600..1200 fps, h 3000..30000 ft, psi 0..2pi, theta/phi +-10 deg, steady wind N/E
 * +-30 fps, throttle cmd 0.3..1) and gusts (sigma 10 fps, tau 2 s); other components
 * keep cfg->ic. */
int f16env_config_cfg5(f16env_config* cfg);

/* Create a handle on `device`; allocates the SoA state (no per-step allocation later). */
int f16env_create(const f16env_config* cfg, int device, f16env_t* out);
int f16env_destroy(f16env_t h);

/* Step kernel family of the handle: bit 0 random IC, bit 1 wind (cfg5 gusts, or lanes that
 * can carry steady wind: config IC / random-IC box wind, or set by f16env_set_state). */
int f16env_step_mode(f16env_t h);

/* Bytes of device state held by the handle (the SoA state, plus cfg5 modes' reset cache of
 * 336 B per env) / persistent bytes per env a step moves (roofline S: 256 B, +32 B for the wind
 * kernels' steady-wind and gust columns). */
size_t f16env_state_bytes(f16env_t h);
int f16env_state_bytes_per_env(void);

/* Reset the lanes where mask[i] != 0 (mask NULL = all).
 *   goals: N x 3 float (x, y, alt in m) or NULL -> device Philox goal RNG; a row whose x is
 *          NaN also takes the device goal (seeded and unseeded lanes in one call)
 *   ic:    N x F16_IC_N double or NULL -> the config's default IC (template copy)
 *   obs:   N x K x 15 float; rows of reset lanes are written (K copies of frame 0).
 * With a per-lane ic on a handle without the wind kernels the call waits for `stream` to read
 * back whether any lane got wind (and switches the handle to the wind kernels if so). */
int f16env_reset(f16env_t h, void* stream, const uint8_t* mask, const float* goals,
                 const double* ic, float* obs);

/* One env step for all N lanes.
 *   act          N x 4 float (aileron, elevator, rudder, throttle cmd; NOT clipped,
 *                as jsbsim_gym.py:216-222)
 *   obs_prev     N x K x 15 float, the previous observation (may equal obs)
 *   obs          N x K x 15 float output (reset obs for lanes that finished)
 *   rew          N float; terminated / truncated N uint8
 *   terminal_obs N x K x 15 float; only rows of finished lanes are written (may be NULL)
 *   ep_return    N double; ep_len N int32: valid where the lane finished (may be NULL)
 *   done_idx     N int32 + n_done (1 int32): compacted list of finished lanes, unordered
 *                (may be NULL; n_done must be zeroed by the callee -- it is) */
int f16env_step(f16env_t h, void* stream, const float* act, const float* obs_prev, float* obs,
                float* rew, uint8_t* terminated, uint8_t* truncated, float* terminal_obs,
                double* ep_return, int32_t* ep_len, int32_t* done_idx, int32_t* n_done);

/* Windowed observations: the same env step without the stack shift copy (the "state-stacking
 * ring buffer" of BASELINE.json north_star: JSBSimEnv's `obs_buffer` deque(maxlen=K),
 * jsbsim_gym.py:150 and its append at :235, and DummyVecEnv's stacked obs buffer,
 * dummy_vec_env.py:56-73). The caller owns two frame histories of T positions, position-major,
 * hist[b] = T x N x 16 float (per env a 15-float frame + one 0: 64-B slots, the N slots of a
 * position contiguous; T >= 2K). The observation of a step is the window
 *     hist_cur[pos-K+1 .. pos][k][0..15)      (a strided N x K x 15 view: strides 16, N*16, 1)
 * with identical values to f16env_step's obs. A step writes only its new frame, one whole
 * 64-B slot at `pos` of both histories (reset lanes also fill their window), alternating hist_cur / hist_other
 * between steps (pos advancing by one); the terminal observation of a lane that finished is
 * the same window of hist_other (no copy; valid until the next step, like terminal_obs).
 * The other parity's window is not written, so an observation stays valid until the step
 * after next. When pos would reach T, f16env_window_restart moves the last K-1 frames to the
 * front and the next step uses pos = K-1. Other arguments as f16env_step. */
int f16env_step_window(f16env_t h, void* stream, const float* act, float* hist_cur, float* hist_other,
                       int64_t T, int32_t pos, float* rew, uint8_t* terminated, uint8_t* truncated,
                       double* ep_return, int32_t* ep_len, int32_t* done_idx, int32_t* n_done);
/* f16env_step_window with the handle's buffers bound once (a per-step call of five arguments:
 * the host cost of a step is the launch, not the argument marshalling). hist_cur = hist[parity],
 * hist_other = hist[parity ^ 1]; the pointers must stay valid while bound. */
int f16env_window_bind(f16env_t h, float* hist0, float* hist1, int64_t T, float* rew, uint8_t* terminated,
                       uint8_t* truncated, double* ep_return, int32_t* ep_len);
int f16env_window_step_bound(f16env_t h, void* stream, const float* act, int32_t parity, int32_t pos);
/* The two feature histories ([T][N][17] float32, parity 0 and 1; T as f16env_window_bind) that
 * rollout-slot steps with F16_SLOT_FEATURE_WINDOW and f16env_window_step_ex with
 * F16_STEP_FEATURE_WINDOW update (NULL, NULL: unbind). */
int f16env_window_feature_bind(f16env_t h, float* feat0, float* feat1);
/* ABI 4. f16env_window_step_bound with extras, in a kernel instance of its own
 * (f16_step_winx_kernel; the plain step's instance carries none of this code):
 *   act == NULL  the actions are drawn in the step from the f16env_sample_actions stream
 *                (act_seed; env id, act_step): bit-identical to f16env_sample_actions followed by
 *                f16env_window_step_bound, without the sampling launch or the action read
 *                (jsbsim_gym.py's action_space.sample() per env, as a device stream);
 *   flags F16_STEP_FEATURE_WINDOW  the step also brings the feature histories bound by
 *                f16env_window_feature_bind to its new position (features.py:37-67 of the new
 *                frame, LMA_features.py:757-765's per-frame transform, written from the frame in
 *                registers: no second launch), exactly as F16_SLOT_FEATURE_WINDOW does in a
 *                rollout-slot step; same precondition (both feature windows current before the
 *                step). Refused with the deferred-reset step (F16ENV_ICC_PERIOD=0).
 *   flags F16_STEP_POSES (ABI 5)  the step also writes the render/telemetry pose of the returned
 *                observation's newest frame per env into the N x 10 buffer bound by
 *                f16env_window_poses_bind -- f16env_poses of that frame (JSBSimEnv.render,
 *                jsbsim_gym.py:381-415), the same bits, without the second launch. Refused with
 *                the deferred-reset step (F16ENV_ICC_PERIOD=0).
 * With act != NULL and flags 0 it is f16env_window_step_bound. */
#define F16_STEP_FEATURE_WINDOW 0x2
#define F16_STEP_POSES 0x4
/* The N x 10 float32 pose buffer F16_STEP_POSES steps write (16-B aligned for whole-line stores;
 * NULL: unbind). Replaces nothing in the reference (a render callback's input, see f16env_poses). */
int f16env_window_poses_bind(f16env_t h, float* poses);
int f16env_window_step_ex(f16env_t h, void* stream, const float* act, int32_t parity, int32_t pos, uint32_t flags,
                          uint64_t act_seed, uint64_t act_step);
/* The kernel instance f16env_window_step_ex launches for `flags` (as rocprofv3 demangles it). */
const char* f16env_window_step_ex_kernel_name(f16env_t h, uint32_t flags);
/* f16env_reset for windowed observations: K copies of frame 0 into hist_cur's window ending at
 * pos (mask / goals / ic as f16env_reset; jsbsim_gym.py:289-331 x N). */
int f16env_reset_window(f16env_t h, void* stream, const uint8_t* mask, const float* goals, const double* ic,
                        float* hist_cur, int64_t T, int32_t pos);
/* Frames pos_old-K+2 .. pos_old of both histories -> 0 .. K-2 (pos_old = T-1 in practice). */
int f16env_window_restart(f16env_t h, void* stream, float* hist0, float* hist1, int64_t T, int32_t pos_old);
/* History order of this handle's windowed calls: 0 (default) position-major T x N x 16 as
 * above; 1 env-major N x T x 16 (view strides T*16, 16, 1). Set before the first windowed call
 * and keep it: the histories must be laid out accordingly. */
int f16env_set_window_order(f16env_t h, int env_major);
/* The caller has written whole observation windows into both histories (e.g. an observation
 * copied in after f16env_set_state): lanes reset since the last step stop refilling their next
 * window from the reset frame. (A reset marks its lanes so that the next windowed step fills
 * the other history's window; f16env_set_state keeps that mark.) */
int f16env_window_clear_fresh(f16env_t h, void* stream);
/* Waves per SIMD the windowed step kernel of this handle is built for (1 or 2), and whether it
 * is the non-temporal-store build (1: the whole grid resident in one round of waves). */
int f16env_step_window_waves_per_simd(f16env_t h);
int f16env_step_window_nt(f16env_t h);
/* ABI 6. 1 when this handle's windowed step leaves its finished lanes to the deferred reset
 * kernel that runs after it (cfg5 modes with F16ENV_ICC_PERIOD=0), 0 when the step resets them
 * itself (the reference task's template reset, cfg5's reset cache) or nobody does
 * (F16_FLAG_NO_AUTORESET). The epilogue extras of f16env_window_step_ex (F16_STEP_POSES,
 * F16_STEP_FEATURE_WINDOW) and the rollout slot's next_frame / features are refused while it
 * reads 1 (they would describe the pre-reset window); the Python front end refuses fused_poses /
 * fused_features handles at construction by it. <0 on a NULL handle. */
int f16env_window_resets_deferred(f16env_t h);

/* One env step that also fills one slot of a device rollout buffer (SURVEY.md 8f rank 1,
 * replacing the per-step stable_baselines3 RolloutBuffer.add, buffers.py:440-479, and the
 * action sampling / clipping of collect_rollouts, on_policy_algorithm.py:194-218, with no
 * extra launch). Every pointer of the slot may be NULL (not written):
 *   frame      N x 15 float: newest frame of obs_prev, i.e. of the observation acted on
 *              (frame-deduplicated storage; f16_jsb_amd/rollout.py rebuilds stacks).
 *              Contiguous layout only (f16env_step_rollout).
 *   next_frame N x 15 float: newest frame of the RETURNED observation (the next slot's frame;
 *              the reset frame where the lane finished). Windowed layout only
 *              (f16env_window_step_rollout): written from the same LDS staging as the window.
 *   actions    N x 4 float: the actions as given (SB3 stores the unclipped policy output,
 *              on_policy_algorithm.py:247-254)
 *   rewards    N float: the step's rewards (same values as rew)
 *   next_start N float: 1.0 where the lane finished (episode_starts of the NEXT slot), else 0
 *   features   N x K x 17 float: policy features of the returned observation (below)
 *   flags      F16_SLOT_CLIP: the env steps np.clip(act, low, high) over the action Box
 *              (on_policy_algorithm.py:216; numpy's clip ufunc semantics, NaN passes), while
 *              `actions` keeps act unclipped; F16_SLOT_FEATURE_WINDOW (windowed layout, ABI 3):
 *              the step also updates the feature histories bound by f16env_window_feature_bind
 *              exactly as f16env_features_window_step (transform 1) would after it -- the
 *              feature window in the step's epilogue, no second launch; the caller keeps the
 *              same precondition (both feature windows current before the step)
 * act == NULL draws the actions in-kernel from the f16env_sample_actions stream
 * (act_seed, act_step), bit-identical to f16env_sample_actions followed by f16env_step. */
#define F16_SLOT_CLIP 0x1
#define F16_SLOT_FEATURE_WINDOW 0x2
typedef struct f16env_rollout_slot {
  uint64_t act_seed, act_step;
  float* frame;
  float* actions;
  float* rewards;
  float* next_start;
  float* features;  /* N x K x 17: policy features of the returned obs (features.py:37-67, as
                       f16env_features), by a second launch in the same call (an epilogue
                       fused into the step kernel measured slower: +9.5 vs +9 us) */
  float* next_frame;
  uint32_t flags;
  uint32_t reserved;
} f16env_rollout_slot;
int f16env_step_rollout(f16env_t h, void* stream, const f16env_rollout_slot* slot, const float* act,
                        const float* obs_prev, float* obs, float* rew, uint8_t* terminated, uint8_t* truncated,
                        float* terminal_obs, double* ep_return, int32_t* ep_len, int32_t* done_idx,
                        int32_t* n_done);

/* f16env_step_rollout on windowed observations, with the buffers bound by f16env_window_bind
 * (parity / pos as f16env_window_step_bound). slot->frame must be NULL (the window layout
 * writes next_frame); slot->features reads the returned window in place. */
int f16env_window_step_rollout(f16env_t h, void* stream, const f16env_rollout_slot* slot, const float* act,
                               int32_t parity, int32_t pos);

/* T env steps of every lane in ONE launch under the uniform random policy (the actions are the
 * f16env_sample_actions stream (seed; env id, step0 + t)): SURVEY.md 8f rank 1's rollout with
 * the policy network out of scope. The state stays in registers for the whole rollout; per step
 * only the rollout slot is written:
 *   frames     T x N x 15  newest frame of the observation acted on at step t (frames[0]: of
 *                          obs_prev; frames[t+1] is written by step t)
 *   actions    T x N x 4   rewards T x N
 *   next_start (T-1) x N   1.0 where the lane finished at step t (episode_starts of slot t+1)
 *   last_start N           the same for step T-1
 * obs_prev / obs: N x K x 15 before step 0 / after step T-1 (distinct buffers; the final stack
 * is rebuilt from the frame log). The same actions and episode starts, frames and rewards as T
 * calls of f16env_step_rollout(seed, step0 + t, ...) (bit-identical). Any stack_k, the cfg5
 * modes included (a lane's first reset in the rollout comes from the reset cache, later ones
 * run their RunIC in the kernel); auto-reset on. Replaces on_policy_algorithm.py:194-262's loop
 * for that policy. */
int f16env_rollout_random(f16env_t h, void* stream, uint64_t seed, uint64_t step0, int32_t T,
                          const float* obs_prev, float* obs, float* frames, float* actions,
                          float* rewards, float* next_start, float* last_start);
/* The same on the bound window histories: the observation before step 0 is hist[parity]'s
 * window ending at pos, the final observation is written into BOTH histories' windows ending at
 * pos_out (which must not overlap the input window), so the next windowed step continues from
 * parity `parity`, position pos_out, with no lane needing a fresh-window fill. (No terminal
 * observation is produced for the last step's finished lanes.) */
int f16env_window_rollout_random(f16env_t h, void* stream, uint64_t seed, uint64_t step0, int32_t T,
                                 int32_t parity, int32_t pos, int32_t pos_out, float* frames, float* actions,
                                 float* rewards, float* next_start, float* last_start);

/* on_policy_algorithm.py:236-245 (timeout bootstrap, SB3 issue #633) over a device batch:
 * rewards[i] += gamma * terminal_values[i] where truncated[i] && !terminated[i], float32 with
 * SB3's rounding (f32(gamma) * v, then the sum). In place; stream-ordered; no handle needed. */
int f16env_bootstrap_timeouts(void* stream, int64_t n, float* rewards, const uint8_t* terminated,
                              const uint8_t* truncated, const float* terminal_values, double gamma);

/* The timeout bootstrap deferred to the end of a rollout. SB3 evaluates V(terminal_obs) lane by
 * lane inside the step loop (on_policy_algorithm.py:236-245); the value network does not change
 * during a rollout, so the evaluation can wait until the loop is done and run once over every
 * terminal observation that needs it, instead of over the whole batch at every step.
 * f16env_bootstrap_stash (once per step, after it): every lane i < n with truncated[i] &&
 * !terminated[i] appends its terminal observation -- K frames of 15 floats, frame j at
 * tobs + i * row_stride + j * frame_stride (floats; the contiguous (N, K, 15) layout or a window
 * view) -- to stash_obs (capacity x K x 15) and flat_base + i to stash_idx, at a slot taken from
 * *count (a wave-aggregated atomic add); slots at or past `capacity` are counted, not written
 * (the caller checks *count <= capacity). f16env_bootstrap_apply (after the rollout):
 * rewards[idx[j]] += f32(gamma) * values[j] for j < m (SB3's rounding, as
 * f16env_bootstrap_timeouts), the idx distinct. */
int f16env_bootstrap_stash(void* stream, int64_t n, int32_t K, const float* tobs, int64_t row_stride,
                           int64_t frame_stride, const uint8_t* terminated, const uint8_t* truncated,
                           int64_t flat_base, float* stash_obs, int64_t* stash_idx, int32_t* count,
                           int64_t capacity);
int f16env_bootstrap_apply(void* stream, int64_t m, float* rewards, const int64_t* idx, const float* values,
                           double gamma);

/* F16ENV_ABI_VERSION of the built library (a binding checks it against its header). */
int f16env_abi_version(void);

/* Lanes quarantined by F16_FLAG_NAN_GUARD since create (waits for `stream`). */
int f16env_nonfinite_count(f16env_t h, void* stream, uint64_t* count);
/* Debug build (libf16env_debug.so, compiled with F16_DEBUG_CHECKS): the bits of
 * the index / range invariants the kernels found violated since the library was loaded
 * (f16_device.h DebugBits; waits for `stream`). Returns 1 in the debug build, 0 (and
 * *violations = 0) in the product build, which carries no checks. */
int f16env_debug_checks(f16env_t h, void* stream, uint32_t* violations);
/* Lane-steps whose new observation frame had a finite value outside the observation space
 * since create (F16_FLAG_OBS_CHECK; waits for `stream`). */
int f16env_obs_bounds_count(f16env_t h, void* stream, uint64_t* count);

/* Canonical state export/import: canon is N x F16C_N double (device). The latch's p/q/r-aero
 * and ground speed are recomputed from the state on import (they are functions of it);
 * set_state waits for `stream` (it reads back whether any lane carries wind). The windowed
 * layout's per-lane "reset since the last step" mark is not part of the canonical state and
 * is kept by set_state (see f16env_window_clear_fresh). */
int f16env_get_state(f16env_t h, void* stream, double* canon);
int f16env_set_state(f16env_t h, void* stream, const double* canon);

/* Trim each lane for steady wings-level flight at ic[F16_IC_H_SL_FT], ic[F16_IC_U_FPS]
 * (interpreted as true airspeed, fps) and write the resulting IC (alpha folded into
 * theta/u/w, trim commands in F16_IC_CMD_*) to ic_out (N x F16_IC_N double, device).
 * residual_out (N x 3 double, may be NULL): |udot|, |wdot|, |qdot| after the solve. */
int f16env_trim(f16env_t h, void* stream, const double* ic_in, double* ic_out,
                double* residual_out);

/* Uniform actions over the Box [-1,-1,-1,0]..[1,1,1,1] from Philox4x32-10 keyed by
 * (seed; global env id, step). act: N x 4 float. */
int f16env_sample_actions(f16env_t h, void* stream, uint64_t seed, uint64_t step, float* act);
/* ABI 6. T batches in one launch: act = T x N x 4 float (16-B aligned), act[t] the batch
 * f16env_sample_actions(seed, step0 + t) draws, bit for bit (a caller pre-generating a run's
 * actions -- bench.py -- makes one launch instead of T). */
int f16env_sample_actions_steps(f16env_t h, void* stream, uint64_t seed, uint64_t step0, int32_t T, float* act);

/* GAE(lambda) advantages and returns over a device rollout laid out [n_steps][n_envs]
 * (float32; episode_starts as 0/1 float, dones uint8 for the step after the last), restating
 * stable_baselines3/common/buffers.py:403-438 RolloutBuffer.compute_returns_and_advantage
 * bit for bit (numpy float32 per-operation rounding). No handle needed. */
int f16env_gae(void* stream, int64_t n_steps, int64_t n_envs, const float* rewards, const float* values,
               const float* episode_starts, const float* last_values, const uint8_t* dones, double gamma,
               double gae_lambda, float* advantages, float* returns);

/* Policy features of every observation frame, replacing
 * jsbsim_gym/features.py:37-67 JSBSimFeatureExtractor.forward (float32):
 *   obs  n_frames x 15 float (any (..., 15) block, e.g. the N x K x 15 stack)
 *   feat n_frames x 17 float: [1/(1+d/1000), dz/15000, h/15000, mach, p, q, r,
 *        cos a, cos b, sin a, sin b, cos phi, cos theta, sin phi, sin theta, cos rb, sin rb]
 *        with d = |goal - pos|_xy, dz = goal_z - h, rb = atan2(dy, dx) - psi.
 * No handle needed; stream-ordered. */
int f16env_features(void* stream, int64_t n_frames, const float* obs, float* feat);

/* f16env_features on a strided (B, K, 15) block: frame (b, k) at obs + b*row_stride +
 * k*frame_stride (floats, any non-negative strides), e.g. a windowed observation read in
 * place (row_stride 16, frame_stride N*16); feat is (B, K, 17) contiguous. */
int f16env_features_strided(void* stream, int64_t n_rows, int32_t K, const float* obs, int64_t row_stride,
                            int64_t frame_stride, float* feat);

/* Feature window (ABI 3, windowed layout): keeps the features of the observation window in two
 * position-major feature histories feat_cur / feat_other ([T][N][17] float32, parity as the
 * frame histories) after a windowed step that wrote position `pos` of hist_cur (strides in
 * floats), transforming only that position's frames: feat_cur[pos] = feat_other[pos] =
 * features of hist_cur[pos]; lanes the step reset (terminated | truncated, autoreset != 0)
 * also fill feat_cur[pos-K+1 .. pos-1] and, ahead of the next step's window fill,
 * feat_other[pos-K+2 .. pos]. Precondition: both feature windows [pos-K .. pos-1] hold the
 * previous call's result (a fresh start: f16env_features_strided over both windows after a
 * step, then this call with transform = 0, which makes only the ahead fills). Replaces the
 * per-step f16env_features_strided over the whole (N, K, 15) view (features.py:37-67 per
 * frame, LMA_features.py:757-765 over the stack). */
int f16env_features_window_step(void* stream, int64_t n, int32_t K, int32_t pos, const float* hist_cur,
                                int64_t pos_stride, int64_t env_stride, float* feat_cur, float* feat_other,
                                const uint8_t* terminated, const uint8_t* truncated, int32_t autoreset,
                                int32_t transform);

/* Render/telemetry poses, replacing the state -> Viewer transform of
 * jsbsim_gym.py:381-415 (JSBSimEnv.render) for every env at once, float32:
 *   frames  n frames of 15 floats, frame i at frames + i * frame_stride (e.g. the newest frame
 *           of an N x K x 15 stack: frames = obs + 15 (K-1), frame_stride = 15 K)
 *   out     n x 10 float: aircraft position in viewer axes (-y, h, x) * 1e-3, attitude
 *           quaternion Quaternion.from_euler(phi, theta, psi) remapped to (w, -y, -z, x), goal
 *           position in viewer axes (-gy, gz, gx) * 1e-3. */
int f16env_poses(void* stream, int64_t n, const float* frames, int64_t frame_stride, float* out);

/* Name of the step kernel instance the handle launches (for profilers: the symbol rocprofv3
 * reports), e.g. "f16_step_win_nt_kernel<0, 1>" once f16env_window_bind was called (windowed
 * layout), else the contiguous-layout instance; it changes when set_state / a per-lane IC
 * switches the handle to the wind kernels. And the algorithmic HBM bytes one env-step moves
 * (SURVEY.md 8d B(K)). */
const char* f16env_step_kernel_name(f16env_t h);
/* Waves per SIMD the handle's step kernel is built for: 1 (up to 64 x 4 x CUs envs), or 2
 * when there are more waves than SIMDs (override: env F16ENV_OCC=1|2 at create). */
int f16env_step_waves_per_simd(f16env_t h);
/* Step kernel variant of the handle: 0 = tables in LDS, one wave per SIMD; 1 = tables in LDS,
 * two waves per SIMD; 2 = tables read from global memory (L1/L2) so that the K-frame stack
 * image alone fills LDS (large K, e.g. the reference's K = 10; override: env F16ENV_GT=0|1). */
int f16env_step_variant(f16env_t h);
double f16env_algorithmic_bytes_per_env_step(int stack_k);

/* Kernel-duration profiling of the step: after f16env_profile_begin(h, n) the next n step
 * launches of the handle record start/stop events from their own dispatch packets
 * (hipExtLaunchKernel), i.e. the kernel's execution without the dependent-launch boundary;
 * f16env_profile_end waits for them and returns the average / minimum duration (ms) and the
 * number of launches timed. Used by bench.py for the roofline's kernel time (rocprofv3's
 * kernel-trace average measures the same interval). */
int f16env_profile_begin(f16env_t h, int max_launches);
int f16env_profile_end(f16env_t h, double* avg_ms, double* min_ms, int* launches);
/* Between f16env_profile_begin and _end: the start / stop time (ms) of each profiled launch
 * relative to the first launch's start, t_ms[2i] / t_ms[2i+1] (waits for them). Returns the
 * number of launches filled (<= max_launches), so gaps between launches can be read off. */
int f16env_profile_times(f16env_t h, double* t_ms, int max_launches);

const char* f16env_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* F16ENV_H */
