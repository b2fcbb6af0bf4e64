/*
 * f16ref -- CPU fp64 restatement of the reference's hot path (the ORACLE).
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library; the product (libf16env.so) never links it.
 *
 * Parity status: JSBSim itself (the library behind jsbsim.FGFDMExec in the reference,
 * requirements.txt:4, unpinned version) is not available in this environment, and
 * importing the reference Python was denied. The FDM parts of this
 * oracle therefore restate JSBSim's published algorithms for the f16.xml model from
 * public knowledge: "JSBSim parity unpinned". The env layer (obs/reward/stack/reset)
 * follows jsbsim_gym/jsbsim_gym.py line by line and is pinned by tests/golden vectors.
 *
 * API mirrors include/f16env.h (same config struct and canonical-state layout) but all
 * arrays are HOST pointers.
 */
#ifndef F16REF_H
#define F16REF_H
#include "../include/f16env.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct f16ref f16ref;

f16ref* f16ref_create(const f16env_config* cfg);
void f16ref_destroy(f16ref* h);
int f16ref_n_envs(const f16ref* h);

int f16ref_reset(f16ref* h, const uint8_t* mask, const float* goals, const double* ic,
                 float* obs);
int f16ref_step(f16ref* h, const float* act, float* obs, float* rew, uint8_t* terminated,
                uint8_t* truncated, float* terminal_obs, double* ep_return, int32_t* ep_len);
int f16ref_get_state(const f16ref* h, double* canon);
int f16ref_set_state(f16ref* h, const double* canon);
int f16ref_trim(f16ref* h, const double* ic_in, double* ic_out, double* residual_out);
int f16ref_sample_actions(const f16ref* h, uint64_t seed, uint64_t step, float* act);
/* Philox4x32-10 (Salmon et al., SC'11), exposed for known-answer tests. */
void f16ref_philox4x32(const uint32_t key[2], const uint32_t ctr[4], uint32_t out[4]);
/* US-1976 standard atmosphere at geometric altitude h_ft:
 * out = {T_R, P_psf, rho_slugft3, a_fps}. */
void f16ref_atmosphere(double h_ft, double out[4]);
/* WGS84 helpers for known-answer tests. */
void f16ref_geodetic_to_ecef(double lat, double lon, double h_ft, double ecef[3]);
double f16ref_geodetic_altitude(const double ecef[3]);
/* Calibrated airspeed (kts) from Mach and static pressure (psf). */
double f16ref_vcas_kts(double mach, double p_psf);
/* Generic clamped table lookups over the generated tables, by aero-function index
 * (for table known-answer tests): returns the table value at (x, y). */
double f16ref_aero_table(int fn_index, double x, double y);
int f16ref_n_aero_fns(void);
/* TEST-ONLY physics switch (default 0 = full model; process-wide): bits drop the
 * aerodynamic forces/moments, the thrust, gravity, or gravity's J2 term, for analytic
 * invariant tests of the equations of motion. */
#define F16REF_PHYS_NO_AERO 0x1
#define F16REF_PHYS_NO_THRUST 0x2
#define F16REF_PHYS_NO_GRAVITY 0x4
#define F16REF_PHYS_NO_J2 0x8
/* not physics: a deliberate env-layer defect for negative controls (PositionReward over the
 * 2-D distance instead of the 3-D one, jsbsim_gym.py:496-500) */
#define F16REF_TEST_SHAPING_2D 0x10
void f16ref_set_physics_mask(int mask);
int f16ref_get_physics_mask(void);
void f16ref_mass_props(double J[9], double* mass);
/* FCS / engine components for unit tests: FGKinematic traverse (detents/times, n entries),
 * FGPID (integral / previous input updated in place), aerosurface_scale (zero-centred),
 * FGTurbine's rate-limited Seek. */
double f16ref_kinematic(double out, double in, const double* detents, const double* times, int n, double dt,
                        int ic);
double f16ref_pid(double in, double* integral, double* prev, double trigger, double kp, double ki, double kd,
                  double dt, int ic);
double f16ref_aero_scale(double in, double inmin, double inmax, double outmin, double outmax);
double f16ref_seek(double v, double target, double accel, double decel, double dt);
/* Number of OpenMP threads the batch loops use (1 if built without OpenMP). */
int f16ref_threads(void);
int f16ref_set_threads(int n);
uint64_t f16ref_obs_bounds_count(const f16ref* h);

#ifdef __cplusplus
}
#endif
#endif
