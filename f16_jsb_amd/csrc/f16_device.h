// f16_device.h -- per-lane F-16 flight dynamics for CDNA4 (gfx950), one lane per env.
//
// The path restated here is the one behind jsbsim.FGFDMExec.run() in the reference
// (jsbsim_gym/jsbsim_gym.py:225-232): FCS (aircraft/f16/f16.xml:309-984), FGTurbine
// (Engines/F100-PW-229.xml), aerodynamics (f16.xml:986-1917), US-1976 atmosphere, WGS84/J2
// gravity, 6-DoF equations of motion with JSBSim's default integrators. The CPU oracle
// (oracle/f16ref.c) is the readable fp64 statement of the same algorithm; this file is the
// fp32 register-resident version with fp64 kept only where fp32 cannot hold the precision
// (ECI position/velocity at |r| ~ 2.1e7 ft, the Earth rotation angle and the geodetic
// altitude). Tables live in LDS (f16_tables.h blob, grouped by shared breakpoint vectors);
// breakpoints are compile-time literals.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/f16env.h"
#include "f16_tables.h"

namespace f16 {

// Debug build (-DF16_DEBUG_CHECKS, build.py debug=True -> libf16env_debug.so):
// index / range invariants the kernels rely on are checked at run time and violations are
// recorded as bits of a device word (f16env_debug_checks reads it). A check never traps: a
// fault or abort on the GPU box would take the box down, a recorded bit fails a test instead.
// The product build compiles every F16_CHECK to nothing.
enum DebugBits {
  DBG_STATE_INDEX = 1,    // a lane index outside [0, n) reached a state access
  DBG_WINDOW_POS = 2,     // a window slot position outside [0, T)
  DBG_DONE_LIST = 4,      // the compacted done list overran N entries
  DBG_TABLE_SEGMENT = 8,  // a table bracket outside its breakpoint vector
  DBG_RESET_INDEX = 16,   // a deferred-reset list entry outside [0, n)
  DBG_RING_SLOT = 32,     // a rollout ring slot outside [0, K)
  DBG_FRAME_INDEX = 64,   // a features / poses frame index outside the block
};
#ifdef F16_DEBUG_CHECKS
__device__ unsigned int g_f16_violations;
#define F16_CHECK(cond, bit)                                   \
  do {                                                         \
    if (!(cond)) atomicOr(&::f16::g_f16_violations, (bit));    \
  } while (0)
#else
#define F16_CHECK(cond, bit) \
  do {                       \
  } while (0)
#endif

// Diagnostic build only (-DF16_STAMPS): per-wave cycle totals per code section, from
// s_memtime (a shader-clock counter), accumulated in scalar registers and stored once per
// wave by lane 0. The production build compiles every F16_STAMP to nothing.
enum StampSection {
  ST_LOAD = 0, ST_PROP, ST_DERIVE, ST_ATM, ST_FCS, ST_AUX, ST_ENGINE, ST_AERO, ST_ACCEL,
  ST_FRAME_OBS, ST_REWARD, ST_RESET, ST_SYNC, ST_COPY, ST_STORE, ST_ENVPRE, ST_N
};
#ifdef F16_STAMPS
struct Stamps {
  unsigned long long acc[ST_N];
  unsigned long long last;
};
__device__ __forceinline__ unsigned long long memtime() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define F16_STAMP(S, sec)                    \
  do {                                       \
    const unsigned long long t_ = memtime(); \
    (S).acc[sec] += t_ - (S).last;           \
    (S).last = t_;                           \
  } while (0)
#define F16_STAMP_ARG , Stamps& stamps
#define F16_STAMP_PASS , stamps
#else
#define F16_STAMP(S, sec) \
  do {                    \
  } while (0)
#define F16_STAMP_ARG
#define F16_STAMP_PASS
#endif

// ------------------------------------------------------------------------------------------
// constants shared with the host (filled by f16env_create from the same formulas as the
// oracle's init_consts(), in double, then stored in the kernel argument block)
// ------------------------------------------------------------------------------------------
struct ModelConsts {
  float inv_gref;            // 1 / (GM/a^2)
  float rho_sl, a_sl, p_sl;  // US-76 sea level (slug/ft3, ft/s, psf)
  float inv_rho_sl, inv_p_sl;
  float kts_per_fps;
  float qc_vc250, qc_vc20, qc_vc10, qc_vc5;  // impact pressure (psf) at these calibrated airspeeds (kts)
  double cos_dE, sin_dE;     // rotation of the Earth per frame (omega * dt)
  double dt;
  double epa_dt;             // OMEGA_E * dt: the Earth angle's advance per frame
  // the frame's fp32 products of dt with constants, formed once on the host (build_consts: the
  // same fp32 multiplications the frames did per frame, so the same values) and read as
  // wave-uniform kernel arguments: dt, dt / 2, dt / 12; the kinematic actuators' per-frame travel
  // (rate * dt); the PID integrators' ki * dt
  float dt_f, half_dt, dt_12;
  float lim_ail, lim_rud, lim_lef, lim_sb;
  float kidt_roll, kidt_pitch, kidt_yaw;
};

// Mass properties (FGMassBalance with the tanks pinned to 1000 lb before every run(),
// jsbsim_gym.py:227-228, so constant): oracle init_consts() restated as a constant expression
// (f16.xml:37-83 empty weight / CG / inertia, :245-300 pilot and tanks), evaluated in double at
// compile time and used by the frames as fp32 literals -- the zero products of inertia (the
// airframe is symmetric, Ixy = Iyz = 0) and the zero lateral offsets of the eye point, the
// aero reference point and the thruster then cost no instructions.
struct MassProps {
  float inv_mass;                 // 1/slug
  float J[9], Jinv[9];            // body inertia about the CG, slug ft^2
  float rp[3], eye[3], eng[3];    // AERORP / EYEPOINT / thruster relative to the CG (body ft)
};
constexpr MassProps f16_mass_props() {
  const double SLUG2LB = 32.174049, IN2FT = 1.0 / 12.0;
  const double empty = 17400.0, cg_e[3] = {-193.0, 0.0, -5.1};
  const double pilot = 230.0, pilot_loc[3] = {-336.2, 0.0, 0.0};
  const double tank_w[4] = {1000.0, 1000.0, 0.0, 0.0};
  const double tank_loc[4][3] = {{-174.4, 65.0, 5.0}, {-174.4, -65.0, 5.0}, {-174.4, 65.0, -15.0}, {-174.4, -65.0, -15.0}};
  double W = empty + pilot, m[3] = {0.0, 0.0, 0.0}, cg[3] = {0.0, 0.0, 0.0};
  for (int i = 0; i < 3; ++i) m[i] = empty * cg_e[i] + pilot * pilot_loc[i];
  for (int t = 0; t < 4; ++t) {
    W += tank_w[t];
    for (int i = 0; i < 3; ++i) m[i] += tank_w[t] * tank_loc[t][i];
  }
  for (int i = 0; i < 3; ++i) cg[i] = m[i] / W;
  const double mass = W / SLUG2LB;
  double J[9] = {9496, 0, -982, 0, 55814, 0, -982, 0, 63100};
  // point masses (pilot, tanks) at their structural locations -> body axes about the CG
  const double* locs[5] = {pilot_loc, tank_loc[0], tank_loc[1], tank_loc[2], tank_loc[3]};
  const double ws[5] = {pilot, tank_w[0], tank_w[1], tank_w[2], tank_w[3]};
  for (int p = 0; p < 5; ++p) {
    const double* r = locs[p];
    const double v[3] = {IN2FT * (cg[0] - r[0]), IN2FT * (r[1] - cg[1]), IN2FT * (cg[2] - r[2])};
    const double mm = ws[p] / SLUG2LB;
    const double sv[3] = {mm * v[0], mm * v[1], mm * v[2]};
    const double xx = sv[0] * v[0], yy = sv[1] * v[1], zz = sv[2] * v[2];
    const double xy = -sv[0] * v[1], xz = -sv[0] * v[2], yz = -sv[1] * v[2];
    J[0] += yy + zz; J[1] += xy; J[2] += xz; J[3] += xy; J[4] += xx + zz; J[5] += yz;
    J[6] += xz; J[7] += yz; J[8] += xx + yy;
  }
  const double a = J[0], b = J[1], c = J[2], d = J[3], e = J[4], f = J[5], g = J[6], h = J[7], k = J[8];
  const double A = e * k - f * h, B = -(d * k - f * g), Cc = d * h - e * g;
  const double det = a * A + b * B + c * Cc, r = 1.0 / det;
  const double Ji[9] = {A * r, -(b * k - c * h) * r, (b * f - c * e) * r, B * r, (a * k - c * g) * r,
                        -(a * f - c * d) * r, Cc * r, -(a * h - b * g) * r, (a * e - b * d) * r};
  MassProps P{};
  P.inv_mass = (float)(1.0 / mass);
  for (int i = 0; i < 9; ++i) { P.J[i] = (float)J[i]; P.Jinv[i] = (float)Ji[i]; }
  const double aerorp[3] = {-189.5, 0.0, 3.9}, eye[3] = {-336.2, 0.0, 29.5}, eng[3] = {0.0, 0.0, 0.0};
  for (int i = 0; i < 3; ++i) {
    const double s = (i == 1) ? 1.0 : -1.0;  // structural -> body: x and z flip, y keeps its sign
    P.rp[i] = (float)(IN2FT * s * (aerorp[i] - cg[i]));
    P.eye[i] = (float)(IN2FT * s * (eye[i] - cg[i]));
    P.eng[i] = (float)(IN2FT * s * (eng[i] - cg[i]));
  }
  return P;
}
static constexpr MassProps MP = f16_mass_props();

static constexpr double WGS_A = 20925646.32546;
static constexpr double WGS_B = 20855486.5951;
static constexpr double GM_E = 14.0764417572e15;
static constexpr double J2_E = 1.08262982e-03;
static constexpr double OMEGA_E = 0.00007292115;
static constexpr double E2 = 1.0 - (WGS_B * WGS_B) / (WGS_A * WGS_A);
static constexpr double EC2 = 1.0 - E2;
static constexpr float S_W = 300.0f, B_W = 30.0f, CBAR = 11.32f;
static constexpr float PI_F = 3.14159265358979323846f;
static constexpr double PI_D = 3.14159265358979323846;
static constexpr float RAD2DEG_F = 57.295779513082320876798f;

// ------------------------------------------------------------------------------------------
// lane state (registers) and its struct-of-arrays image in HBM
// ------------------------------------------------------------------------------------------
// Layout: 16-byte columns, column j of env k at c[j * n + k] (float4). A wave moves each
// column with one coalesced dwordx4 access (1 KiB per wave-instruction): 16 wide loads and
// stores per lane -- the step's store tail is issue-bound at 4 B/lane (MI355X_MICROARCH.md,
// epilogue store tail). fp64 fields occupy two lanes of a column.
//   C0  rI.x rI.y (f64)        C6  aI.z aIp.xyz           C12 pid_p_i pid_y_i pid_y_p n2'
//   C1  rI.z vI.x (f64)        C7  q0 q1 q2 q3            C13 alpha beta mach qc      (latch)
//   C2  vI.y vI.z (f64)        C8  wI.xyz wId.x           C14 last_d' step (i32) npy npz
//   C3  epa ep_ret (f64)       C9  wId.yz ba.y ba.z       C15 goal.xyz ep_count (i32) (per episode)
//   C4  ndv1.xyz dv2.x         C10 tef ail ele rud        C16 steady wind.xyz, 0  (wind kernels only)
//   C5  dv2.yz aI.xy           C11 lef sb pid_r_i pid_r_p C17 gust.xyz, 0         (wind kernels only)
// n2' = N2 with the augmentation flag in its sign bit (N2 >= 60 %), last_d' = last distance
// with the FRESH flag in its sign bit (a norm, >= 0). C15 changes only when the lane resets, so
// the step stores it for the lanes it reset and no others (round 5: 16 B of the 256 per env
// step not written back). Not stored, because a step never reads
// them from the previous one: the latch's body rates wrt ECEF (p/q/r-aero = wI - Ti2b (0, 0,
// w_earth), a function of q and wI) and ground speed (a function of rI, vI), recomputed at load
// (latch_from_state) exactly as a frame computes them (the last frame of a step runs after the
// step's final integration, so its latch is a function of the stored state); FGTurbine's N1
// (thrust under augmethod 2 reads N2 only, and nothing observes N1); the g-load PID's previous
// input (kd = 0); the body force's x component (only the same frame's accelerations read it).
// get_state reports those three as 0. Handles whose lanes can carry wind (config / random-IC
// wind, cfg5 gusts, set_state) run the wind kernels (MODE bit 1) and move C16-C17 as well.
enum { NCOL = 16, NCOL_ALL = 18, COL_WIND = 16, COL_GUST = 17 };
static constexpr int LANE_FLAG_AUG = 1;
// set by every reset path, cleared by the next step: the windowed-observation step fills the
// lane's new history window with its reset frame (f16env_step_window)
static constexpr int LANE_FLAG_FRESH = 2;
// persistent bytes per env moved by a step (SURVEY.md 8d "S"); +32 in the wind kernels
static constexpr int STATE_BYTES = NCOL * 16;
static constexpr int STATE_BYTES_GUST = NCOL_ALL * 16;

struct SoA {
  float4* c;  // NCOL_ALL columns of n float4
  int64_t n;
};

struct Lane {
  double rI[3], vI[3], epa, ep_ret;
  // ndv1 = -dv1: the AB3 history kept negated (= the last frame's velocity increment), which the
  // frame then stores without a negation per component
  float ndv1[3], dv2[3], aI[3], aIp[3], q[4], wI[3], wId[3], ba[3];
  float tef, ail, ele, rud, lef, sb;
  float pri, prp, ppi, ppp, pyi, pyp;
  float n1, n2;
  float lx[F16L_N];
  float goal[3], last_d;
  float wind[3];  // wind the FDM sees (NED fps): steady + gust
  float wst[3];   // steady wind (column 16)
  float gust[3];  // the cfg5 gust (column 17)
  int32_t step, ep_count, flags;
};

// The halves of a double for the state columns. The empty asm pins the double in a register
// pair first: without it the optimiser narrows "load double; take the low/high word" into two
// 4-byte loads, SROA then cannot promote the Lane's fp64 members (mixed double / float accesses
// of one slot), and they lived in scratch for the whole kernel (72 B per lane, r02).
__device__ __forceinline__ double f2d(float lo, float hi) {
  return __builtin_bit_cast(double, ((uint64_t)__float_as_uint(hi) << 32) | __float_as_uint(lo));
}
__device__ __forceinline__ uint64_t dbits(double d) {
  asm("" : "+v"(d));
  return __builtin_bit_cast(uint64_t, d);
}
__device__ __forceinline__ float dlo(double d) { return __uint_as_float((uint32_t)dbits(d)); }
__device__ __forceinline__ float dhi(double d) { return __uint_as_float((uint32_t)(dbits(d) >> 32)); }
// a flag bit carried in the sign of a non-negative float
__device__ __forceinline__ float with_sign_flag(float v, bool f) {
  return __uint_as_float((__float_as_uint(v) & 0x7fffffffu) | (f ? 0x80000000u : 0u));
}
__device__ __forceinline__ bool sign_flag(float v) { return (__float_as_uint(v) >> 31) != 0; }
__device__ __forceinline__ float without_sign_flag(float v) { return __uint_as_float(__float_as_uint(v) & 0x7fffffffu); }

// body rates wrt ECEF: pqr = wI - Ti2b (0, 0, w_earth) (FGPropagate; the same expression as
// derive's, so the recomputed latch equals the one the last frame of the previous step held)
__device__ __forceinline__ void pqr_aero(const float* q, const float* wI, float* pqr) {
  const float q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
  // explicit FMAs: the same rounding in every build that inlines it (see derive)
  const float T2 = 2.0f * __builtin_fmaf(q1, q3, -(q0 * q2));
  const float T5 = 2.0f * __builtin_fmaf(q2, q3, q0 * q1);
  const float T8 = __builtin_fmaf(q3, q3, __builtin_fmaf(-q2, q2, __builtin_fmaf(-q1, q1, q0 * q0)));
  const float we = (float)0.00007292115;
  pqr[0] = __builtin_fmaf(-T2, we, wI[0]);
  pqr[1] = __builtin_fmaf(-T5, we, wI[1]);
  pqr[2] = __builtin_fmaf(-T8, we, wI[2]);
}
// ground speed (FGAuxiliary Vground): horizontal part of the velocity wrt the rotating Earth,
// |v|^2 - (v . r_hat)^2 with r_hat the geocentric up (the local frame's down axis is -r_hat).
// Frames compute it the same way from their fp32 quantities (ground_speed below).
__device__ __forceinline__ float ground_speed(float vx, float vy, float vz, float rx, float ry, float rz) {
  const float vv = vx * vx + vy * vy + vz * vz;
  const float vr = vx * rx + vy * ry + vz * rz;
  const float rr = rx * rx + ry * ry + rz * rz;
  return __builtin_amdgcn_sqrtf(fmaxf(vv - vr * vr * __builtin_amdgcn_rcpf(rr), 0.0f));
}
__device__ __forceinline__ void latch_from_state(Lane& L) {
  float pqr[3];
  pqr_aero(L.q, L.wI, pqr);
  L.lx[F16L_P_AERO] = pqr[0]; L.lx[F16L_Q_AERO] = pqr[1]; L.lx[F16L_R_AERO] = pqr[2];
  const double w = 0.00007292115;
  L.lx[F16L_VG_FPS] = ground_speed((float)(L.vI[0] + w * L.rI[1]), (float)(L.vI[1] - w * L.rI[0]), (float)L.vI[2],
                                   (float)L.rI[0], (float)L.rI[1], (float)L.rI[2]);
}

// 16-B output store of the step kernels (state columns, window frame slots); NT: non-temporal
// (global_store_dwordx4 ... nt; a compile-time choice: as a runtime branch the compiler merges
// the two stores and drops the hint), which the windowed step uses when its whole grid is
// resident at once (f16_step_win_nt_kernel: 65 536 envs 17.2-17.6 -> 16.6-16.7 us, 131 072 25.0 -> 23.5,
// cfg5 131 072 34.7 -> 32.6; 262 144 envs, two rounds of waves, 47.1 -> 49.3, so not there;
// the contiguous layout is slower with it everywhere; write-through sc1 slower everywhere:
// profiles/r02_variants_store*.json, r02_variants_nt*.json)
template <bool NT = false>
__device__ __forceinline__ void st16(float4* p, float4 v) {
  if (NT) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(__builtin_bit_cast(v4f, v), reinterpret_cast<v4f*>(p));
  } else {
    *p = v;
  }
}

template <bool GUST>
__device__ __forceinline__ void lane_unpack(const float4 (&c)[NCOL], float4 w, float4 g, Lane& L) {
  L.rI[0] = f2d(c[0].x, c[0].y); L.rI[1] = f2d(c[0].z, c[0].w);
  L.rI[2] = f2d(c[1].x, c[1].y); L.vI[0] = f2d(c[1].z, c[1].w);
  L.vI[1] = f2d(c[2].x, c[2].y); L.vI[2] = f2d(c[2].z, c[2].w);
  L.epa = f2d(c[3].x, c[3].y); L.ep_ret = f2d(c[3].z, c[3].w);
  L.ndv1[0] = c[4].x; L.ndv1[1] = c[4].y; L.ndv1[2] = c[4].z; L.dv2[0] = c[4].w;
  L.dv2[1] = c[5].x; L.dv2[2] = c[5].y; L.aI[0] = c[5].z; L.aI[1] = c[5].w;
  L.aI[2] = c[6].x; L.aIp[0] = c[6].y; L.aIp[1] = c[6].z; L.aIp[2] = c[6].w;
  L.q[0] = c[7].x; L.q[1] = c[7].y; L.q[2] = c[7].z; L.q[3] = c[7].w;
  L.wI[0] = c[8].x; L.wI[1] = c[8].y; L.wI[2] = c[8].z; L.wId[0] = c[8].w;
  L.wId[1] = c[9].x; L.wId[2] = c[9].y; L.ba[0] = 0.0f; L.ba[1] = c[9].z; L.ba[2] = c[9].w;
  L.tef = c[10].x; L.ail = c[10].y; L.ele = c[10].z; L.rud = c[10].w;
  L.lef = c[11].x; L.sb = c[11].y; L.pri = c[11].z; L.prp = c[11].w;
  L.ppi = c[12].x; L.pyi = c[12].y; L.pyp = c[12].z; L.ppp = 0.0f;
  L.n2 = without_sign_flag(c[12].w); L.n1 = 0.0f;
  L.lx[F16L_ALPHA] = c[13].x; L.lx[F16L_BETA] = c[13].y; L.lx[F16L_MACH] = c[13].z; L.lx[F16L_VC_KTS] = c[13].w;
  L.last_d = without_sign_flag(c[14].x); L.step = __float_as_int(c[14].y);
  L.lx[F16L_NPY] = c[14].z; L.lx[F16L_NPZ] = c[14].w;
  L.goal[0] = c[15].x; L.goal[1] = c[15].y; L.goal[2] = c[15].z; L.ep_count = __float_as_int(c[15].w);
  L.flags = (sign_flag(c[12].w) ? LANE_FLAG_AUG : 0) | (sign_flag(c[14].x) ? LANE_FLAG_FRESH : 0);
  latch_from_state(L);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    L.wst[j] = GUST ? (&w.x)[j] : 0.0f;
    L.gust[j] = GUST ? (&g.x)[j] : 0.0f;
    L.wind[j] = L.wst[j] + L.gust[j];
  }
}
// the lane's raw columns (and the wind columns of GUST handles), loads only: callers that want
// every load of their prologue in flight before the first use unpack after their own wait
template <bool GUST = false>
__device__ __forceinline__ void lane_fetch(const SoA& s, int64_t k, float4 (&c)[NCOL], float4& w, float4& g) {
  const int64_t n = s.n;
  // column pointers by increment (one 64-bit scalar add per column, not a 64-bit multiply)
  const float4* p = s.c + k;
#pragma unroll
  for (int j = 0; j < NCOL; ++j, p += n) c[j] = *p;
  w = make_float4(0.f, 0.f, 0.f, 0.f);
  g = w;
  if (GUST) {
    w = *p;
    g = *(p + n);
  }
}
template <bool GUST = false>
__device__ __forceinline__ void lane_load(const SoA& s, int64_t k, Lane& L) {
  float4 c[NCOL], w, g;
  lane_fetch<GUST>(s, k, c, w, g);
  lane_unpack<GUST>(c, w, g, L);
}
// the one-env IC template staged in LDS (columns contiguous): no vector-memory traffic, so
// the reset of a finished lane adds no vmcnt dependency to the step's store tail (MODE 0:
// the template carries no wind)
__device__ __forceinline__ void lane_load_lds(const float4* cols, Lane& L) {
  float4 c[NCOL];
#pragma unroll
  for (int j = 0; j < NCOL; ++j) c[j] = cols[j];
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  lane_unpack<false>(c, z, z, L);
}

// PART: 0 every column; 1 the columns a step's frames leave final (all but C3, C14 and C15,
// which the env layer still changes: episode return, last distance, a reset); 2 C3, C14 and C15.
// with15 false: C15 (goal, episode count) is left as it is in memory -- a step whose lane did not
// reset has not changed it.
template <bool GUST = false, int PART = 0, bool NT = false>
__device__ __forceinline__ void lane_store(const SoA& s, int64_t k, const Lane& L, bool with15 = true) {
  const int64_t n = s.n;
  float4 c[NCOL];
  c[0] = make_float4(dlo(L.rI[0]), dhi(L.rI[0]), dlo(L.rI[1]), dhi(L.rI[1]));
  c[1] = make_float4(dlo(L.rI[2]), dhi(L.rI[2]), dlo(L.vI[0]), dhi(L.vI[0]));
  c[2] = make_float4(dlo(L.vI[1]), dhi(L.vI[1]), dlo(L.vI[2]), dhi(L.vI[2]));
  c[3] = make_float4(dlo(L.epa), dhi(L.epa), dlo(L.ep_ret), dhi(L.ep_ret));
  c[4] = make_float4(L.ndv1[0], L.ndv1[1], L.ndv1[2], L.dv2[0]);
  c[5] = make_float4(L.dv2[1], L.dv2[2], L.aI[0], L.aI[1]);
  c[6] = make_float4(L.aI[2], L.aIp[0], L.aIp[1], L.aIp[2]);
  c[7] = make_float4(L.q[0], L.q[1], L.q[2], L.q[3]);
  c[8] = make_float4(L.wI[0], L.wI[1], L.wI[2], L.wId[0]);
  c[9] = make_float4(L.wId[1], L.wId[2], L.ba[1], L.ba[2]);
  c[10] = make_float4(L.tef, L.ail, L.ele, L.rud);
  c[11] = make_float4(L.lef, L.sb, L.pri, L.prp);
  c[12] = make_float4(L.ppi, L.pyi, L.pyp, with_sign_flag(L.n2, (L.flags & LANE_FLAG_AUG) != 0));
  c[13] = make_float4(L.lx[F16L_ALPHA], L.lx[F16L_BETA], L.lx[F16L_MACH], L.lx[F16L_VC_KTS]);
  c[14] = make_float4(with_sign_flag(L.last_d, (L.flags & LANE_FLAG_FRESH) != 0), __int_as_float(L.step),
                      L.lx[F16L_NPY], L.lx[F16L_NPZ]);
  c[15] = make_float4(L.goal[0], L.goal[1], L.goal[2], __int_as_float(L.ep_count));
  float4* p = s.c + k;
#pragma unroll
  for (int j = 0; j < NCOL; ++j, p += n)
    if (PART == 0 || (PART == 1) == (j != 3 && j != 14 && j != 15))
      if (j != 15 || with15) st16<NT>(p, c[j]);
  if (GUST && PART != 2) {
    st16<NT>(p, make_float4(L.wst[0], L.wst[1], L.wst[2], 0.0f));
    st16<NT>(p + n, make_float4(L.gust[0], L.gust[1], L.gust[2], 0.0f));
  }
}

// ------------------------------------------------------------------------------------------
// table lookups (FGTable semantics: clamped, no extrapolation). Breakpoints are literals.
// ------------------------------------------------------------------------------------------
struct Seg {  // bracketing segment i-1..i and clamped factor
  int i;
  float f;
};
__device__ __forceinline__ float rcpf(float x) { return __builtin_amdgcn_rcpf(x); }
// v_sqrt_f32 (~1 ulp) for the physics; the env layer keeps IEEE sqrtf (bit-exact thresholds)
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float fdiv(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }

// FGTable::GetValue bracket: i = 1 + #{k in 1..N-2 : bp[k] < x} (literal compares), then the
// segment's (lo, 1/span) pair from LDS; factor clamped to [0, 1] (2-D semantics, and the
// 1-D end clamps coincide with it).
template <int N>
__device__ __forceinline__ Seg bracket(const float (&bp)[N], const float* pairs, float x) {
#ifdef F16_BRACKET_CMP
  int i = 1;
#pragma unroll
  for (int k = 1; k < N - 1; ++k) i += (bp[k] < x) ? 1 : 0;
#else
  // bp[k] < x  <=>  sign bit of the fp32 difference bp[k] - x (exact in sign: a difference
  // of finite floats rounds to zero only when they are equal, and +0 for x == bp[k]). Counting
  // sign bits keeps the count in VALU integer ops; the compare form costs a VCC write, an
  // SGPR literal and an s_nop hazard pad per breakpoint on gfx950.
  uint32_t c = 0;
#pragma unroll
  for (int k = 1; k < N - 1; ++k) c += __float_as_uint(bp[k] - x) >> 31;
  const int i = 1 + (int)c;
#endif
  F16_CHECK(i >= 1 && i <= N - 1, DBG_TABLE_SEGMENT);
  const float2 p = reinterpret_cast<const float2*>(pairs)[i - 1];
  float f = (x - p.x) * p.y;
  f = __builtin_amdgcn_fmed3f(f, 0.0f, 1.0f);
  return {i, f};
}
// Guess-and-correct bracket (round 5): the same segment and factor as bracket(), from a guess
// instead of a count. u(x) is a monotone map whose integer crossings b'_k (k = 1 .. N-3) lie
// strictly inside segment k's span, bp[k] < b'_k <= bp[k+1]; the guess g = clamp(floor(u), 0,
// N-3) is then the true 0-based segment s = #{k in 1..N-2 : bp[k] < x} or s - 1, and ONE compare
// against the next segment's low end -- read with the guess's own (lo, 1/span) pair, both pairs
// in one ds_read2_b64 -- settles it. ~10 VALU instead of ~3 per interior breakpoint.
// (NaN x: the guess clamps to 0 and no compare is true, as the count gives segment 0; +-inf land
// in the end segments, as the count.)
template <int N>
__device__ __forceinline__ Seg bracket_guess(const float* pairs, float x, float u) {
  static_assert(N >= 3, "guess bracket needs an interior breakpoint");
  const int g = (int)__builtin_amdgcn_fmed3f(u, 0.0f, (float)(N - 3));  // truncation == floor on [0, N-3]
  const float2* P = reinterpret_cast<const float2*>(pairs);
  const float2 p0 = P[g], p1 = P[g + 1];
  const bool up = x > p1.x;
  const float lo = up ? p1.x : p0.x, iv = up ? p1.y : p0.y;
  const int i = g + 1 + (up ? 1 : 0);
  F16_CHECK(i >= 1 && i <= N - 1, DBG_TABLE_SEGMENT);
  float f = (x - lo) * iv;
  f = __builtin_amdgcn_fmed3f(f, 0.0f, 1.0f);
  return {i, f};
}
// near-uniform grid: u = (x - (bp[0] + h/2)) / h with h the mean spacing, crossings at the
// segments' midpoints; guess_ok checks (in double, with a margin far above fp32 rounding) that
// every crossing lies strictly inside its segment
template <int N>
constexpr double guess_h(const float (&bp)[N]) { return ((double)bp[N - 1] - (double)bp[0]) / (N - 1); }
template <int N>
constexpr bool guess_ok_uniform(const float (&bp)[N]) {
  const double h = guess_h(bp), x0 = (double)bp[0] + 0.5 * h;
  for (int k = 1; k <= N - 3; ++k) {
    const double b = x0 + k * h;
    if (!((double)bp[k] + 1e-5 < b && b < (double)bp[k + 1] - 1e-5)) return false;
  }
  return true;
}
template <int N>
__device__ __forceinline__ Seg bracket_g_uniform(const float (&bp)[N], const float* pairs, float x) {
  // (bp is a constexpr table: these fold to literals after inlining)
  const double h = guess_h(bp);
  const float ginv = (float)(1.0 / h), c0 = (float)(-((double)bp[0] + 0.5 * h) / h);
  return bracket_guess<N>(pairs, x, __builtin_fmaf(x, ginv, c0));
}
// The union Mach grid {0, .4, .6, .7, .8, .81, .9, 1, 1.1, 1.2, 1.4, 1.6, 1.8} is not uniform:
// u = 10 x - 4.5, one more past 0.805 (the 0.81 breakpoint), and 5 per unit instead of 10 past
// 1.2 -- crossings at .55 .65 .75 .805 .85 .95 1.05 1.15 1.3 1.5 (machu_guess_ok checks them)
__device__ __forceinline__ float machu_u(float x) {
  x = fminf(x, 4.0f);  // (+inf would make inf - inf below; past 1.8 the guess is the last segment anyway)
  float u = __builtin_fmaf(x, 10.0f, -4.5f);
  u += (x > 0.805f) ? 1.0f : 0.0f;
  return __builtin_fmaf(-5.0f, fmaxf(x - 1.2f, 0.0f), u);
}
constexpr bool machu_guess_ok() {
  // the crossings of machu_u, in double
  const double b[11] = {0, 0.55, 0.65, 0.75, 0.805, 0.85, 0.95, 1.05, 1.15, 1.3, 1.5};
  if (sizeof(BP_machu) / sizeof(BP_machu[0]) != 13) return false;
  for (int k = 1; k <= 10; ++k)
    if (!((double)BP_machu[k] + 1e-4 < b[k] && b[k] < (double)BP_machu[k + 1] - 1e-4)) return false;
  return true;
}
// uniform grid x0 + k*h (k = 0..N-1): same bracket semantics without a search. The clamp is
// done on the float before the floor (v_med3 + v_floor: g = floor(clamp(u, 0, n-2)) equals
// clamp(floor(u), 0, n-2) for every u), and the factor is u - g: the same segment and factor
// as flooring to an int first, without the integer min / compare / select and the
// int-to-float conversion (round 5: 2 x 5 VALU fewer per frame for the engine tables)
template <bool OLD = false>
__device__ __forceinline__ Seg bracket_uniform(float x, float x0, float inv_h, int n) {
  const float u = (x - x0) * inv_h;
  if (OLD) {  // (pre-round-5 form)
    int i = (int)floorf(u) + 1;
    i = i < 1 ? 1 : (i > n - 1 ? n - 1 : i);
    float f = u - (float)(i - 1);
    f = __builtin_amdgcn_fmed3f(f, 0.0f, 1.0f);
    return {i, f};
  }
  const float g = floorf(__builtin_amdgcn_fmed3f(u, 0.0f, (float)(n - 2)));
  const int i = (int)g + 1;
  F16_CHECK(i >= 1 && i <= n - 1, DBG_TABLE_SEGMENT);
  float f = u - g;
  f = __builtin_amdgcn_fmed3f(f, 0.0f, 1.0f);
  return {i, f};
}
__device__ __forceinline__ float lerp1(float f, float a, float b) { return f * (b - a) + a; }

// atan2 for finite arguments: octant reduction + odd minimax polynomial on [0, 1]
// (|err| < 1e-7 rad, vs ~40 instructions + special-case handling for OCML atan2f)
// OLD (the 256-register two-wave builds): IEEE fmaxf / fminf as before round 5, whose code those
// builds register-allocate without the extra spills the select form cost them
// XPOS: x is known to be +0 or positive (a square root): |x| = x and the x < 0 half-turn never
// applies (the same values, three instructions fewer)
template <bool OLD = false, bool XPOS = false>
__device__ __forceinline__ float fatan2(float y, float x) {
  const float ax = XPOS ? x : fabsf(x), ay = fabsf(y);
  // (max / min as one compare and two selects, the compare reused for the octant below: IEEE
  // fmaxf / fminf quiet their |x| operands first, two extra instructions per call)
  const bool steep = ay > ax;
  const float mx = OLD ? fmaxf(ax, ay) : (steep ? ay : ax), mn = OLD ? fminf(ax, ay) : (steep ? ax : ay);
  const float a = (mx > 0.0f) ? mn * __builtin_amdgcn_rcpf(mx) : 0.0f;
  const float s = a * a;
  float p = 2.4566815505e-03f;
  p = __builtin_fmaf(p, s, -1.4401176748e-02f);
  p = __builtin_fmaf(p, s, 3.9780909971e-02f);
  p = __builtin_fmaf(p, s, -7.2348286170e-02f);
  p = __builtin_fmaf(p, s, 1.0498931099e-01f);
  p = __builtin_fmaf(p, s, -1.4161224781e-01f);
  p = __builtin_fmaf(p, s, 1.9985906079e-01f);
  p = __builtin_fmaf(p, s, -3.3332596980e-01f);
  p = __builtin_fmaf(p, s, 9.9999988637e-01f);
  float r = a * p;
  r = steep ? 1.57079632679489662f - r : r;
  if (!XPOS) r = (x < 0.0f) ? 3.14159265358979324f - r : r;
  return copysignf(r, y);
}

// 1-D lookup with a wave-uniform shortcut past the last interior breakpoint (every lane
// above bp[N-2]: the segment is the last one, no search) -- the ground-effect table, whose
// argument h/b is above 1.1 for any aircraft more than ~33 ft up
template <int N>
__device__ __forceinline__ float tab1_fast_end(const float (&bp)[N], const float* pairs, const float* vd, float x);

// blend with a precomputed slope: v + f (v_next - v), the slope stored beside the value in
// the blob (tools/gen_tables.py), i.e. the same fp32 FMA as lerp1 without the subtraction
__device__ __forceinline__ float blend(float f, float v, float slope) { return __builtin_fmaf(f, slope, v); }
// the same on two tables at once (v_pk_fma_f32: two fp32 FMAs per lane per instruction, the
// factor broadcast by op_sel); values/slopes come from LDS as register pairs
typedef float f2v __attribute__((ext_vector_type(2)));
// (p at an even float offset -- every pair the blob stores for a packed blend, tools/gen_tables.py
// -- read as one aligned 8-byte element, so the pair lands in an aligned register pair)
__device__ __forceinline__ f2v ld2(const float* p) {
  const float2 v = *reinterpret_cast<const float2*>(p);
  return f2v{v.x, v.y};
}
__device__ __forceinline__ f2v blend2(float f, f2v v, f2v slope) {
  return __builtin_elementwise_fma(f2v{f, f}, slope, v);
}
// (No inline asm that emits VALU instructions, round 6: round 5's PK_FMA / PK_MUL macros -- raw
// v_pk_fma_f32 / v_pk_mul_f32 with hand-written op_sel / neg modifiers -- were opaque to the
// compiler's scheduler and hazard recognizer; a build that used them inside the 256-register
// kernels' RunIC faulted. Packed fp32 comes only from the compiler, e.g.
// blend2's __builtin_elementwise_fma; tests/test_isa_lint.py enforces it.)

// 1-D lookup: literal breakpoints, LDS (lo, 1/span) pairs, LDS (value, slope) pairs
template <int N>
__device__ __forceinline__ float tab1(const float (&bp)[N], const float* pairs, const float* vd, float x) {
  const Seg s = bracket(bp, pairs, x);
  const float2 p = reinterpret_cast<const float2*>(vd)[s.i - 1];
  return blend(s.f, p.x, p.y);
}
template <int N>
__device__ __forceinline__ float tab1_fast_end(const float (&bp)[N], const float* pairs, const float* vd, float x) {
  if (__ballot(!(x > bp[N - 2])) == 0) {  // same segment and factor as bracket() would give
    const float2 q = reinterpret_cast<const float2*>(pairs)[N - 2];
    const float f = __builtin_amdgcn_fmed3f((x - q.x) * q.y, 0.0f, 1.0f);
    const float2 p = reinterpret_cast<const float2*>(vd)[N - 2];
    return blend(f, p.x, p.y);
  }
  return tab1(bp, pairs, vd, x);
}
// beta7's breakpoints are beta13's even-indexed ones, so its bracket follows from beta13's
constexpr bool beta7_is_even_beta13() {
  for (int j = 0; j < F16_N_B7; ++j)
    if (BP_beta7_bp[j] != BP_beta13_bp[2 * j]) return false;
  return 2 * (F16_N_B7 - 1) == F16_N_B13 - 1;
}

// ------------------------------------------------------------------------------------------
// atmosphere: US-1976 (FGStandardAtmosphere), troposphere..mesosphere, English units out
// ------------------------------------------------------------------------------------------
struct Atm {
  float T, P, rho, a;
};
__device__ __forceinline__ Atm atmosphere(float h_ft) {
  // layer bases (geopotential m), lapse (K/m), base T (K), base P (Pa) -- same recurrence
  // as the oracle, evaluated at compile time below
  constexpr float Hb[8] = {0.0f, 11000.0f, 20000.0f, 32000.0f, 47000.0f, 51000.0f, 71000.0f, 84852.0f};
  constexpr float Lb[7] = {-0.0065f, 0.0f, 0.001f, 0.0028f, 0.0f, -0.0028f, -0.002f};
  constexpr float Tb[7] = {288.15f, 216.65f, 216.65f, 228.65f, 270.65f, 270.65f, 214.65f};
  constexpr float Pb[7] = {101325.0f, 22632.064f, 5474.88867f, 868.018685f, 110.906306f,
                           66.9388731f, 3.95642043f};  // oracle recurrence, rounded
  constexpr float GMR = 9.80665f * 0.0289644f / 8.31432f;
  constexpr float R = 8.31432f / 0.0289644f;
  const float z = h_ft * 0.3048f;
  const float H = 6356766.0f * z * rcpf(6356766.0f + z);
  constexpr float EX[7] = {GMR / Lb[0], 0.0f, GMR / Lb[2], GMR / Lb[3], 0.0f, GMR / Lb[5], GMR / Lb[6]};
  // P = pb (tb/T)^ex in the gradient layers, pb exp(-GMR (H - hb) / tb) in the isothermal
  // ones: both as one v_log_f32 + one v_exp_f32 (OCML powf is ~130 VALU of compensated
  // double-float arithmetic; v_log/v_exp keep P within ~1e-7 relative)
  float T, lg2, pb;
  // layer search only when some lane of the wave is above the troposphere (wave-uniform
  // branch; the reference task and the cfg5 IC box stay below 11 km almost always); the
  // troposphere path has its layer constants as literals
  if (__builtin_expect(__ballot(H >= Hb[1]) != 0, 0)) {
    float hb = Hb[0], lb = Lb[0], tb = Tb[0], ex = EX[0];
    pb = Pb[0];
    int b = 0;
#pragma unroll
    for (int k = 1; k < 7; ++k) b += (H >= Hb[k]) ? 1 : 0;
#pragma unroll
    for (int k = 1; k < 7; ++k) {
      if (b == k) { hb = Hb[k]; lb = Lb[k]; tb = Tb[k]; pb = Pb[k]; ex = EX[k]; }
    }
    T = tb + lb * (H - hb);
    lg2 = (lb != 0.0f) ? ex * __builtin_amdgcn_logf(tb * rcpf(T))
                       : (-GMR * 1.4426950408889634f) * (H - hb) * rcpf(tb);
  } else {
    T = Tb[0] + Lb[0] * H;  // hb = 0
    lg2 = EX[0] * __builtin_amdgcn_logf(Tb[0] * rcpf(T));
    pb = Pb[0];
  }
  const float P = pb * __builtin_amdgcn_exp2f(lg2);
  const float rho = P * rcpf(R * T);
  Atm o;
  o.T = T * 1.8f;
  o.P = P * (1.0f / 47.88025898033584f);
  o.rho = rho * (1.0f / 515.3788183931961f);
  o.a = fsqrt(1.4f * R * T) * (1.0f / 0.3048f);
  return o;
}

// FGAuxiliary::VcalibratedFromMach, split in two. The FCS reads velocities/vc-kts only
// through four thresholds (f16.xml: TEF switch 250 kts, PID triggers 20 / 5 / 10 kts), and
// the calibrated airspeed is a monotone function of the impact pressure qc = pt - p, so the
// frame latches qc (psf) and the FCS compares it with the qc of each threshold
// (ModelConsts::qc_vc*, computed in fp64 at create); vc itself (kts) is evaluated from the
// latch only where it is reported (f16env_get_state).
// (round 5: the subsonic form for every lane and the supersonic one only in waves that hold a
// supersonic lane -- a wave-uniform branch instead of the exec-mask if / else; the same
// expressions, so the same values)
template <bool OLD = false>
__device__ __forceinline__ float impact_pressure(float mach, float p);
template <>
__device__ __forceinline__ float impact_pressure<true>(float mach, float p) {  // (pre-round-5 form)
  if (!(fabsf(mach) > 0.0f)) return 0.0f;
  float pt;
  if (mach < 1.0f) {
    float x = 1.0f + 0.2f * mach * mach;
    pt = p * (x * x * x * fsqrt(x));
  } else {  // Rayleigh pitot
    float m2 = mach * mach, d = 7.0f * m2 - 1.0f;
    pt = p * 166.92158009316827f * (m2 * m2 * m2 * mach) * rcpf(d * d * fsqrt(d));
  }
  return pt - p;
}
template <>
__device__ __forceinline__ float impact_pressure<false>(float mach, float p) {
  const float x = 1.0f + 0.2f * mach * mach;
  float pt = p * (x * x * x * fsqrt(x));
  if (__ballot(mach >= 1.0f) != 0) {  // Rayleigh pitot
    const float m2 = mach * mach, d = 7.0f * m2 - 1.0f;
    const float ps = p * 166.92158009316827f * (m2 * m2 * m2 * mach) * rcpf(d * d * fsqrt(d));
    pt = (mach < 1.0f) ? pt : ps;
  }
  return (fabsf(mach) > 0.0f) ? pt - p : 0.0f;
}
// calibrated airspeed (kts) from the latched impact pressure
__device__ __forceinline__ float vcas_from_qc(float qc, const ModelConsts& C) {
  if (!(qc != 0.0f)) return 0.0f;
  const float A = qc * C.inv_p_sl + 1.0f;
  float M = fsqrt(5.0f * (__builtin_amdgcn_exp2f((1.0f / 3.5f) * __builtin_amdgcn_logf(A)) - 1.0f));
  if (M > 1.0f) {
    // Supersonic: the Rayleigh pitot relation M = c sqrt(A (1 - 1/(7 M^2))^2.5), which the
    // oracle solves by 10 fixed-point steps (contraction ~0.3 per step, converged to fp32
    // precision), solved here by Newton on y = M^2 from the subsonic estimate: 3 steps, each
    // quadratically convergent (9 transcendentals instead of 30).
    float y = M * M;
    const float cA = 0.8812848543473311f * 0.8812848543473311f * A;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float iy = rcpf(y);
      const float t = 1.0f - (1.0f / 7.0f) * iy;
      const float tst = t * fsqrt(t);
      const float g = cA * t * tst;                               // cA t^2.5
      const float dg = (2.5f / 7.0f) * cA * tst * iy * iy;        // dg/dy
      y -= (y - g) * rcpf(1.0f - dg);
    }
    M = fsqrt(y);
  }
  return C.a_sl * M * C.kts_per_fps;
}

// inverse of vcas_from_qc (fp64): the impact pressure of a calibrated airspeed, for
// f16env_set_state's canonical vc-kts latch
__device__ __forceinline__ float qc_from_vcas(double vc_kts, const ModelConsts& C) {
  const double m = vc_kts / (double)C.kts_per_fps / (double)C.a_sl;
  double A;
  if (m < 1.0) {
    A = pow(1.0 + 0.2 * m * m, 3.5);
  } else {
    const double d = 7.0 * m * m - 1.0;
    A = 166.92158009316827 * pow(m, 7.0) / pow(d, 2.5);
  }
  return (float)((A - 1.0) * (double)C.p_sl);
}

// ------------------------------------------------------------------------------------------
// frames
// ------------------------------------------------------------------------------------------
struct Derived {
  float Ti2b[9], Tl2b[9];
  float uvw[3], pqr[3];
  float vg;         // ground speed (latch_from_state's expression)
  float gI[3];      // J2 gravity in ECI axes
  double h_ft;
};

__device__ __forceinline__ void quat_T(const float* q, float* T) {
  const float q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
  // explicit FMAs: the same rounding in every build that inlines it (see derive)
  const float q0q0 = q0 * q0;
  T[0] = __builtin_fmaf(-q3, q3, __builtin_fmaf(-q2, q2, __builtin_fmaf(q1, q1, q0q0)));
  T[1] = 2.0f * __builtin_fmaf(q1, q2, q0 * q3);
  T[2] = 2.0f * __builtin_fmaf(q1, q3, -(q0 * q2));
  T[3] = 2.0f * __builtin_fmaf(q1, q2, -(q0 * q3));
  T[4] = __builtin_fmaf(-q3, q3, __builtin_fmaf(q2, q2, __builtin_fmaf(-q1, q1, q0q0)));
  T[5] = 2.0f * __builtin_fmaf(q2, q3, q0 * q1);
  T[6] = 2.0f * __builtin_fmaf(q1, q3, q0 * q2);
  T[7] = 2.0f * __builtin_fmaf(q2, q3, -(q0 * q1));
  T[8] = __builtin_fmaf(q3, q3, __builtin_fmaf(-q2, q2, __builtin_fmaf(-q1, q1, q0q0)));
}
__device__ __forceinline__ void mmul(const float* A, const float* B, float* C) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C[3 * i + j] = __builtin_fmaf(A[3 * i + 2], B[6 + j], __builtin_fmaf(A[3 * i + 1], B[3 + j], A[3 * i] * B[j]));
}
// Explicit FMAs in the small products: left to the compiler, contraction is chosen per
// kernel instance, and the contiguous and windowed cfg5 builds then rounded the wind-axis
// velocity differently (tools/diag/layout_identity.py)
__device__ __forceinline__ float dot3f(float a0, float b0, float a1, float b1, float a2, float b2) {
  return __builtin_fmaf(a2, b2, __builtin_fmaf(a1, b1, a0 * b0));
}
__device__ __forceinline__ void mvec(const float* M, const float* v, float* o) {
  o[0] = dot3f(M[0], v[0], M[1], v[1], M[2], v[2]);
  o[1] = dot3f(M[3], v[0], M[4], v[1], M[5], v[2]);
  o[2] = dot3f(M[6], v[0], M[7], v[1], M[8], v[2]);
}
__device__ __forceinline__ void mtvec(const float* M, const float* v, float* o) {
  o[0] = dot3f(M[0], v[0], M[3], v[1], M[6], v[2]);
  o[1] = dot3f(M[1], v[0], M[4], v[1], M[7], v[2]);
  o[2] = dot3f(M[2], v[0], M[5], v[1], M[8], v[2]);
}
__device__ __forceinline__ void crossf(const float* a, const float* b, float* o) {
  const float x = __builtin_fmaf(a[1], b[2], -(a[2] * b[1]));
  const float y = __builtin_fmaf(a[2], b[0], -(a[0] * b[2]));
  const float z = __builtin_fmaf(a[0], b[1], -(a[1] * b[0]));
  o[0] = x; o[1] = y; o[2] = z;
}

// Products with a compile-time constant matrix / vector (MP): the terms whose constant is
// zero are left out at compile time (an IEEE compiler may not drop x * 0.0f by itself).
__device__ __forceinline__ float dot3c(const float* m, const float* v) {
  float s = 0.0f;
  bool any = false;
#pragma unroll
  for (int j = 0; j < 3; ++j)
    if (m[j] != 0.0f) {
      s = any ? __builtin_fmaf(m[j], v[j], s) : m[j] * v[j];
      any = true;
    }
  return s;
}
__device__ __forceinline__ void mvec_c(const float* M, const float* v, float* o) {
#pragma unroll
  for (int i = 0; i < 3; ++i) o[i] = dot3c(M + 3 * i, v);
}
// a x b and b x a with a compile-time constant a
__device__ __forceinline__ void cross_c(const float* a, const float* b, float* o) {
  auto term = [](float ai, float bj, float ak, float bk) {  // ai bj - ak bk
    if (ai == 0.0f && ak == 0.0f) return 0.0f;
    if (ak == 0.0f) return ai * bj;
    if (ai == 0.0f) return -ak * bk;
    return __builtin_fmaf(ai, bj, -ak * bk);
  };
  o[0] = term(a[1], b[2], a[2], b[1]);
  o[1] = term(a[2], b[0], a[0], b[2]);
  o[2] = term(a[0], b[1], a[1], b[0]);
}

// Geodetic altitude from ECEF (FGLocation's geodetic altitude), plus the geodetic surface
// normal (for the per-step altitude reference below). The latitude comes from Bowring's
// formula in fp32; the altitude is then h = p cos(lat) + |z| sin(lat) - a sqrt(1 - e^2 sin^2)
// in fp64, which is STATIONARY in the latitude at the true geodetic latitude, so the fp32
// latitude error (~1e-7 rad) enters only quadratically (R * 1e-14 ~ 1e-6 ft). fp64 pieces:
// p = |(x, y)| and the ellipsoid root by one Newton step from fp32 seeds, (cos, sin) renormalised
// to a unit pair (an off-unit pair would err linearly, ~R * 6e-8). Worst error vs the exact
// geodetic altitude over latitudes +-90 deg and -2 000 .. 120 000 ft: 7.4e-7 ft (numpy emulation
// of these operations; the fp32 observation resolves 1e-3 ft). ~16 fp64 instructions instead of
// the ~120 of an fp64 Fukushima step with its four fp64 square roots and a division.
struct AltRef {
  double r0[3];  // ECEF position where h0 was evaluated exactly
  double h0;
  float n[3];    // geodetic up-normal there
};
__device__ __forceinline__ void alt_ref_init(double x, double y, double z, AltRef& A) {
  constexpr double EP2 = (WGS_A * WGS_A) / (WGS_B * WGS_B) - 1.0;
  const double p2 = x * x + y * y;
  const float r0 = p2 > 0.0 ? __builtin_amdgcn_rsqf((float)p2) : 0.0f;
  const double p0 = p2 * (double)r0;
  const double p = __builtin_fma((double)(0.5f * r0), __builtin_fma(-p0, p0, p2), p0);
  const double s0 = fabs(z);
  const float pf = (float)p, zf = (float)s0;
  // Bowring: parametric latitude, then the geodetic one, as unit (cos, sin) pairs
  const float u = zf * (float)WGS_A, v = pf * (float)WGS_B;
  const float ri = __builtin_amdgcn_rsqf(u * u + v * v);
  const float st = u * ri, ct = v * ri;
  const float num = zf + (float)(EP2 * WGS_B) * (st * st * st);
  const float den = pf - (float)(E2 * WGS_A) * (ct * ct * ct);
  const float r2 = __builtin_amdgcn_rsqf(num * num + den * den);
  const float slf = num * r2, clf = den * r2;
  double c = clf, sn = slf;
  const double k = __builtin_fma(-0.5, __builtin_fma(c, c, sn * sn), 1.5);
  c *= k;
  sn *= k;
  const double w = __builtin_fma(-E2 * sn, sn, 1.0);
  const float sw0 = __builtin_amdgcn_sqrtf((float)w);
  const double swd = sw0;
  const double sw = __builtin_fma((double)(0.5f * __builtin_amdgcn_rcpf(sw0)), __builtin_fma(-swd, swd, w), swd);
  A.h0 = __builtin_fma(p, c, __builtin_fma(s0, sn, -WGS_A * sw));
  const float cl = clf, sl = slf * (z < 0.0 ? -1.0f : 1.0f);
  float clon = 1.0f, slon = 0.0f;
  if (pf != 0.0f) {
    const float ir = __builtin_amdgcn_rcpf(pf);
    clon = (float)x * ir;
    slon = (float)y * ir;
  }
  A.n[0] = cl * clon; A.n[1] = cl * slon; A.n[2] = sl;
  A.r0[0] = x; A.r0[1] = y; A.r0[2] = z;
}

// Everything FGPropagate / FGInertial derive from the integrated state.
// ce, se: cos/sin of the Earth position angle (fp64).
// The geodetic altitude is evaluated (alt_ref_init, ~1e-6 ft) once per env step (AltRef) and
// advanced within the step along the geodetic normal: h = h0 + n . (rE - r0). Over one env
// step |rE - r0| < 70 ft, so the neglected curvature term |dr|^2/2R < 2e-4 ft (far below the
// 4e-4 ft fp32 resolution of the observed altitude).
__device__ __forceinline__ void derive(const Lane& L, double ce, double se, const AltRef& A, Derived& d) {
  const double xE = ce * L.rI[0] + se * L.rI[1];
  const double yE = -se * L.rI[0] + ce * L.rI[1];
  const double zE = L.rI[2];
  {
    const float dx = (float)(xE - A.r0[0]), dy = (float)(yE - A.r0[1]), dz = (float)(zE - A.r0[2]);
    d.h_ft = A.h0 + (double)__builtin_fmaf(A.n[2], dz, __builtin_fmaf(A.n[1], dy, A.n[0] * dx));
  }
  // The local NED frame (FGLocation's, geocentric) and J2 gravity (FGInertial::GetGravityJ2)
  // are symmetric about the Earth's axis, so they are evaluated in ECI axes from the ECI
  // position: the same rotations as ECEF -> local composed with Ti2b * Tec2i, without
  // forming Tec2b (FGPropagate's Tec2b and Tec2l products). fp32 direction cosines.
  const float xi = (float)L.rI[0], yi = (float)L.rI[1], zf = (float)zE;
  const float rxyf = fsqrt(__builtin_fmaf(xi, xi, yi * yi));
  const float rf = fsqrt(__builtin_fmaf(rxyf, rxyf, zf * zf));
  const float inv_r = rcpf(rf);
  const float slat = zf * inv_r, clat = rxyf * inv_r;
  float slon = 0.0f, clon = 1.0f;  // of the ECI position (Earth longitude + Earth angle)
  if (rxyf != 0.0f) {
    const float inv = rcpf(rxyf);
    slon = yi * inv;
    clon = xi * inv;
  }
  // Ti2l rows (north, east, down) in ECI
  const float L0 = -clon * slat, L1 = -slon * slat, L2 = clat;
  const float L3 = -slon, L4 = clon;
  const float L6 = -clon * clat, L7 = -slon * clat, L8 = -slat;
  quat_T(L.q, d.Ti2b);
  // Tl2b = Ti2b * Ti2l^T
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float a = d.Ti2b[3 * i], b = d.Ti2b[3 * i + 1], e = d.Ti2b[3 * i + 2];
    // explicit FMAs (as in euler / fatan2 / make_frame_from): the observation's Euler angles
    // come out of these, and compiler-chosen contraction paired them differently in the one-
    // and two-waves-per-SIMD windowed builds (last-bit phi / theta / psi differences)
    d.Tl2b[3 * i] = __builtin_fmaf(e, L2, __builtin_fmaf(b, L1, a * L0));
    d.Tl2b[3 * i + 1] = __builtin_fmaf(b, L4, a * L3);
    d.Tl2b[3 * i + 2] = __builtin_fmaf(e, L8, __builtin_fmaf(b, L7, a * L6));
  }
  // vUVW = Ti2b * (vI - w x rI)
  const float vr[3] = {(float)(L.vI[0] + OMEGA_E * L.rI[1]), (float)(L.vI[1] - OMEGA_E * L.rI[0]),
                       (float)L.vI[2]};
  mvec(d.Ti2b, vr, d.uvw);
  // vPQR = vPQRi - Ti2b * (0,0,w)
  pqr_aero(L.q, L.wI, d.pqr);
  d.vg = ground_speed(vr[0], vr[1], vr[2], xi, yi, zf);
  // J2 gravity (FGInertial::GetGravityJ2), ECEF
  const float adivr = (float)WGS_A * inv_r;
  const float pre = 1.5f * (float)J2_E * adivr * adivr;
  const float gm = (float)GM_E * inv_r * inv_r;
  const float xy = 1.0f - 5.0f * slat * slat, zz = 3.0f - 5.0f * slat * slat;
  const float kxy = -gm * (1.0f + pre * xy);
  d.gI[0] = kxy * clat * clon;
  d.gI[1] = kxy * clat * slon;
  d.gI[2] = -gm * (1.0f + pre * zz) * slat;
}

__device__ __forceinline__ AltRef alt_ref(const Lane& L, double ce, double se) {
  AltRef A;
  alt_ref_init(ce * L.rI[0] + se * L.rI[1], -se * L.rI[0] + ce * L.rI[1], L.rI[2], A);
  return A;
}

// Euler angles from Tl2b (FGMatrix33::GetEuler)
__device__ __forceinline__ void euler(const float* T, float& phi, float& tht, float& psi) {
  if (T[2] <= -1.0f) {
    tht = 0.5f * PI_F; phi = atan2f(-T[7], T[4]); psi = 0.0f;
  } else if (T[2] >= 1.0f) {
    tht = -0.5f * PI_F; phi = atan2f(-T[7], T[4]); psi = 0.0f;
  } else {
    // theta = asin(-T13) as atan2(-T13, cos theta) with cos theta = |(T23, T33)| (Tl2b is a
    // rotation); the polynomial atan2 (|err| < 1e-7 rad) instead of OCML's asinf / atan2f
    // (once per step, outside the frame loop: the pre-round-5 form, same values)
    tht = fatan2<true>(-T[2], fsqrt(__builtin_fmaf(T[5], T[5], T[8] * T[8])));
    phi = fatan2<true>(T[5], T[8]);
    float p = fatan2<true>(T[1], T[0]);
    if (p < 0.0f) p += 2.0f * PI_F;
    psi = p;
  }
}

// FCS components
// clamp as one v_med3_f32 (lo <= hi; equals min(max(x, lo), hi) for every non-NaN x)
__device__ __forceinline__ float clipf(float x, float lo, float hi) { return __builtin_amdgcn_fmed3f(x, lo, hi); }
__device__ __forceinline__ bool eq_roundoff(float a, float b) {
  return fabsf(a - b) <= 2.0f * 1.1920929e-07f * fmaxf(fabsf(a), fabsf(b));
}
// FGKinematic with two detents (single segment): rate = (d1 - d0) / t. The traverse moves
// the output toward the (clamped) input by at most dt * rate per frame, which is the oracle's
// "dt < |in - out| / rate ? out +- dt rate : in" as one clamp of the difference (the reached
// value is out + (in - out): exactly in whenever the difference is exact, else within an ulp).
// FGKinematic's "already there within round-off" test (oracle eq_roundoff, fp64) is not
// restated in fp32: it would hold the output up to 2 fp32 ulps short of the input where the
// oracle moves it onto the input. Branch-free.
// lim = dt * rate (ModelConsts lim_*)
__device__ __forceinline__ float kin2(float out, float in, float d0, float d1, float lim, bool ic) {
  in = clipf(in, d0, d1);
  if (ic) return in;  // compile-time after inlining
  return out + clipf(in - out, -lim, lim);
}
// TEF kinematic: detents {-1, 0, 1}, times {3, 0, 3} (f16.xml:334-350), the FGKinematic
// while-loop of oracle kinematic() in closed form. Segment [-1, 0] has transition time 0 (the
// output jumps to the input whenever the traverse starts in it), segment [0, 1] moves at 1/3
// per second, so at most two passes run: a partial or complete move inside [0, 1], then, if
// time is left and the input is negative, the jump from 0 to it.
__device__ __forceinline__ float kin_tef(float out, float in, float dt, bool ic) {
  in = clipf(in, -1.0f, 1.0f);
  if (ic) return in;
  const bool down = in < out;
  const bool seg1 = down ? !(0.0f < out) : !(0.0f <= out);  // first pass in [-1, 0]: jump
  const float tin = clipf(in, 0.0f, 1.0f);
  const float tdt = fabsf((tin - out) * 3.0f);               // / rate, rate = 1/3
  const bool partial = dt < tdt;
  const float step = (out < in) ? dt * (1.0f / 3.0f) : -dt * (1.0f / 3.0f);
  // second pass: output at 0 (tin), time left, input below it -> jump to the input
  const bool jump2 = (dt - tdt > 0.0f) && !eq_roundoff(in, tin);
  const float o = seg1 ? in : (partial ? out + step : (jump2 ? in : tin));
  return eq_roundoff(in, out) ? out : o;
}
// FGPID (rectangular integrator) with the F-16's triggers, which are switch outputs 0 / 1
// (f16.xml:383-389, :594-604, :716-727): trigger 0 integrates, 1 holds, and the reset branch
// (trigger < 0) cannot occur, so the trigger is passed as `integrate` (trigger == 0). KD: the
// g-load PID has kd = 0 (no derivative term; its previous input is still tracked).
// kidt = ki * dt (ModelConsts kidt_*)
template <bool KD = true>
__device__ __forceinline__ float pidf(float in, float& itot, float& prev, bool integrate, float kp,
                                      float kidt, float kd, float dt, bool ic) {
  if (!ic && integrate) itot += kidt * in;
  float out = kp * in + itot;
  if (KD) out += kd * (ic ? 0.0f : (in - prev) * rcpf(dt));
  prev = in;
  return out;
}
__device__ __forceinline__ float aero_scale(float in, float outmax) {
  // zero-centred aerosurface_scale with symmetric domain [-1,1] and range [-outmax,outmax]
  // (in == 0 -> +-0, the same value)
  return in * outmax;
}

struct FcsOut {
  float de, da, dr, dlef, flap_mix, dsb, throttle;
};
struct FcsTab {  // scheduled gains of the FCS, looked up from the previous frame's latch
  float asc, ele, yaw;
};
__device__ __forceinline__ FcsTab fcs_tables(const Lane& L, const float* T) {
  FcsTab t;
  t.asc = tab1(BP_fcs_aileron_speed_compensated, T + OFF_pair_fcs_aileron_speed_compensated,
               T + OFF_fcs_vd_aileron_speed_compensated, L.lx[F16L_MACH]);
  t.ele = tab1(BP_fcs_elevator_scheduler, T + OFF_pair_fcs_elevator_scheduler,
               T + OFF_fcs_vd_elevator_scheduler, L.lx[F16L_ALPHA]);
  t.yaw = tab1(BP_fcs_yaw_rate_norm, T + OFF_pair_fcs_yaw_rate_norm, T + OFF_fcs_vd_yaw_rate_norm,
               L.lx[F16L_VG_FPS]);
  return t;
}

// f16.xml:309-984 (document order). T = LDS table blob.
template <bool OLD = false>
__device__ __forceinline__ void fcs_run(Lane& L, const float* cmd, float tl2b_33, float v_fps,
                                        const float* T, const FcsTab& tb, const ModelConsts& C, float dt, bool ic,
                                        FcsOut& o) {
  // qc: the impact-pressure latch (vcas_from_qc); "vc < V kts" is "qc < qc(V)"
  const float alpha = L.lx[F16L_ALPHA], mach = L.lx[F16L_MACH], qc = L.lx[F16L_VC_KTS];
  // Flaps
  // switch (:319-327) as selects of the normalised command (tef_rad * 2.864789)
  const float tef_norm = (qc < C.qc_vc250) ? 0.349f * 2.864789f : ((mach > 0.9f) ? -0.0349f * 2.864789f : 0.0f);
  // the flaps sit at their commanded detent almost always (the switch moves only when the
  // airspeed crosses 250 kts or Mach 0.9): a wave whose every lane is there skips the traverse,
  // whose result would be its input (kin_tef returns `out` when in == out)
  if (OLD || ic || __ballot(clipf(tef_norm, -1.0f, 1.0f) != L.tef) != 0) L.tef = kin_tef(L.tef, tef_norm, dt, ic);
  // Roll
  const float roll_err = cmd[0] - L.lx[F16L_P_AERO] * 0.31821f;
  const float roll_pid = pidf(roll_err, L.pri, L.prp, qc < C.qc_vc20, 3.0f, C.kidt_roll, -0.00125f, dt, ic);
  const float roll_cmd = clipf(roll_pid + cmd[0], -1.0f, 1.0f);
  o.da = aero_scale(roll_cmd, 0.375f);
  L.ail = kin2(L.ail, roll_cmd, -1.0f, 1.0f, C.lim_ail, ic);
  const float asc = L.ail * tb.asc;
  const float lflap = clipf(-L.tef - asc, -1.0f, 1.0f);
  const float rflap = clipf(L.tef - asc, -1.0f, 1.0f);
  o.flap_mix = (lflap + rflap) * 1.4324f;
  // Pitch
  const float g_corr = L.lx[F16L_NPZ] - tl2b_33;  // cos(theta)cos(phi) == Tl2b(3,3)
  const float ele_lim = clipf(cmd[1], -1.0f, 0.44f);
  const float ele_sched = ele_lim * tb.ele;
  const float pitch_err = ele_sched + L.lx[F16L_Q_AERO] * 6.2f - g_corr * 0.020f;
  const float gpid = clipf(pidf<false>(pitch_err, L.ppi, L.ppp, qc < C.qc_vc5, 0.3f, C.kidt_pitch, 0.0f, dt, ic), -1.0f, 1.0f);
  const float pitch_sched = clipf(ele_sched + alpha * 1.0472f + gpid, -1.0f, 1.0f);
  L.ele = kin2(L.ele, pitch_sched, -1.0f, 1.0f, C.lim_ail, ic);  // (the same 2 / 0.3 s rate)
  o.de = aero_scale(L.ele, 0.436f);
  // Yaw
  const float yaw_err = cmd[2] + L.lx[F16L_R_AERO] * tb.yaw + L.lx[F16L_NPY] * 0.25f;
  const float ypid = clipf(pidf(yaw_err, L.pyi, L.pyp, qc < C.qc_vc10, 0.1055f, C.kidt_yaw, 0.00005f, dt, ic), -1.0f, 1.0f);
  const float yaw_sched = clipf(cmd[2] + ypid, -1.0f, 1.0f);
  L.rud = kin2(L.rud, yaw_sched, -1.0f, 1.0f, C.lim_rud, ic);
  o.dr = aero_scale(L.rud, 0.524f);
  // Leading edge flap (gear pinned up, no WOW)
  // (as three selects in sequence: the nested conditional compiled to exec-mask branches)
  float lef_rad;
  if (OLD) {
    lef_rad = (alpha > 0.2618f) ? 0.436f : ((alpha > 0.0873f) ? 0.262f : ((mach > 0.9f) ? -0.0349f : 0.0f));
  } else {
    lef_rad = (mach > 0.9f) ? -0.0349f : 0.0f;
    lef_rad = (alpha > 0.0873f) ? 0.262f : lef_rad;
    lef_rad = (alpha > 0.2618f) ? 0.436f : lef_rad;
  }
  o.dlef = lef_rad;
  L.lef = kin2(L.lef, lef_rad * 2.293578f, -1.0f, 1.0f, C.lim_lef, ic);
  // Throttle
  o.throttle = cmd[3] * 2.0f;
  // Speedbrake
  const float sb_init = (alpha * RAD2DEG_F >= 53.0f && v_fps <= 18.0f) ? 1.0f : 0.0f;
  const float sb_sched = sb_init * T[OFF_fcs_vd_speedbrake_scheduler];  // gear-cmd-norm = 0
  L.sb = kin2(L.sb, sb_sched * 60.0f, 0.0f, 60.0f, C.lim_sb, ic);
  o.dsb = L.sb * (1.0f / RAD2DEG_F);
}

// FGTurbine tpRun, augmethod 2
__device__ __forceinline__ float seekf(float v, float target, float accel, float decel, float dt) {
  const float dn = fmaxf(v - dt * decel, target);
  const float up = fminf(v + dt * accel, target);
  return (v > target) ? dn : ((v < target) ? up : v);
}
template <bool OLD = false>
__device__ __forceinline__ float engine_run(Lane& L, float throttle_pos, float mach, float h_rho,
                                            float sigma, const float* T, float dt, bool ic) {
  float tp = throttle_pos, aug_cmd = 0.0f;
  if (tp > 1.0f) { aug_cmd = tp - 1.0f; tp -= aug_cmd; }
  // IdleThrust / MilThrust / AugThrust on one (mach 0..2.6 step 0.2) x (density-alt
  // -10000..60000 step 10000) grid, [14][8][2 values | 2 mach-slopes | value | mach-slope]
  // (Idle/Mil rows clamped beyond their last mach row, as FGTable does)
  const Seg er = bracket_uniform<OLD>(mach, 0.0f, 5.0f, ENGU_NR);
  const Seg ec = bracket_uniform<OLD>(h_rho, -10000.0f, 1e-4f, ENGU_NC);
  const float* e00 = T + (OFF_engu_v + __umul24((unsigned)((er.i - 1) * ENGU_NC + ec.i - 1), 6u));
  const float* e01 = e00 + 6;
  float ev[3];
  {
    const f2v c1 = blend2(er.f, ld2(e00), ld2(e00 + 2)), c2 = blend2(er.f, ld2(e01), ld2(e01 + 2));
    const f2v r = blend2(ec.f, c1, c2 - c1);
    ev[0] = r.x; ev[1] = r.y;
    const f2v t1 = ld2(e00 + 4), t2 = ld2(e01 + 4);
    const float d1 = blend(er.f, t1.x, t1.y), d2 = blend(er.f, t2.x, t2.y);
    ev[2] = d1 + ec.f * (d2 - d1);
  }
  const float idle = 17800.0f * ev[0];
  const float mil = (17800.0f - idle) * ev[1];
  if (ic) {
    L.n2 = 60.0f + tp * 40.0f;
    L.n1 = 30.0f + tp * 70.0f;
    L.flags = (aug_cmd > 0.0f) ? (L.flags | LANE_FLAG_AUG) : (L.flags & ~LANE_FLAG_AUG);
  } else {
    const float nn = fminf((L.n2 - 60.0f) * (1.0f / 40.0f) + 0.1f, 1.0f);
    const float u = 1.0f - nn;
    const float spool = (90.0f / 3.36f) * rcpf(1.0f + 3.0f * u * u * u + (1.0f - sigma));
    L.n2 = seekf(L.n2, 60.0f + tp * 40.0f, spool, spool * 3.0f, dt);
    L.n1 = seekf(L.n1, 30.0f + tp * 70.0f, spool, spool * 2.4f, dt);
  }
  const float n2n = (L.n2 - 60.0f) * (1.0f / 40.0f);
  float thrust = idle + mil * n2n * n2n;
  if (!(L.flags & LANE_FLAG_AUG)) thrust *= (1.0f - 0.03f);
  if (aug_cmd > 0.0f) {
    L.flags |= LANE_FLAG_AUG;
    const float tdiff = 29000.0f * ev[2] - thrust;
    thrust += tdiff * aug_cmd;
  } else {
    L.flags &= ~LANE_FLAG_AUG;
  }
  return thrust;
}

// Aerodynamics (f16.xml:986-1917), hand-fused: shared (index, factor) per breakpoint vector.
struct AeroIn {
  float qbar, alpha, beta, mach, p, q, r, bi2vel, ci2vel, kclge;
  float de, da, dr, dlef, flap, dsb;
};
__device__ __forceinline__ void aero(const AeroIn& a, const float* T, float* F6) {
#ifdef F16_GUESS_BRACKET
  static_assert(guess_ok_uniform(BP_alpha_bp) && guess_ok_uniform(BP_beta13_bp) && machu_guess_ok(),
                "guess-bracket crossings must lie inside their segments");
  const Seg sa = bracket_g_uniform(BP_alpha_bp, T + OFF_pair_alpha, a.alpha);
#else
  const Seg sa = bracket(BP_alpha_bp, T + OFF_pair_alpha, a.alpha);
#endif
  // 16 alpha 1-D tables, [12][16 values | 16 alpha-slopes]; FGTable 1-D semantics (clamp
  // at the ends)
  float A[F16_N_A1D];
  {
    const float* r0 = T + (OFF_alpha1d + __umul24((unsigned)(sa.i - 1), 2u * F16_N_A1D));
#pragma unroll
    for (int k = 0; k < F16_N_A1D / 2; ++k) {
      const f2v r = blend2(sa.f, ld2(r0 + 2 * k), ld2(r0 + F16_N_A1D + 2 * k));
      A[2 * k] = r.x;
      A[2 * k + 1] = r.y;
    }
  }
  // 2-D over (alpha, X), entries [12][X][G values | G alpha-slopes] (the three (alpha, elevator)
  // tables pairwise: [2 values | 2 alpha-slopes | value | alpha-slope]): blend along alpha at the
  // two bracketing X columns, then along X
  const Seg se = bracket(BP_de_bp, T + OFF_pair_de, a.de);
  float ADE[3];  // CDDh, CLDh, CmDh over (alpha, elevator)
  {
    // (table offsets as 32-bit 24-bit products: v_mul_u32_u24, not 64-bit multiply-adds)
    const float* p0 = T + (OFF_ade + __umul24(__umul24((unsigned)(sa.i - 1), F16_N_DE) + (unsigned)(se.i - 1), 6u));
    const float* p1 = p0 + 6;
    const f2v c1 = blend2(sa.f, ld2(p0), ld2(p0 + 2)), c2 = blend2(sa.f, ld2(p1), ld2(p1 + 2));
    const f2v r = blend2(se.f, c1, c2 - c1);
    ADE[0] = r.x; ADE[1] = r.y;
    const f2v t1 = ld2(p0 + 4), t2 = ld2(p1 + 4);
    const float d1 = blend(sa.f, t1.x, t1.y), d2 = blend(sa.f, t2.x, t2.y);
    ADE[2] = d1 + se.f * (d2 - d1);
  }
#ifdef F16_GUESS_BRACKET
  const Seg sb13 = bracket_g_uniform(BP_beta13_bp, T + OFF_pair_beta13, a.beta);
#else
  const Seg sb13 = bracket(BP_beta13_bp, T + OFF_pair_beta13, a.beta);
#endif
  float AB13[2];  // Clb, Cnb over (alpha, beta 13)
  {
    const float* p0 = T + (OFF_ab13 + 4u * (__umul24((unsigned)(sa.i - 1), F16_N_B13) + (unsigned)(sb13.i - 1)));
    const float* p1 = p0 + 4;
    const f2v c1 = blend2(sa.f, ld2(p0), ld2(p0 + 2)), c2 = blend2(sa.f, ld2(p1), ld2(p1 + 2));
    const f2v r = blend2(sb13.f, c1, c2 - c1);
    AB13[0] = r.x; AB13[1] = r.y;
  }
  // i7 - 1 = #{even-indexed interior beta13 breakpoints below beta} = (i13 - 1) / 2
  static_assert(beta7_is_even_beta13(), "beta7 grid must be the even beta13 breakpoints");
  Seg sb7;
  {
    sb7.i = 1 + ((sb13.i - 1) >> 1);
    const float2 p = reinterpret_cast<const float2*>(T + OFF_pair_beta7)[sb7.i - 1];
    sb7.f = __builtin_amdgcn_fmed3f((a.beta - p.x) * p.y, 0.0f, 1.0f);
  }
  float AB7[4];  // Clda, Cldr, Cnda, Cndr over (alpha, beta 7)
  {
    const float* p0 = T + (OFF_ab7 + 8u * (__umul24((unsigned)(sa.i - 1), F16_N_B7) + (unsigned)(sb7.i - 1)));
    const float* p1 = p0 + 8;
#pragma unroll
    for (int k = 0; k < 4; k += 2) {
      const f2v c1 = blend2(sa.f, ld2(p0 + k), ld2(p0 + k + 4)), c2 = blend2(sa.f, ld2(p1 + k), ld2(p1 + k + 4));
      const f2v r = blend2(sb7.f, c1, c2 - c1);
      AB7[k] = r.x; AB7[k + 1] = r.y;
    }
  }
  // the nine mach tables on their union breakpoint grid, [13][(2 values | 2 mach-slopes) x 4 |
  // value | mach-slope]
#ifdef F16_GUESS_BRACKET
  const Seg sm = bracket_guess<13>(T + OFF_pair_machu, a.mach, machu_u(a.mach));
#else
  const Seg sm = bracket(BP_machu, T + OFF_pair_machu, a.mach);
#endif
  float MU[MACHU_NT];
  {
    const float* r0 = T + (OFF_machu_v + __umul24((unsigned)(sm.i - 1), 2u * MACHU_NT));
#pragma unroll
    for (int k = 0; k + 1 < MACHU_NT; k += 2) {
      const f2v r = blend2(sm.f, ld2(r0 + 2 * k), ld2(r0 + 2 * k + 2));
      MU[k] = r.x; MU[k + 1] = r.y;
    }
    if (MACHU_NT & 1) {
      const f2v t = ld2(r0 + 2 * MACHU_NT - 2);
      MU[MACHU_NT - 1] = blend(sm.f, t.x, t.y);
    }
  }
  const float CDmach = MU[MU_CDmach], CYb_M = MU[MU_CYb_M], Clb_M = MU[MU_Clb_M];
  const float Clda_M = MU[MU_Clda_M], Cldr_M = MU[MU_Cldr_M], Cma_M = MU[MU_Cma_M];
  const float Cnb_M = MU[MU_Cnb_M], Cnda_M = MU[MU_Cnda_M], Cndr_M = MU[MU_Cndr_M];

  const float qS = a.qbar * S_W;
  const float qc = a.q * a.ci2vel, pb = a.p * a.bi2vel, rb = a.r * a.bi2vel;
  // DRAG (f16.xml:1010-1174)
  const float D = qS * (ADE[ADE_CDDh] + CDmach + a.dlef * A[A1D_CDDlef] + a.flap * 0.08f +
                        0.0f * 0.027f + a.dsb * A[A1D_CDDsb] + qc * A[A1D_CDq] +
                        qc * a.dlef * A[A1D_CDq_Dlef]);
  // SIDE (:1176-1272)
  const float Y = qS * (a.beta * -1.146f + a.beta * CYb_M + a.da * -0.0226f + a.dr * 0.086f +
                        pb * A[A1D_CYp] + rb * A[A1D_CYr]);
  // LIFT (:1274-1418)
  const float Lf = qS * (a.kclge * ADE[ADE_CLDh] + a.dlef * a.kclge * A[A1D_CLDlef] +
                         a.flap * a.kclge * 0.35f + a.kclge * a.dsb * A[A1D_CLDsb] +
                         qc * a.kclge * A[A1D_CLq] + qc * a.dsb * A[A1D_CLq_Dsb]);
  const float qSb = qS * B_W, qSc = qS * CBAR;
  // ROLL (:1420-1613)
  const float Lm = qSb * (AB13[AB13_Clb] + a.beta * Clb_M + pb * A[A1D_Clp] + rb * A[A1D_Clr] +
                          a.da * AB7[AB7_Clda] + a.alpha * a.da * Clda_M + a.alpha * a.dr * Cldr_M +
                          a.dr * AB7[AB7_Cldr]);
  // PITCH (:1615-1716)
  const float Mm = qSc * (ADE[ADE_CmDh] + a.alpha * Cma_M + a.dsb * A[A1D_CmDsb] + qc * A[A1D_Cmq]);
  // YAW (:1718-1916)
  const float Nm = qSb * (AB13[AB13_Cnb] + a.beta * Cnb_M + pb * A[A1D_Cnp] + rb * A[A1D_Cnr] +
                          a.da * Cnda_M + a.da * AB7[AB7_Cnda] + a.dr * AB7[AB7_Cndr] +
                          a.alpha * a.dr * Cndr_M);
  F6[0] = D; F6[1] = Y; F6[2] = Lf; F6[3] = Lm; F6[4] = Mm; F6[5] = Nm;
}

// One FGFDMExec::Run(). ce/se: Earth angle cos/sin at the START of the frame (updated here).
// One FGFDMExec::Run(). ce/se: Earth angle cos/sin at the START of the frame (updated here).
// Same arithmetic as the oracle's frame(), ordered for one wave's latency: the FCS gain
// lookups (previous latch) are issued first, the wind-axis kinematics run while the fp64
// altitude chain is in flight, and the calibrated airspeed (only read by the NEXT frame's
// FCS) is computed last. No data-dependent branches except the rare large-rotation QExp
// path and the supersonic vcas iteration.
// LOWREG (the two-waves-per-SIMD build, 256 registers): the latch below is fenced off so the
// scheduler cannot hoist the calibrated-airspeed chain into the aerodynamics' live range
// (scratch 168 -> 152 B; 131 072 envs 39.4 -> 38.1 us, 65 536 envs unchanged: only the
// 256-register build takes it)
// WIND: the lane may carry wind (the wind kernels, IC passes); false skips the air-relative
// velocity's wind term (reference task: no wind, jsbsim_gym.py never enables FGWinds).
template <bool LOWREG = false, bool WIND = true>
__device__ __forceinline__ void frame(Lane& L, const float* cmd, double& ce, double& se, const AltRef& A,
                                      const float* T, const ModelConsts& C, bool ic F16_STAMP_ARG) {
  const float dt = C.dt_f;
  const FcsTab tb = fcs_tables(L, T);
  if (!ic) {
    // -- FGPropagate: integrate with the previous frame's derivatives --
    const float hx = C.half_dt * L.wI[0], hy = C.half_dt * L.wI[1], hz = C.half_dt * L.wI[2];
    const float a2 = hx * hx + hy * hy + hz * hz;  // = fma(hz, hz, fma(hx, hx, hy hy)) (contraction)
    // QExp: cos(a), sin(a)/a; series through a^8 (error < 3e-10 for |a| < 0.5, i.e. body
    // rates below 120 rad/s), exact functions beyond
    // (the same nested FMAs, each level fma(-a2, t, k), written with -a2 as a value so that every
    // level after the first is one v_fmaak_f32 (a VOP2 form takes the literal; the VOP3 FMA with
    // a negated operand needs the constant moved into a register first))
    // (-a2 formed as its own sum of negated products, exactly -a2, and made opaque by an empty
    // asm: left as "-a2" the compiler folds the negation back into VOP3 operand modifiers, and
    // the polynomial's constants then need registers instead of the v_fmaak literal)
    float na2 = __builtin_fmaf(-hz, hz, __builtin_fmaf(-hx, hx, -(hy * hy)));
    if constexpr (!LOWREG) asm("" : "+v"(na2));
    float ca, sa;
    if constexpr (LOWREG) {  // (pre-round-5 form: the same values)
      ca = 1.0f - a2 * (0.5f - a2 * (1.0f / 24.0f - a2 * (1.0f / 720.0f - a2 * (1.0f / 40320.0f))));
      sa = 1.0f - a2 * (1.0f / 6.0f - a2 * (1.0f / 120.0f - a2 * (1.0f / 5040.0f - a2 * (1.0f / 362880.0f))));
    } else {
    ca = __builtin_fmaf(na2, __builtin_fmaf(na2, __builtin_fmaf(na2, __builtin_fmaf(na2, 1.0f / 40320.0f,
                                                                                         1.0f / 720.0f),
                                                                       1.0f / 24.0f), 0.5f), 1.0f);
    sa = __builtin_fmaf(na2, __builtin_fmaf(na2, __builtin_fmaf(na2, __builtin_fmaf(na2, 1.0f / 362880.0f,
                                                                                   1.0f / 5040.0f),
                                                                 1.0f / 120.0f), 1.0f / 6.0f), 1.0f);
    }
    if (__builtin_expect(na2 <= -0.25f, 0)) {  // a2 >= 1/4
      const float ang = fsqrt(-na2);
      float sn;
      sincosf(ang, &sn, &ca);  // (one OCML argument reduction for both)
      sa = sn / ang;
    }
    const float p0 = ca, p1 = hx * sa, p2 = hy * sa, p3 = hz * sa;
    // n = q (x) p, as the scalar statement
    //   n0 = q0 p0 - q1 p1 - q2 p2 - q3 p3      n1 = q0 p1 + q1 p0 + q2 p3 - q3 p2
    //   n2 = q0 p2 - q1 p3 + q2 p0 + q3 p1      n3 = q0 p3 + q1 p2 - q2 p1 + q3 p0
    // (fp-contract=on: a product, then three FMAs in that order). Round 5 issued it as 8 packed
    // instructions from inline asm in the one-wave builds; round 6 dropped the asm (+10 VALU per
    // frame): the compiler's own packed form (__builtin_elementwise_fma on the pairs, splats and
    // swaps left to op_sel folding) put the headline kernel into 40 B of scratch
    {
      const float q0 = L.q[0], q1 = L.q[1], q2 = L.q[2], q3 = L.q[3];
      const float n0 = q0 * p0 - q1 * p1 - q2 * p2 - q3 * p3;
      const float n1 = q0 * p1 + q1 * p0 + q2 * p3 - q3 * p2;
      const float n2 = q0 * p2 - q1 * p3 + q2 * p0 + q3 * p1;
      const float n3 = q0 * p3 + q1 * p2 - q2 * p1 + q3 * p0;
      const float rn = __builtin_amdgcn_rsqf(n0 * n0 + n1 * n1 + n2 * n2 + n3 * n3);  // |n| ~ 1
      L.q[0] = n0 * rn; L.q[1] = n1 * rn; L.q[2] = n2 * rn; L.q[3] = n3 * rn;
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) L.wI[j] += dt * L.wId[j];
    // AB3 position: r += dt/12 (23 v0 - 16 v1 + 5 v2) = dt v0 + dt/12 (-16 dv1 + 5 dv2)
    // AB2 velocity: v += dt (1.5 a - 0.5 ap)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      // (16 ndv1 = -16 dv1 exactly: the same FMA, the same rounding)
      const float corr = C.dt_12 * (16.0f * L.ndv1[j] + 5.0f * L.dv2[j]);
      L.rI[j] += C.dt * L.vI[j] + (double)corr;
      const float dv = dt * (1.5f * L.aI[j] - 0.5f * L.aIp[j]);
      L.vI[j] += (double)dv;
      L.dv2[j] = -L.ndv1[j] - dv;  // dv1 - dv
      L.ndv1[j] = dv;              // dv1 = -dv
      L.aIp[j] = L.aI[j];
    }
    L.epa += C.epa_dt;
    const double c2 = ce * C.cos_dE - se * C.sin_dE;
    const double s2 = se * C.cos_dE + ce * C.sin_dE;
    ce = c2; se = s2;
  }
  F16_STAMP(stamps, ST_PROP);
  Derived d;
  derive(L, ce, se, A, d);
  F16_STAMP(stamps, ST_DERIVE);
  // -- Auxiliary, wind-axis part (needs no atmosphere) --
  float wb[3] = {0.0f, 0.0f, 0.0f};
  if (WIND) mvec(d.Tl2b, L.wind, wb);
  const float ua = d.uvw[0] - wb[0], va = d.uvw[1] - wb[1], wa = d.uvw[2] - wb[2];
  const float muw = ua * ua + wa * wa;
  const float vt = fsqrt(muw + va * va);
  const bool moving = muw > 0.0f;
  // JSBSim's alpha = beta = 0 when not moving, as fatan2(+0, 0) = +0 on guarded inputs:
  // straight-line code instead of two divergent branches around the polynomials
  const float alpha = fatan2<LOWREG>(moving ? wa : 0.0f, ua);
  const float suw = fsqrt(muw);
  const float beta = fatan2<LOWREG, true>(moving ? va : 0.0f, suw);  // (suw = sqrt of a sum of squares)
  const float iuw = rcpf(suw), ivt = rcpf(vt);
  const float ca_ = moving ? ua * iuw : 1.0f, sa_ = moving ? wa * iuw : 0.0f;
  const float cb_ = moving ? suw * ivt : 1.0f, sb_ = moving ? va * ivt : 0.0f;
  const float inv2v = (vt != 0.0f) ? 0.5f * ivt : 0.0f;
  const float bi2vel = B_W * inv2v, ci2vel = CBAR * inv2v;
  const float vg = d.vg;
  // pilot-station load factors from the PREVIOUS frame's accelerations (FGAuxiliary runs
  // before FGAccelerations)
  // (eye x w = -(w x eye): u1 = -(wId x eye), u3 = -(wI x (wI x eye)))
  float u1[3], u2[3], u3[3];
  cross_c(MP.eye, L.wId, u1);
  cross_c(MP.eye, L.wI, u2);
  crossf(L.wI, u2, u3);
  const float npy = (L.ba[1] - u1[1] - u3[1]) * C.inv_gref;
  const float npz = (L.ba[2] - u1[2] - u3[2]) * C.inv_gref;
  // -- Atmosphere (standard day: density altitude == altitude) --
  const float h = (float)d.h_ft;
  const Atm atm = atmosphere(h);
  const float sigma = atm.rho * C.inv_rho_sl;
  const float qbar = 0.5f * atm.rho * vt * vt;
  const float mach = vt * rcpf(atm.a);
  // h_b-mac = (h - (Tb2l * rp)_down) / b
  const float down_b[3] = {d.Tl2b[2], d.Tl2b[5], d.Tl2b[8]};
  const float vmac_d = dot3c(MP.rp, down_b);
  const float hbmac = (h - vmac_d) * (1.0f / B_W);
  F16_STAMP(stamps, ST_ATM);
  // -- Systems (reads the previous frame's latch) --
  FcsOut fc;
  fcs_run<LOWREG>(L, cmd, d.Tl2b[8], d.uvw[1], T, tb, C, dt, ic, fc);
  F16_STAMP(stamps, ST_FCS);
  // -- Propulsion --
  const float thrust = engine_run<LOWREG>(L, fc.throttle, mach, h, sigma, T, dt, ic);
  F16_STAMP(stamps, ST_ENGINE);
  // -- Aerodynamics --
  AeroIn ai;
  ai.qbar = qbar; ai.alpha = alpha; ai.beta = beta; ai.mach = mach;
  ai.p = d.pqr[0]; ai.q = d.pqr[1]; ai.r = d.pqr[2];
  ai.bi2vel = bi2vel; ai.ci2vel = ci2vel;
  ai.kclge = tab1_fast_end(BP_kclge, T + OFF_pair_kclge, T + OFF_kclge_vd, hbmac);
  ai.de = fc.de; ai.da = fc.da; ai.dr = fc.dr; ai.dlef = fc.dlef; ai.flap = fc.flap_mix; ai.dsb = fc.dsb;
  float A6[6];
  aero(ai, T, A6);
  // wind (D, Y, L) -> body, vFw = (-D, Y, -L)
  const float fw0 = -A6[0], fw1 = A6[1], fw2 = -A6[2];
  float F[3], M[3];
  F[0] = ca_ * cb_ * fw0 - ca_ * sb_ * fw1 - sa_ * fw2;
  F[2] = sa_ * cb_ * fw0 - sa_ * sb_ * fw1 + ca_ * fw2;
  // (F[0] and F[2] as one packed chain -- five VOP3P instructions for ten, bit-identical -- cost
  // +0.7 us per step on a same-box A/B, profiles/r05_ab_pk_variants.json "noder": not used)
  F[1] = sb_ * fw0 + cb_ * fw1;
  float rxF[3];
  cross_c(MP.rp, F, rxF);
  M[0] = A6[3] + rxF[0];
  M[1] = A6[4] + rxF[1];
  M[2] = A6[5] + rxF[2];
  // thrust along +x at the thruster: r x (T,0,0) = (0, rz T, -ry T)
  F[0] += thrust;
  if (MP.eng[2] != 0.0f) M[1] += MP.eng[2] * thrust;
  if (MP.eng[1] != 0.0f) M[2] -= MP.eng[1] * thrust;
  F16_STAMP(stamps, ST_AERO);
  // -- Accelerations --
#pragma unroll
  for (int j = 0; j < 3; ++j) L.ba[j] = F[j] * MP.inv_mass;
  // inertial acceleration = Ti2b^T (specific force + body gravity) = Ti2b^T ba + gI
  float abI[3];
  mtvec(d.Ti2b, L.ba, abI);
#pragma unroll
  for (int j = 0; j < 3; ++j) L.aI[j] = abI[j] + d.gI[j];
  float Jw[3], wxJw[3], rhs[3];
  mvec_c(MP.J, L.wI, Jw);
  crossf(L.wI, Jw, wxJw);
#pragma unroll
  for (int j = 0; j < 3; ++j) rhs[j] = M[j] - wxJw[j];
  mvec_c(MP.Jinv, rhs, L.wId);
  // -- Auxiliary latch for the next frame's FCS --
  if (LOWREG) __builtin_amdgcn_sched_barrier(0);
  L.lx[F16L_ALPHA] = alpha; L.lx[F16L_BETA] = beta; L.lx[F16L_MACH] = mach;
  L.lx[F16L_VC_KTS] = impact_pressure<LOWREG>(mach, atm.P); L.lx[F16L_VG_FPS] = vg;
  L.lx[F16L_P_AERO] = d.pqr[0]; L.lx[F16L_Q_AERO] = d.pqr[1]; L.lx[F16L_R_AERO] = d.pqr[2];
  L.lx[F16L_NPY] = npy; L.lx[F16L_NPZ] = npz;
  F16_STAMP(stamps, ST_ACCEL);
}

}  // namespace f16
