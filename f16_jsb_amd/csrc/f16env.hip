// f16env.hip -- HIP kernels (gfx950) + the extern "C" ABI declared in include/f16env.h.
//
// Hot path: k_step = one VecEnv step for N envs in ONE launch: 4 FDM frames per lane with
// the state in VGPRs (f16_device.h), then the env layer of jsbsim_gym/jsbsim_gym.py
// (:172-197 frame, :237-261 reward/termination, :487-509 shaping, TimeLimit, Monitor
// stats) and the DummyVecEnv auto-reset (dummy_vec_env.py:56-73) for lanes that finished,
// with the ordered K-frame stack rebuilt by a coalesced per-wave row copy.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/f16env.h"
#include "f16_device.h"
#ifndef F16_C15_ALWAYS
#define F16_C15_ALWAYS 0
#endif

using namespace f16;

// ------------------------------------------------------------------------------------------
// error handling
// ------------------------------------------------------------------------------------------
static thread_local std::string g_err;
static int set_err(int code, const char* msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      char b_[256];                                                                 \
      snprintf(b_, sizeof b_, "%s failed: %s", #x, hipGetErrorString(e_));          \
      return set_err(-2, b_);                                                       \
    }                                                                               \
  } while (0)

// ------------------------------------------------------------------------------------------
// Philox4x32-10 (same stream definition as oracle/f16ref.c)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void philox(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1,
                                       uint32_t c2, uint32_t c3, uint32_t* o) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  o[0] = c0; o[1] = c1; o[2] = c2; o[3] = c3;
}
__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}
// goal RNG: jsbsim_gym.py:312-323 formula on a Philox stream keyed by (seed; gid, episode)
__device__ __forceinline__ void rng_goal(uint64_t seed, uint64_t gid, uint32_t ep, float* g) {
  uint32_t o[4], o2[4];
  philox((uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)gid, (uint32_t)(gid >> 32), ep,
         0x474F414Cu, o);
  philox((uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)gid, (uint32_t)(gid >> 32), ep,
         0x474F414Cu ^ 1u, o2);
  const double dist = 1000.0 + (10000.0 - 1000.0) * u53(o[0], o[1]);
  const double bear = 0.0 + (2.0 * PI_D - 0.0) * u53(o[2], o[3]);
  const double alt = 1000.0 + (4000.0 - 1000.0) * u53(o2[0], o2[1]);
  double sb, cb;
  sincos(bear, &sb, &cb);  // one argument reduction for both (same values as cos / sin)
  g[0] = (float)(dist * cb);
  g[1] = (float)(dist * sb);
  g[2] = (float)alt;
}

// cfg5 random IC (include/f16env.h F16_FLAG_RANDOM_IC), mirrors oracle rng_ic()
__device__ void rng_ic(uint64_t seed, uint64_t gid, uint32_t ep, const double* lo, const double* hi, double* ic) {
  uint32_t o[4];
#pragma unroll  // constant indices: ic[] and o[] stay in registers (no scratch)
  for (int j = 0; j < F16_IC_N; ++j) {
    if ((j & 3) == 0)
      philox((uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)gid, (uint32_t)(gid >> 32), ep,
             0x52494300u + (uint32_t)(j >> 2), o);
    const double u = ((double)o[j & 3] + 0.5) * (1.0 / 4294967296.0);
    ic[j] = lo[j] + (hi[j] - lo[j]) * u;
  }
}
// cfg5 gust noise: three Box-Muller normals (fp32), mirrors oracle rng_normals() (fp64)
__device__ __forceinline__ void rng_normals(uint64_t seed, uint64_t gid, uint32_t ep, uint32_t s, float* xi) {
  uint32_t o[4];
  philox((uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)gid, (uint32_t)(gid >> 32) ^ 0x47555354u, ep, s, o);
  const float s24 = 1.0f / 16777216.0f;
  const float u1 = ((float)(o[0] >> 8) + 0.5f) * s24, u2 = (float)(o[1] >> 8) * s24;
  const float u3 = ((float)(o[2] >> 8) + 0.5f) * s24, u4 = (float)(o[3] >> 8) * s24;
  const float r1 = sqrtf(-2.0f * logf(u1)), r2 = sqrtf(-2.0f * logf(u3));
  float s2, c2, s4, c4;
  sincospif(2.0f * u2, &s2, &c2);
  sincospif(2.0f * u4, &s4, &c4);
  xi[0] = r1 * c2;
  xi[1] = r1 * s2;
  xi[2] = r2 * c4;
}

// uniform action over the Box [-1,-1,-1,0]..[1,1,1,1] (jsbsim_gym.py:143-148) keyed by
// (seed; global env id, step): the f16env_sample_actions stream, also drawn in-kernel by the
// rollout step
__device__ __forceinline__ float4 philox_action(uint64_t seed, uint64_t gid, uint64_t step) {
  uint32_t o[4];
  philox((uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)step,
         (uint32_t)(step >> 32), o);
  const float lo[4] = {-1.f, -1.f, -1.f, 0.f}, hi[4] = {1.f, 1.f, 1.f, 1.f};
  float4 v;
  float* pv = &v.x;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float u = (float)(o[j] >> 8) * (1.0f / 16777216.0f);
    pv[j] = lo[j] + (hi[j] - lo[j]) * u;
  }
  return v;
}

// np.clip(actions, action_space.low, action_space.high) (on_policy_algorithm.py:216: SB3 clips
// the policy's Gaussian sample to the Box before env.step) on float32, as numpy's clip ufunc
// computes it: min(max(x, lo), hi) with max(a, b) = isnan(a) ? a : (a > b ? a : b) and min
// likewise with < (numpy/_core/src/umath/clip.cpp _NPY_CLIP): NaN passes through, -0 clips to +0
// at a 0 bound
__device__ __forceinline__ float np_clip(float x, float lo, float hi) {
  const float m = (x != x) ? x : (x > lo ? x : lo);
  return (m != m) ? m : (m < hi ? m : hi);
}
__device__ __forceinline__ float4 clip_box(float4 a) {  // Box [-1,-1,-1,0]..[1,1,1,1] (jsbsim_gym.py:143-148)
  return make_float4(np_clip(a.x, -1.0f, 1.0f), np_clip(a.y, -1.0f, 1.0f), np_clip(a.z, -1.0f, 1.0f),
                     np_clip(a.w, 0.0f, 1.0f));
}

#define FEAT_IN 15
#define FEAT_OUT 17
// jsbsim_gym/features.py:37-67 on one frame o[15] -> y[17], float32 with torch's per-op
// rounding (IEEE division / sqrt, no FMA contraction, ~1-ulp atan2 / cos / sin)
__device__ __forceinline__ void frame_features(const float* o, float* y) {
#pragma clang fp contract(off)
  // features.py:39-45 unpack; :47-53 position transform
  const float dx = o[12] - o[0], dy = o[13] - o[1], dz = o[14] - o[2];
  float d2 = dx * dx;
  d2 = __fadd_rn(d2, __fmul_rn(dy, dy));
  const float distance = __fsqrt_rn(d2);
  const float abs_bearing = atan2f(dy, dx);
  const float rel_bearing = abs_bearing - o[11];
  y[0] = __fdiv_rn(1.0f, __fadd_rn(1.0f, __fmul_rn(distance, 1e-3f)));  // :56 dist_norm
  y[1] = __fdiv_rn(dz, 15000.0f);                                         // :59 dz_norm
  y[2] = __fdiv_rn(o[2], 15000.0f);                                       // :60 alt_norm
  y[3] = o[3];                                                            // mach
  y[4] = o[6]; y[5] = o[7]; y[6] = o[8];                                  // angular rates
  y[7] = cosf(o[4]); y[8] = cosf(o[5]);                                   // :63 cos(alpha, beta)
  y[9] = sinf(o[4]); y[10] = sinf(o[5]);                                  //     sin(alpha, beta)
  y[11] = cosf(o[9]); y[12] = cosf(o[10]);                                // :64 cos(phi, theta)
  y[13] = sinf(o[9]); y[14] = sinf(o[10]);                                //     sin(phi, theta)
  y[15] = cosf(rel_bearing); y[16] = sinf(rel_bearing);                   // :65
}

// frame_features split into four parts of about equal cost (the feature-window kernel gives
// each part to a wave): the same expressions, so the same values, as frame_features
__device__ __forceinline__ void frame_features_part(const float* o, float* y, int part) {
#pragma clang fp contract(off)
  const float dx = o[12] - o[0], dy = o[13] - o[1];
  if (part == 0) {
    const float abs_bearing = atan2f(dy, dx);
    const float rel_bearing = abs_bearing - o[11];
    y[15] = cosf(rel_bearing); y[16] = sinf(rel_bearing);
  } else if (part == 1) {
    y[7] = cosf(o[4]); y[8] = cosf(o[5]);
    y[9] = sinf(o[4]); y[10] = sinf(o[5]);
  } else if (part == 2) {
    y[11] = cosf(o[9]); y[12] = cosf(o[10]);
    y[13] = sinf(o[9]); y[14] = sinf(o[10]);
  } else {
    const float dz = o[14] - o[2];
    float d2 = dx * dx;
    d2 = __fadd_rn(d2, __fmul_rn(dy, dy));
    const float distance = __fsqrt_rn(d2);
    y[0] = __fdiv_rn(1.0f, __fadd_rn(1.0f, __fmul_rn(distance, 1e-3f)));
    y[1] = __fdiv_rn(dz, 15000.0f);
    y[2] = __fdiv_rn(o[2], 15000.0f);
    y[3] = o[3];
    y[4] = o[6]; y[5] = o[7]; y[6] = o[8];
  }
}

// ------------------------------------------------------------------------------------------
// IC (FGFDMExec::RunIC + InitRunning), mirrors oracle apply_ic()
// ------------------------------------------------------------------------------------------
// LOWREG: the enclosing kernel's register budget (frame<LOWREG>: the two-waves-per-SIMD 256-register
// kernels run their in-kernel RunIC with the same build of the frame as their steps -- round 6;
// before, every RunIC ran the one-wave build's code, also inside the 256-register kernels)
template <bool LOWREG = false>
__device__ void apply_ic(Lane& L, const double* ic, const float* T, const ModelConsts& C) {
  const double lat = ic[F16_IC_LAT_GEOD_RAD], lon = ic[F16_IC_LON_RAD], h = ic[F16_IC_H_SL_FT];
  // (sincos: one argument reduction per angle, the same values as sin / cos)
  double sl, cl, slo, clo;
  sincos(lat, &sl, &cl);
  sincos(lon, &slo, &clo);
  const double N = WGS_A / sqrt(1.0 - E2 * sl * sl);
  const double rE[3] = {(N + h) * cl * clo, (N + h) * cl * slo, (EC2 * N + h) * sl};
  L.epa = 0.0;
  for (int j = 0; j < 3; ++j) L.rI[j] = rE[j];
  const double rxy = sqrt(rE[0] * rE[0] + rE[1] * rE[1]);
  const double r = sqrt(rxy * rxy + rE[2] * rE[2]);
  const double slat = rE[2] / r, clat = rxy / r;
  const double slon = rxy == 0.0 ? 0.0 : rE[1] / rxy, clon = rxy == 0.0 ? 1.0 : rE[0] / rxy;
  const double Lm[9] = {-clon * slat, -slon * slat, clat, -slon, clon, 0.0, -clon * clat, -slon * clat, -slat};
  const double ph = ic[F16_IC_PHI_RAD], th = ic[F16_IC_THETA_RAD], ps = ic[F16_IC_PSI_RAD];
  double cp, sp, ct, st, cs, ss;
  sincos(ph, &sp, &cp);
  sincos(th, &st, &ct);
  sincos(ps, &ss, &cs);
  const double Tl[9] = {ct * cs, ct * ss, -st,
                        sp * st * cs - cp * ss, sp * st * ss + cp * cs, sp * ct,
                        cp * st * cs + sp * ss, cp * st * ss - sp * cs, cp * ct};
  double Ti[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Ti[3 * i + j] = Tl[3 * i] * Lm[j] + Tl[3 * i + 1] * Lm[3 + j] + Tl[3 * i + 2] * Lm[6 + j];
  // FGMatrix33::GetQuaternion
  double t[4] = {1.0 + Ti[0] + Ti[4] + Ti[8], 1.0 + Ti[0] - Ti[4] - Ti[8],
                 1.0 - Ti[0] + Ti[4] - Ti[8], 1.0 - Ti[0] - Ti[4] + Ti[8]};
  int idx = 0;
  for (int i = 1; i < 4; ++i)
    if (t[i] > t[idx]) idx = i;
  double q[4];
  if (idx == 0) {
    q[0] = 0.5 * sqrt(t[0]);
    q[1] = 0.25 * (Ti[5] - Ti[7]) / q[0]; q[2] = 0.25 * (Ti[6] - Ti[2]) / q[0]; q[3] = 0.25 * (Ti[1] - Ti[3]) / q[0];
  } else if (idx == 1) {
    q[1] = 0.5 * sqrt(t[1]);
    q[0] = 0.25 * (Ti[5] - Ti[7]) / q[1]; q[2] = 0.25 * (Ti[1] + Ti[3]) / q[1]; q[3] = 0.25 * (Ti[2] + Ti[6]) / q[1];
  } else if (idx == 2) {
    q[2] = 0.5 * sqrt(t[2]);
    q[0] = 0.25 * (Ti[6] - Ti[2]) / q[2]; q[1] = 0.25 * (Ti[1] + Ti[3]) / q[2]; q[3] = 0.25 * (Ti[5] + Ti[7]) / q[2];
  } else {
    q[3] = 0.5 * sqrt(t[3]);
    q[0] = 0.25 * (Ti[1] - Ti[3]) / q[3]; q[1] = 0.25 * (Ti[2] + Ti[6]) / q[3]; q[2] = 0.25 * (Ti[5] + Ti[7]) / q[3];
  }
  if (q[0] < 0) for (int i = 0; i < 4; ++i) q[i] = -q[i];
  const double qn = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  for (int i = 0; i < 4; ++i) { q[i] /= qn; L.q[i] = (float)q[i]; }
  // Ti2b from the normalised quaternion (double), velocities
  const double q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
  const double T0 = q0 * q0 + q1 * q1 - q2 * q2 - q3 * q3, T1 = 2.0 * (q1 * q2 + q0 * q3), T2 = 2.0 * (q1 * q3 - q0 * q2);
  const double T3 = 2.0 * (q1 * q2 - q0 * q3), T4 = q0 * q0 - q1 * q1 + q2 * q2 - q3 * q3, T5 = 2.0 * (q2 * q3 + q0 * q1);
  const double T6 = 2.0 * (q1 * q3 + q0 * q2), T7 = 2.0 * (q2 * q3 - q0 * q1), T8 = q0 * q0 - q1 * q1 - q2 * q2 + q3 * q3;
  const double u = ic[F16_IC_U_FPS], v = ic[F16_IC_V_FPS], w = ic[F16_IC_W_FPS];
  const double vb[3] = {T0 * u + T3 * v + T6 * w, T1 * u + T4 * v + T7 * w, T2 * u + T5 * v + T8 * w};
  L.vI[0] = vb[0] - OMEGA_E * L.rI[1];
  L.vI[1] = vb[1] + OMEGA_E * L.rI[0];
  L.vI[2] = vb[2];
  L.wI[0] = (float)(ic[F16_IC_P_RPS] + T2 * OMEGA_E);
  L.wI[1] = (float)(ic[F16_IC_Q_RPS] + T5 * OMEGA_E);
  L.wI[2] = (float)(ic[F16_IC_R_RPS] + T8 * OMEGA_E);
  for (int j = 0; j < 3; ++j) {
    L.wId[j] = 0.0f; L.ba[j] = 0.0f; L.aI[j] = 0.0f; L.aIp[j] = 0.0f; L.ndv1[j] = -0.0f; L.dv2[j] = 0.0f;
    L.wst[j] = (float)ic[F16_IC_WIND_N_FPS + j];
    L.wind[j] = L.wst[j] + L.gust[j];  // callers set the gust (0 outside the cfg5 gust mode)
  }
  L.tef = L.ail = L.ele = L.rud = L.lef = L.sb = 0.0f;
  L.pri = L.prp = L.ppi = L.ppp = L.pyi = L.pyp = 0.0f;
  L.n1 = 30.0f; L.n2 = 60.0f; L.flags = 0;
  for (int j = 0; j < F16L_N; ++j) L.lx[j] = 0.0f;
  const float cmd[4] = {(float)ic[F16_IC_CMD_AIL], (float)ic[F16_IC_CMD_ELE], (float)ic[F16_IC_CMD_RUD],
                        (float)ic[F16_IC_CMD_THR]};
  double ce = 1.0, se = 0.0;
#ifdef F16_STAMPS
  Stamps stamps = {};
#endif
  const AltRef A = alt_ref(L, ce, se);
  // three passes, as oracle apply_ic(); a loop, not three inlined copies: the reset kernels run
  // one RunIC per lane from a cold instruction cache, so one copy of the frame code is fetched
  // once and hit twice
#pragma nounroll
  for (int pass = 0; pass < 3; ++pass) frame<LOWREG>(L, cmd, ce, se, A, T, C, true F16_STAMP_PASS);
  for (int j = 0; j < 3; ++j) { L.ndv1[j] = -0.0f; L.dv2[j] = 0.0f; L.aIp[j] = L.aI[j]; }  // (dv1 = +0)
}

// ------------------------------------------------------------------------------------------
// env layer
// ------------------------------------------------------------------------------------------
// normalize_angle_mpi_pi (jsbsim_gym.py:60-78) on a float32 value (numpy-1.x promotion)
__device__ __forceinline__ float norm_angle(float a) {
  if (isnan(a) || isinf(a)) return 0.0f;
  double x = (double)a;
  if (!(fabs(x) < 2.0 * PI_D)) x = fmod(x, 2.0 * PI_D);
  if (x < 0.0) x += 2.0 * PI_D;
  if (x >= PI_D) x -= 2.0 * PI_D;
  if (x == 0.0) x = 0.0;
  return (float)x;
}
// _get_current_single_observation (jsbsim_gym.py:172-197)
// The observation frame (jsbsim_gym.py:172-197) from the derived quantities of the lane's
// state; the latitude / longitude are evaluated here. (Reusing the last FDM frame's Derived
// instead -- the frame's accelerations do not move rI, vI, q, wI -- saved 0.7 us per step at
// 4 096 envs and nothing at 65 536 in the windowed step, r02_variants_keep.json, but the
// two builds then round the observation differently: kept out, the one- and two-waves-per-
// SIMD builds stay bit-identical.)
__device__ void make_frame_from(const Lane& L, double ce, double se, const Derived& d, float* f) {
  // explicit FMAs: with contraction left to the compiler, the one- and two-waves-per-SIMD
  // windowed builds paired these products differently, and yE (a difference of two ~2e7 ft
  // terms near the start meridian) and so the observed longitude differed in the last bits
  // (tests/test_gpu_production.py two-million-env case)
  const double xE = __builtin_fma(ce, L.rI[0], se * L.rI[1]);
  const double yE = __builtin_fma(ce, L.rI[1], -se * L.rI[0]);
  const float xf = (float)xE, yf = (float)yE, zf = (float)L.rI[2];
  const float rxyE = fsqrt(__builtin_fmaf(xf, xf, yf * yf));
  const float lat = atan2f(zf, rxyE);
  const float lon = (rxyE == 0.0f) ? 0.0f : atan2f(yf, xf);
  float phi, tht, psi;
  euler(d.Tl2b, phi, tht, psi);
  f[0] = (float)((double)lat * 6.3781e6);
  f[1] = (float)((double)lon * 6.3781e6);
  f[2] = (float)(d.h_ft * 0.3048);
  f[3] = L.lx[F16L_MACH];
  f[4] = L.lx[F16L_ALPHA];
  f[5] = L.lx[F16L_BETA];
  f[6] = d.pqr[0]; f[7] = d.pqr[1]; f[8] = d.pqr[2];
  f[9] = norm_angle(phi); f[10] = norm_angle(tht); f[11] = norm_angle(psi);
  f[12] = L.goal[0]; f[13] = L.goal[1]; f[14] = L.goal[2];
}
__device__ void make_frame(const Lane& L, double ce, double se, const AltRef& A, float* f) {
  Derived d;
  derive(L, ce, se, A, d);
  make_frame_from(L, ce, se, d, f);
}
__device__ __forceinline__ float norm3f(float a, float b, float c) {
#pragma clang fp contract(off)
  float s = a * a;
  s = s + b * b;
  s = s + c * c;
  return sqrtf(s);
}

// observation_space.contains on one frame, finite values only (jsbsim_gym.py:268-285 against
// SINGLE_OBS_LOW / SINGLE_OBS_HIGH, :28-53, float32 bounds): a component outside its bounds
// that is finite. (The infinite bounds of the other components admit every finite value.)
__device__ __forceinline__ bool obs_out_of_bounds(const float* f) {
  const float pe = (float)(PI_D + 1e-5), he = (float)(0.5 * PI_D + 1e-5);
  bool bad = f[3] < 0.0f;                                 // mach >= 0
  bad = bad || f[4] < -pe || f[4] > pe || f[5] < -pe || f[5] > pe;  // alpha, beta
  bad = bad || f[9] < -pe || f[9] > pe || f[11] < -pe || f[11] > pe;  // phi, psi
  bad = bad || f[10] < -he || f[10] > he;               // theta
  bad = bad || f[14] < 0.0f;                            // goal z >= 0
  return bad;  // NaN compares false: non-finite values never count
}

struct EnvArgs {
  int64_t n;
  int32_t K, down_sample, max_steps, flags;
  float dg, crash;
  double gain;
  uint64_t seed;
  int64_t id_base;
  const double* ic_cfg;  // config IC, RANDOM_IC box lo / hi (device, F16_IC_N each)
  const double* ic_lo;
  const double* ic_hi;
  float gust_a, gust_b, gust_sigma;  // cfg5 Gauss-Markov gust coefficients
};

// reward / termination (jsbsim_gym.py:237-261) in float32, then PositionReward (:493-507), on
// the new frame f; Monitor's return (monitor.py:96-99). Returns the flags: bit 0 terminated,
// 1 truncated, 2 quarantined by F16_FLAG_NAN_GUARD (a non-finite position / Mach / alpha /
// beta / body rate; the angles f[9..11] are already NaN -> 0 by normalize_angle_mpi_pi).
__device__ __forceinline__ int env_reward(Lane& L, const float* f, const EnvArgs& E, float& r32) {
  int te = 0, tr;
  bool bad = false;
  if (E.flags & F16_FLAG_NAN_GUARD) {
#pragma unroll
    for (int j = 0; j < 9; ++j) bad = bad || !isfinite(f[j]);
  }
  if (bad) {
    te = 5;  // terminated + quarantined (bit 2), reported as terminated[i] = 3
    tr = 0;
    r32 = 0.0f;
  } else {
#pragma clang fp contract(off)
    double r = 0.0;
    const float alt = f[2];
    if (alt < E.crash) { r = -10.0; te = 1; }
    const float dx = f[0] - f[12], dy = f[1] - f[13];
    float d2 = dx * dx;
    d2 = d2 + dy * dy;
    if (!te && sqrtf(d2) < E.dg && fabsf(alt - f[14]) < E.dg) { r = 10.0; te = 1; }
    tr = L.step >= E.max_steps ? 1 : 0;                   // env :260 | TimeLimit
    // The previous distance is moved into a register of its own first. SROA keeps the Lane's
    // {goal.z, last_d, wind.x, wind.y} as one 4-VGPR tuple, and the new distance below is
    // written into the same tuple's last_d lane; in f16_step_win_nt_kernel<2|3, 1> (ROCm 7.2,
    // LLVM 22) the register allocator then placed that write before the read of the old value
    // (`v_sub_f32 v0, v207, v207`: every shaping term, hence every reward, was 0 -- the "all-zero
    // rewards" of round 2). The empty asm breaks the tuple's live range; tests/test_isa_lint.py
    // scans the built code object for x - x subtractions.
    float last_d = L.last_d;
    asm volatile("" : "+v"(last_d));
    const float dcur = norm3f(f[12] - f[0], f[13] - f[1], f[14] - f[2]);
    const float ddiff = last_d - dcur;
    r = r + E.gain * (double)ddiff;
    L.last_d = dcur;
    L.ep_ret += r;                                         // monitor.py:96-99
    r32 = (float)r;
  }
  return te | (tr << 1);
}

// reset a lane and produce its frame 0: the IC template copy (default config), or the full
// RunIC of a per-lane / random / config IC (cfg5 modes: the gust enters the IC passes)
__device__ void lane_reset(Lane& L, const SoA& tmpl, const double* ic, const float* goal,
                           const EnvArgs& E, int64_t k, const float* T, const ModelConsts& C,
                           float* f0) {
  const int32_t ep = L.ep_count;
  const uint64_t gid = (uint64_t)(E.id_base + k);
  if (ic || (E.flags & (F16_FLAG_RANDOM_IC | F16_FLAG_GUSTS))) {
    double ric[F16_IC_N];
    if (!ic) {
      if (E.flags & F16_FLAG_RANDOM_IC) {
        rng_ic(E.seed, gid, (uint32_t)ep, E.ic_lo, E.ic_hi, ric);
        ic = ric;
      } else {
        ic = E.ic_cfg;
      }
    }
    if (E.flags & F16_FLAG_GUSTS) {
      float xi[3];
      rng_normals(E.seed, gid, (uint32_t)ep, 0u, xi);
      for (int j = 0; j < 3; ++j) L.gust[j] = E.gust_sigma * xi[j];
    } else {
      L.gust[0] = L.gust[1] = L.gust[2] = 0.0f;
    }
    apply_ic(L, ic, T, C);
  } else {
    lane_load<true>(tmpl, 0, L);  // the config IC (its wind included: MODE 0 handles have none)
  }
  if (goal) {
    L.goal[0] = goal[0]; L.goal[1] = goal[1]; L.goal[2] = goal[2];
  } else {
    rng_goal(E.seed, gid, (uint32_t)ep, L.goal);
  }
  L.ep_count = ep + 1;
  L.step = 0;
  L.ep_ret = 0.0;
  L.flags |= LANE_FLAG_FRESH;
  make_frame(L, 1.0, 0.0, alt_ref(L, 1.0, 0.0), f0);
  L.last_d = norm3f(f0[12] - f0[0], f0[13] - f0[1], f0[14] - f0[2]);
}

// lane_reset for a kernel compiled for one MODE (the windowed step's in-step RunIC): the random
// IC stays a register array (lane_reset selects between it and the global config IC through
// one pointer, which puts both in scratch)
template <int MODE, bool LOWREG = false>
__device__ void lane_reset_mode(Lane& L, const EnvArgs& E, int64_t k, const float* T, const ModelConsts& C,
                                float* f0) {
  const int32_t ep = L.ep_count;
  const uint64_t gid = (uint64_t)(E.id_base + k);
  if (E.flags & F16_FLAG_GUSTS) {  // (MODE bit 1 is also set by steady wind alone)
    float xi[3];
    rng_normals(E.seed, gid, (uint32_t)ep, 0u, xi);
    for (int j = 0; j < 3; ++j) L.gust[j] = E.gust_sigma * xi[j];
  } else {
    L.gust[0] = L.gust[1] = L.gust[2] = 0.0f;
  }
  if (MODE & 1) {
    double ric[F16_IC_N];
    rng_ic(E.seed, gid, (uint32_t)ep, E.ic_lo, E.ic_hi, ric);
    apply_ic<LOWREG>(L, ric, T, C);
  } else {
    apply_ic<LOWREG>(L, E.ic_cfg, T, C);
  }
  rng_goal(E.seed, gid, (uint32_t)ep, L.goal);
  L.ep_count = ep + 1;
  L.step = 0;
  L.ep_ret = 0.0;
  L.flags |= LANE_FLAG_FRESH;
  make_frame(L, 1.0, 0.0, alt_ref(L, 1.0, 0.0), f0);
  L.last_d = norm3f(f0[12] - f0[0], f0[13] - f0[1], f0[14] - f0[2]);
}

// The template's frame 0 without the goal (12 floats) follows its NCOL_ALL state columns as
// TMPL_FRAME_COLS float4s, written once by f16_ic_kernel with the same make_frame: an
// auto-reset then costs the goal draw only, not a frame evaluation (fp64 altitude, Euler
// angles, atan2s) on the critical path of every wave that holds a finished lane.
enum { TMPL_FRAME_COLS = 3, TMPL_COLS = NCOL_ALL + TMPL_FRAME_COLS };
__device__ __forceinline__ void lane_reset_template(Lane& L, const float4* sTmpl, const EnvArgs& E, int64_t k,
                                                    float* f0) {
  const int32_t ep = L.ep_count;
  lane_load_lds(sTmpl, L);
  rng_goal(E.seed, (uint64_t)(E.id_base + k), (uint32_t)ep, L.goal);
  L.ep_count = ep + 1;
  L.step = 0;
  L.ep_ret = 0.0;
  L.flags |= LANE_FLAG_FRESH;
#ifdef F16_RESET_MAKE_FRAME  // A/B only: evaluate frame 0 per finished lane
  make_frame(L, 1.0, 0.0, alt_ref(L, 1.0, 0.0), f0);
#else
#pragma unroll
  for (int j = 0; j < TMPL_FRAME_COLS; ++j) {
    const float4 v = sTmpl[NCOL + j];
    f0[4 * j] = v.x; f0[4 * j + 1] = v.y; f0[4 * j + 2] = v.z; f0[4 * j + 3] = v.w;
  }
  f0[12] = L.goal[0]; f0[13] = L.goal[1]; f0[14] = L.goal[2];
#endif
  L.last_d = norm3f(f0[12] - f0[0], f0[13] - f0[1], f0[14] - f0[2]);
}

// Earth position angle -> (cos, sin), once per env step (fp64)
__device__ __forceinline__ void earth_angle(double epa, double& ce, double& se) {
  if (fabs(epa) < 0.01) {  // series, exact in fp64 for |epa| < 0.01 (40 s episodes: 3e-3)
    const double e2 = epa * epa;
    ce = 1.0 - e2 * (0.5 - e2 * (1.0 / 24.0 - e2 * (1.0 / 720.0 - e2 * (1.0 / 40320.0))));
    se = epa * (1.0 - e2 * (1.0 / 6.0 - e2 * (1.0 / 120.0 - e2 * (1.0 / 5040.0 - e2 * (1.0 / 362880.0)))));
  } else {
    ce = cos(epa);
    se = sin(epa);
  }
}

// ------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------
#ifndef BLOCK
#define BLOCK 256
#endif
#define FRAME_PITCH 16
// The previous stack block lands in the wave's LDS image IMG_OFF floats past its 16-byte
// aligned base. IMG_OFF = 1 makes the shifted copy-out out[j] = img[IMG_OFF + j + 15] whole
// aligned float4s (ds_read_b128 instead of four dwords), but the misaligned LDS-DMA landing
// costs more than it saves (measured 23.0 vs 23.3 us per step at 65 536 envs, K = 4; 31.2 vs
// 32.3 at K = 10: profiles/r01_variants_w.json), so the image stays aligned.
#ifndef IMG_OFF
#define IMG_OFF 0
#endif

// Wait for every outstanding vector-memory operation (s_waitcnt vmcnt(0)) as the compiler's
// own wait: its wait-insertion pass then knows the LDS-DMA issued before is retired. (An
// inline-asm s_waitcnt is opaque to that pass: it kept treating the fresh-frame DMA into the
// staging area as pending and put another vmcnt(0) before the slot staging's LDS writes --
// which on CDNA also waits for every state store issued in between.) The empty asm statements
// keep the compiler from moving memory operations across it.
#ifdef F16_ASM_VMCNT  // (round 5's form, for the same-box A/B)
#define VM_DRAIN() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#else
#define VM_DRAIN()                          \
  do {                                      \
    asm volatile("" ::: "memory");          \
    __builtin_amdgcn_s_waitcnt(0x0F70);     \
    asm volatile("" ::: "memory");          \
  } while (0)
#endif

// LDS-DMA of 16 B per lane: lane i's 16 bytes land at lds + 16*i (gfx950 global_load_lds_dwordx4)
__device__ __forceinline__ void dma16(const float* g, float* lds) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                   (void __attribute__((address_space(3)))*)lds, 16, 0, 0);
}
// ... and of 4 B per lane (lane i's dword lands at lds + 4*i)
__device__ __forceinline__ void dma4(const float* g, float* lds) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                   (void __attribute__((address_space(3)))*)lds, 4, 0, 0);
}
// Table blob -> LDS by LDS-DMA (no VGPRs, no wait at issue): the caller issues its other
// loads behind it and completes the staging with one s_waitcnt vmcnt(0) + barrier.
__device__ __forceinline__ void stage_tables_issue(float* sT) {
  constexpr int NP = F16_BLOB_FLOATS / 4;  // 16-byte pieces (the generator pads the blob)
  static_assert(F16_BLOB_FLOATS % 4 == 0, "blob must be whole 16-byte pieces");
  const int wave_base = threadIdx.x & ~63;
  // stride BLOCK, not blockDim.x: every kernel that stages the tables launches BLOCK threads, and
  // blockDim.x is a load from the implicit kernel arguments -- the wait for it held the DMA (and
  // the state loads behind it) until the whole argument block had arrived
#ifdef F16_STAGE_BLOCKDIM  // (round 5's form, for the same-box A/B)
  for (int r = 0; r < NP; r += blockDim.x) {
#else
  for (int r = 0; r < NP; r += BLOCK) {
#endif
    const int piece = r + threadIdx.x;
    if (piece < NP) dma16(F16_BLOB_INIT + 4 * piece, sT + 4 * (r + wave_base));
  }
}
__device__ __forceinline__ void stage_tables(float* sT) {
  stage_tables_issue(sT);
  VM_DRAIN();
  __syncthreads();
}

// Render/telemetry pose of one observation frame x: what JSBSimEnv.render
// (jsbsim_gym/jsbsim_gym.py:381-415) hands the Viewer -- the aircraft position in viewer axes
// (-y, h, x) * 1e-3, its attitude Quaternion.from_euler(phi, theta, psi) (visualization/
// quaternion.py:38-45, q_psi * q_theta * q_phi) remapped (w, -y, -z, x), and the goal position
// in viewer axes -- in float32 with the reference's operation order (no contraction). Shared
// by f16_poses_kernel and the plain step's epilogue (F16_STEP_POSES), so both give the same bits.
__device__ __forceinline__ void quat_mul_ref(const float* a, const float* b, float* o) {
#pragma clang fp contract(off)
  // quaternion.py:11-14: w = a0 b0 - a.b ; v = a0 b + b0 a + a x b  (float32, left to right)
  const float dot = a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
  o[0] = a[0] * b[0] - dot;
  const float cx = a[2] * b[3] - a[3] * b[2], cy = a[3] * b[1] - a[1] * b[3], cz = a[1] * b[2] - a[2] * b[1];
  o[1] = a[0] * b[1] + b[0] * a[1] + cx;
  o[2] = a[0] * b[2] + b[0] * a[2] + cy;
  o[3] = a[0] * b[3] + b[0] * a[3] + cz;
}
__device__ __forceinline__ void pose_of_frame(const float* x, float* o) {
#pragma clang fp contract(off)
  const float s = 1e-3f;
  o[0] = -x[1] * s; o[1] = x[2] * s; o[2] = x[0] * s;
  const float hp = x[9] / 2.0f, ht = x[10] / 2.0f, hs = x[11] / 2.0f;
  float sp, cp, st, ct, ss, cs;
  sincosf(hp, &sp, &cp);
  sincosf(ht, &st, &ct);
  sincosf(hs, &ss, &cs);
  const float q1[4] = {cp, sp, 0.0f, 0.0f};
  const float q2[4] = {ct, 0.0f, st, 0.0f};
  const float q3[4] = {cs, 0.0f, 0.0f, ss};
  float q32[4], q[4];
  quat_mul_ref(q3, q2, q32);
  quat_mul_ref(q32, q1, q);
  o[3] = q[0]; o[4] = -q[2]; o[5] = -q[3]; o[6] = q[1];
  o[7] = -x[13] * s; o[8] = x[14] * s; o[9] = x[12] * s;
}

struct StepArgs {
  SoA s, tmpl;
  const float* act;
  const float* obs_prev;
  float* obs;
  float* rew;
  uint8_t* term;
  uint8_t* trunc;
  float* tobs;
  double* ep_ret;
  int32_t* ep_len;
  int32_t* done_idx;
  int32_t* n_done;
  unsigned long long* nonfinite;  // F16_FLAG_NAN_GUARD quarantine count (handle-owned); [2]:
                                  // F16_FLAG_OBS_CHECK out-of-bounds lane-steps
  int32_t lds_image;
  // rollout slot (f16env_step_rollout; all NULL / 0 for f16env_step)
  int32_t sample_act;          // act == NULL: draw the actions in-kernel (seed, step)
  int32_t clip_act;            // F16_SLOT_CLIP: the env steps np.clip(act, low, high), r_act keeps act
  uint64_t act_seed, act_step;
  float* r_frame;              // N x 15: newest frame of obs_prev (contiguous layout)
  float* r_next_frame;         // N x 15: newest frame of the returned obs (windowed layout)
  float* r_act;                // N x 4: the actions (as given: unclipped)
  float* r_rew;                // N: rewards
  float* r_next_start;         // N: done as 0/1 float (episode_starts of the next slot)
  // windowed observations (f16env_step_window): the frame histories of this step (wx, the one
  // whose window is the returned observation) and of the other parity (wy), [T][N][16] each
  // (position-major: the N slots of one position are contiguous)
  float* wx;
  float* wy;
  int64_t wrow;                // floats between positions (position-major: N * 16; env-major: 16)
  int64_t wenv;                // floats between envs (position-major: 16; env-major: T * 16)
  int32_t wpos;                // newest frame position p (window = p-K+1 .. p)
  int32_t half_delay;          // HALF builds (experiment): cycles the second half of the grid waits
  // the feature window in the rollout-slot build (F16_SLOT_FEATURE_WINDOW): the feature
  // histories [T][N][17] of this step's parity (fwx) and the other (fwy); nullptr: none
  float* fwx;
  float* fwy;
  // cfg5 modes, windowed layout: the reset cache (f16_ic_fill_kernel): per lane the state and
  // frame 0 (without the goal) of its NEXT reset, ICC_COLS columns; c == nullptr: deferred
  // resets by f16_reset_done_kernel instead
  SoA icc;
  EnvArgs E;
  ModelConsts C;
  // the plain step's pose export (f16env_window_step_ex with F16_STEP_POSES): N x 10 floats, the
  // pose of the returned observation's newest frame per env; nullptr: none
  float* poses;
};

#ifdef F16_STAMPS
__device__ unsigned long long g_stamps[1 << 14][ST_N];  // per wave (diagnostic build)
#endif


// Dynamic LDS: image mode holds, per wave, the previous stack block of its 64 rows
// (64*KC floats) + one spare frame; fallback mode holds the final/reset frames per lane.
__device__ __forceinline__ size_t image_floats_per_wave(int KC) { return (size_t)64 * KC + 16; }

// MODE bit 0: F16_FLAG_RANDOM_IC, bit 1: F16_FLAG_GUSTS. MODE 0 (the reference's task) resets
// finished lanes inline from the IC template; other modes leave finished lanes to
// f16_reset_done_kernel (a full RunIC per lane is too long to run divergently in-wave).
// GT: tables read from the global blob (L1/L2-resident, 12 KB) instead of an LDS copy, which
// frees the LDS for the stack image at large K (K = 10: four 38.5 KB images + the blob exceed
// 160 KB). sT is then unused.
// Windowed observations (WIN, f16env_step_window): two frame histories [T][N][16] (wx: this
// step's parity, wy: the other; position-major 16-float = 64-B frame slots, the 16th float 0),
// the observation of a step being the view wx[p-K+1 .. p][k][0..15) (strides 16, N*16, 1). A step
// writes its new frame at position p of BOTH histories -- no stack shift copy, no
// previous-stack read -- as four aligned 16-B stores filling one whole 64-B sector (a 60-B
// frame at a 60-B pitch leaves partial sectors, which cost as much as the whole-row rewrite
// they replace: 22.6 vs 18.5 us per step at 65 536 envs, K = 4, gpurun r02n). Lanes reset right
// before this step (FRESH) fill wx[p-K+1 .. p-1] with their reset frame (LDS-DMA'd from
// wy[p-1], which that reset wrote); lanes reset by this step fill wx[p-K+1 .. p] with the new
// reset frame and keep their final frame in wy[p], so wy's window IS the terminal observation
// (no copy). The other parity's window is untouched by a step, so an observation stays valid
// until the step after next, as with the ping-pong buffers of f16env_step.
static constexpr int WPITCH = 16;  // floats per history frame slot
template <bool NT = false>
__device__ __forceinline__ void put_slot(float* d, const float* f) {
  float4* q = reinterpret_cast<float4*>(d);
  st16<NT>(q, make_float4(f[0], f[1], f[2], f[3]));
  st16<NT>(q + 1, make_float4(f[4], f[5], f[6], f[7]));
  st16<NT>(q + 2, make_float4(f[8], f[9], f[10], f[11]));
  st16<NT>(q + 3, make_float4(f[12], f[13], f[14], 0.0f));
}
static constexpr int WFRESH = 16 * 64;  // LDS floats per wave for the fresh-frame DMA ([4][64] float4)
static constexpr int WSTASH = 16 * 64;  // ... and for the env-field stash of the 256-register builds
static constexpr int WIN_WAVE_FLOATS = WFRESH + WSTASH;

// The prologue's first loads from kernel arguments preloaded into SGPRs (StepPre, windowed
// kernels): the state, action and template addresses and N are in registers when the wave
// starts, so the state / action loads and the table and template DMA issue without first
// waiting for the scalar load of the argument block (-amdgpu-kernarg-preload-count, build.py).
struct StepPre {
  const float4* sc;
  const float* act;
  const float4* tmpl;
  int64_t n;
};
// HALF (windowed builds, an experiment: F16ENV_HALF=1): 32 envs per wave in lanes 0-31, so a
// grid of N envs is N/32 waves -- two per SIMD at 65 536 envs -- and the second half of the
// grid may start `half_delay` cycles late, so that one wave's memory phases (prologue loads,
// store tail) overlap the other's frames on the same SIMD.
// XV (windowed plain-step extras, f16_step_winx_kernel / f16env_window_step_ex): XV_FEAT keeps the
// bound feature histories in the step's epilogue (the rollout-slot build's F16_SLOT_FEATURE_WINDOW
// code, without the slot); every winx build draws the actions in-kernel when act == NULL
// (a.sample_act: the f16env_sample_actions stream) and writes the pose export when a.poses is set
// (F16_STEP_POSES, a run-time choice: no further instances). The headline instances (XV = 0)
// carry none of this code.
enum { XV_X = 1, XV_FEAT = 2 };
template <int MODE, bool GT = false, bool ROLL = false, bool LOWREG = false, bool WIN = false, bool NT = false,
          bool HALF = false, int XV = 0>
__device__ __forceinline__ void step_body(const StepArgs& a, float* sT_lds, float4* sTmpl, int* sDone, float* dynl,
                                          const StepPre* pre = nullptr) {
  const float* sT = GT ? static_cast<const float*>(F16_BLOB_INIT) : sT_lds;
  constexpr bool GUST = (MODE & 2) != 0, DEFER = MODE != 0;
  // builds that may draw the actions in-kernel (act == NULL): the rollout slot's and the winx
  constexpr bool SAMPLE = ROLL || (XV & XV_X) != 0;
  constexpr bool FEATW = ROLL || (XV & XV_FEAT) != 0;  // builds with the feature-window epilogue
  constexpr int EPW = HALF ? 32 : 64;  // envs per wave
#ifdef F16_STAMPS
  Stamps stamps = {};
  stamps.last = memtime();
#endif
  if (HALF && a.half_delay > 0 && blockIdx.x >= gridDim.x / 2) {
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < (uint64_t)a.half_delay) __builtin_amdgcn_s_sleep(8);
  }
  const int KC = a.E.K * F16_OBS_DIM, HC = (a.E.K - 1) * F16_OBS_DIM;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row0 = (int64_t)blockIdx.x * (4 * EPW) + wave * EPW;
  const int64_t nE = pre ? pre->n : a.E.n;
  const int rows = (int)(nE - row0 < EPW ? (nE - row0 > 0 ? nE - row0 : 0) : EPW);
  const bool image = a.lds_image != 0;
  // cfg5 modes in the windowed layout reset finished lanes in the step (reset cache)
  const bool in_step_reset = WIN && DEFER && a.icc.c != nullptr && !(a.E.flags & F16_FLAG_NO_AUTORESET);
#ifdef F16_NO_STASH
  constexpr bool STASH = false;
#else
  constexpr bool STASH = LOWREG && WIN;
#endif
  float* img = dynl + (size_t)wave * image_floats_per_wave(KC);
  // 1) DMA of this wave's previous stack block into LDS (overlaps the physics)
  auto issue_stack_dma = [&]() {
    if (image && rows > 0) {
      const float* prev = a.obs_prev + row0 * KC;
      const int total = rows * KC;  // floats
      const int n16 = total >> 2;   // whole 16-byte pieces (wave blocks are 16-B aligned)
      for (int b = 0; b < n16; b += 64) {
        const int piece = b + lane;
        if (piece < n16) dma16(prev + 4 * piece, img + IMG_OFF + 4 * b);
      }
      if (lane < (total & 3)) dma4(prev + 4 * n16 + lane, img + IMG_OFF + 4 * n16);  // tail, never past the end
    }
  };
  const int64_t k = row0 + lane;
  const bool live = (!HALF || lane < EPW) && k < nE;
  F16_CHECK(rows >= 0 && rows <= 64 && (!live || row0 + lane < nE), DBG_STATE_INDEX);
  if (WIN) F16_CHECK(a.wpos >= a.E.K - 1 && a.wpos >= 0, DBG_WINDOW_POS);
  int done = 0;
  Lane L;
  float4 av = make_float4(0.f, 0.f, 0.f, 0.f);
  // the loads the physics needs are in flight at once (table DMA, IC template, state and
  // action), then one wait: a single HBM round trip before the physics. The previous stack
  // (only needed by the obs rebuild) is DMA'd after that wait, so it streams in while the
  // first frame runs instead of sharing the prologue's HBM bandwidth.
  if (!GT) stage_tables_issue(sT_lds);
  // IC template: the NCOL state columns, then its frame-0 columns (lane i lands at sTmpl[i])
  if (!DEFER && threadIdx.x < NCOL + TMPL_FRAME_COLS)
    dma16(reinterpret_cast<const float*>((pre ? pre->tmpl : a.tmpl.c) + (threadIdx.x < NCOL ? threadIdx.x : threadIdx.x + NCOL_ALL - NCOL)),
          reinterpret_cast<float*>(sTmpl));
  // (the columns are unpacked after the wait, behind a scheduling barrier: a first use the
  // scheduler hoists between the loads puts a vmcnt(0) there -- the table DMA and the first two
  // columns' round trip, then the other fourteen's. Unconditional loads -- a lane past the end
  // reading env 0 -- let the argument fetches issue before the wait too, but measured no faster
  // at 65 536 envs and 0.5 us slower for cfg5's two-wave kernel: profiles/r06_ab_prologue.json)
  float4 cl[NCOL], wl, gl;
  if (live) {
    if (pre) {
      const SoA sp = {const_cast<float4*>(pre->sc), pre->n};
      lane_fetch<GUST>(sp, k, cl, wl, gl);
      if (!SAMPLE || !a.sample_act) av = reinterpret_cast<const float4*>(pre->act)[k];
    } else {
      lane_fetch<GUST>(a.s, k, cl, wl, gl);
      if (!SAMPLE || !a.sample_act) av = reinterpret_cast<const float4*>(a.act)[k];
    }
  }
  VM_DRAIN();
#ifndef F16_PROLOGUE_NO_SCHED_BARRIER  // (for the same-box A/B)
  __builtin_amdgcn_sched_barrier(0);
#endif
  if (live) lane_unpack<GUST>(cl, wl, gl, L);
  __syncthreads();
  issue_stack_dma();
  if (SAMPLE && a.sample_act && live) av = philox_action(a.act_seed, (uint64_t)(a.E.id_base + k), a.act_step);
  // a lane reset since the last step: the windowed step reads its reset frame (wy[p-1]) now,
  // so the load streams in behind the physics
  // (LDS-DMA into the wave's staging area, [15][64] floats, not registers: nothing stays live
  // across the frames; the vmcnt(0) after the frames retires it)
  bool fresh = false;
  float* stg = dynl + (size_t)wave * WIN_WAVE_FLOATS;
  if (live) {
    fresh = (L.flags & LANE_FLAG_FRESH) != 0;
    L.flags &= ~LANE_FLAG_FRESH;
  }
  if (WIN && fresh && a.E.K > 1) {
    const float* src = a.wy + k * a.wenv + (int64_t)(a.wpos - 1) * a.wrow;
#pragma unroll
    for (int j = 0; j < 4; ++j) dma16(src + 4 * j, stg + j * 256);  // [j][lane] float4
  }
  F16_STAMP(stamps, ST_LOAD);
  float f[F16_OBS_DIM], f0[F16_OBS_DIM];
  float rew_out = 0.0f;
  int flags_out = 0;
  double ce = 1.0, se = 0.0;
  AltRef A;
  if (live) {
    const float4 ac = (ROLL && a.clip_act) ? clip_box(av) : av;  // the env steps the clipped action
    const float cmd[4] = {ac.x, ac.y, ac.z, ac.w};
    L.step += 1;                                              // jsbsim_gym.py:215
    if (GUST) {  // cfg5 Gauss-Markov gust update, once per env step before the frames
      float xi[3];
      rng_normals(a.E.seed, (uint64_t)(a.E.id_base + k), (uint32_t)(L.ep_count - 1), (uint32_t)L.step, xi);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        L.gust[j] = __builtin_fmaf(a.E.gust_a, L.gust[j], a.E.gust_b * xi[j]);  // explicit: every build alike
        L.wind[j] = L.wst[j] + L.gust[j];
      }
    }
    earth_angle(L.epa, ce, se);
    A = alt_ref(L, ce, se);  // exact geodetic altitude once per env step
    F16_STAMP(stamps, ST_ENVPRE);
    // 256-register windowed builds: the env fields the frames never read (goal, last distance,
    // step, episode count and return) wait in the wave's LDS stash instead of VGPRs, which the
    // frame loop needs (they were part of what spilled to scratch around it)
    float4* stash = reinterpret_cast<float4*>(stg + WFRESH);
    if (STASH) {
      stash[lane] = make_float4(L.goal[0], L.goal[1], L.goal[2], L.last_d);
      stash[64 + lane] = make_float4(__int_as_float(L.step), __int_as_float(L.ep_count), dlo(L.ep_ret), dhi(L.ep_ret));
      // the Earth angle: the frames advance it by a constant each (replayed below, the same
      // fp64 adds) and otherwise read only its cos / sin; the gust model's pieces: the frames
      // read the wind sum only
      stash[128 + lane] = make_float4(dlo(L.epa), dhi(L.epa), GUST ? L.gust[0] : 0.0f, GUST ? L.gust[1] : 0.0f);
      if (GUST) stash[192 + lane] = make_float4(L.gust[2], L.wst[0], L.wst[1], L.wst[2]);
      asm volatile("" ::: "memory");
    }
    for (int s = 0; s < a.E.down_sample; ++s)  // :225-232
      frame<LOWREG, GUST>(L, cmd, ce, se, A, sT, a.C, false F16_STAMP_PASS);
    if (STASH) {
      asm volatile("" ::: "memory");
      const float4 g = stash[lane], e = stash[64 + lane];
      L.goal[0] = g.x; L.goal[1] = g.y; L.goal[2] = g.z; L.last_d = g.w;
      L.step = __float_as_int(e.x); L.ep_count = __float_as_int(e.y); L.ep_ret = f2d(e.z, e.w);
      const float4 w = stash[128 + lane];
      L.epa = f2d(w.x, w.y);
      for (int s = 0; s < a.E.down_sample; ++s) L.epa += a.C.epa_dt;  // frame()'s per-frame advance
      if (GUST) {
        const float4 u = stash[192 + lane];
        L.gust[0] = w.z; L.gust[1] = w.w; L.gust[2] = u.x; L.wst[0] = u.y; L.wst[1] = u.z; L.wst[2] = u.w;
      }
    }
  }
  // Early state store, with no done list to compact (its atomic's return would wait for every
  // store before it): retire the stack DMA and store the state columns the frames left final
  // now, so their drain overlaps the observation frame, reward and obs writes instead of
  // adding to the tail. Two-waves-per-SIMD builds only (gpurun r02m, MODE 0: 131 072 envs
  // 30.35 -> 29.89 us, 262 144 62.35 -> 60.0 us). At one wave per SIMD: the contiguous build
  // gained nothing at 65 536 envs and lost 0.4 us at 4 096; the non-temporal windowed build
  // gained 0.35 us on fresh episodes but lost 0.3-0.4 us in the bench's steady state, where
  // a lane reset by the step stores its row twice (r02_variants_early_store.txt).
  const bool early_store = LOWREG && !a.done_idx;
  if (early_store) {
    VM_DRAIN();
    if (live) lane_store<GUST, 1, NT>(a.s, k, L);
  }
  if (live) {
    make_frame(L, ce, se, A, f);  // :234
    F16_STAMP(stamps, ST_FRAME_OBS);
    // reward / termination (:237-261), PositionReward (:493-507)
    float r32;
    flags_out = env_reward(L, f, a.E, r32);  // bit 0 terminated, 1 truncated, 2 quarantined
    F16_STAMP(stamps, ST_REWARD);
    done = flags_out & 3;
    rew_out = r32;
  }
  // the stack DMA issued after the prologue has long landed; retire it here, before any
  // store of this step (vmcnt also counts stores on CDNA, so a later wait would drain them)
  // -- unless the early state store above already did
  if (!early_store) VM_DRAIN();
  // compaction of finished lanes (wave64 ballot), before any store of this step so the
  // atomic's return waits on nothing else
  if (a.done_idx) {  // (always set in deferred modes: the handle's own list if the caller gave none)
    const unsigned long long m = __ballot(done);
    if (m) {
      int base = 0;
      if (lane == 0) base = atomicAdd(a.n_done, __popcll(m));
      base = __shfl(base, 0);
      F16_CHECK(base + __popcll(m) <= nE, DBG_DONE_LIST);
      if (done) a.done_idx[base + __popcll(m & ((1ull << lane) - 1ull))] = (int32_t)k;
    }
  }
  if (a.E.flags & F16_FLAG_NAN_GUARD) {
    const unsigned long long qm = __ballot(flags_out & 4);
    if (qm && lane == 0) atomicAdd(a.nonfinite, (unsigned long long)__popcll(qm));
  }
  if (a.E.flags & F16_FLAG_OBS_CHECK) {  // jsbsim_gym.py:268-285 on the new frame
    const unsigned long long om = __ballot(live && obs_out_of_bounds(f));
    if (om && lane == 0) atomicAdd(a.nonfinite + 2, (unsigned long long)__popcll(om));
  }
  if (live) {
    a.rew[k] = rew_out;
    a.term[k] = (uint8_t)((flags_out & 1) | ((flags_out >> 1) & 2));
    a.trunc[k] = (uint8_t)((flags_out >> 1) & 1);
    if (ROLL) {
      if (a.r_rew) a.r_rew[k] = rew_out;
      if (a.r_act) reinterpret_cast<float4*>(a.r_act)[k] = av;
      if (a.r_next_start) a.r_next_start[k] = done ? 1.0f : 0.0f;
    }
    if (done) {
      if (a.ep_ret) a.ep_ret[k] = L.ep_ret;
      if (a.ep_len) a.ep_len[k] = L.step;
      if (!DEFER && !(a.E.flags & F16_FLAG_NO_AUTORESET)) {
        lane_reset_template(L, sTmpl, a.E, k, f0);
      } else if (in_step_reset) {
        // cfg5 modes, windowed layout: the lane's next reset from the cache when it holds that
        // episode's (tag: the cached row's episode count = this lane's + 1; a reset is a pure
        // function of (seed, env id, episode), so any row with that tag is the one), else the
        // full RunIC here (a lane that finished twice within one fill period)
        if (__float_as_int(a.icc.c[(int64_t)15 * a.icc.n + k].w) == L.ep_count + 1) {
          lane_load<GUST>(a.icc, k, L);
#pragma unroll
          for (int j = 0; j < TMPL_FRAME_COLS; ++j) {
            const float4 v = a.icc.c[(int64_t)(NCOL_ALL + j) * a.icc.n + k];
            f0[4 * j] = v.x; f0[4 * j + 1] = v.y; f0[4 * j + 2] = v.z; f0[4 * j + 3] = v.w;
          }
          f0[12] = L.goal[0]; f0[13] = L.goal[1]; f0[14] = L.goal[2];
        } else {
          lane_reset_mode<MODE, LOWREG>(L, a.E, k, sT, a.C, f0);
        }
      } else {
#pragma unroll
        for (int j = 0; j < F16_OBS_DIM; ++j) f0[j] = f[j];
      }
    }
    F16_STAMP(stamps, ST_RESET);
    // C15 (goal, episode count) changes only in a reset: written back for the lanes reset here
    // (F16_C15_ALWAYS=1: every lane, the A/B reference)
    const bool reset_here = done && (!DEFER || in_step_reset) && !(a.E.flags & F16_FLAG_NO_AUTORESET);
    if (!early_store || reset_here)
      lane_store<GUST, 0, NT>(a.s, k, L, F16_C15_ALWAYS || reset_here);  // every column (a lane reset just now rewrites its row)
    else
      lane_store<GUST, 2, NT>(a.s, k, L, false);  // the rest
    F16_STAMP(stamps, ST_STORE);
  }
  sDone[threadIdx.x] = done;
  // deferred modes: f16_reset_done_kernel rewrites finished rows after this kernel, unless the
  // windowed step resets them itself (in_step_reset)
  const bool autoreset = (!DEFER || in_step_reset) && !(a.E.flags & F16_FLAG_NO_AUTORESET);
  // rollout slot frame = newest frame of obs_prev (what the policy acted on), for every lane
  // (contiguous layout; the windowed build writes the returned observation's newest frame
  // below, r_next_frame)
  if (ROLL && !WIN && a.r_frame && rows > 0) {
    if (image) {
      __builtin_amdgcn_wave_barrier();
      float* dst = a.r_frame + row0 * F16_OBS_DIM;
      if (rows == 64) {  // 960 floats = 240 float4, 16-B aligned (row0 is a multiple of 64)
        for (int q = lane; q < 64 * F16_OBS_DIM / 4; q += 64) {
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int j = 4 * q + i, r = j / F16_OBS_DIM, c = j - r * F16_OBS_DIM;
            v[i] = img[IMG_OFF + r * KC + HC + c];
          }
          reinterpret_cast<float4*>(dst)[q] = make_float4(v[0], v[1], v[2], v[3]);
        }
      } else {
        for (int j = lane; j < rows * F16_OBS_DIM; j += 64) {
          const int r = j / F16_OBS_DIM, c = j - r * F16_OBS_DIM;
          dst[j] = img[IMG_OFF + r * KC + HC + c];
        }
      }
      __builtin_amdgcn_wave_barrier();
    } else if (live) {
#pragma unroll
      for (int c = 0; c < F16_OBS_DIM; ++c) a.r_frame[k * F16_OBS_DIM + c] = a.obs_prev[k * KC + HC + c];
    }
  }
  if (WIN) {
    const int K = a.E.K, p = a.wpos;
    const bool reset_now = live && done && autoreset;
    if (live && K > 1 && (fresh || reset_now)) {  // rare: whole-window fills of reset lanes
      float* X = a.wx + k * a.wenv;
      if (fresh) {
        float f0p[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 v = reinterpret_cast<const float4*>(stg)[j * 64 + lane];
          f0p[4 * j] = v.x; f0p[4 * j + 1] = v.y; f0p[4 * j + 2] = v.z; f0p[4 * j + 3] = v.w;
        }
        for (int r = p - K + 1; r < p; ++r) put_slot(X + (int64_t)r * a.wrow, f0p);
      }
      if (reset_now)  // after the fresh fill: a one-step episode ends in its own reset window
        for (int r = p - K + 1; r < p; ++r) put_slot(X + (int64_t)r * a.wrow, f0);
    }
    // this step's frame at position p of both histories (wx: the reset frame of a lane reset
    // now, else the new frame; wy: the new frame). The wave's 64 slots are one contiguous
    // 4 KiB block; the wave transposes them through its LDS staging area so that each dwordx4
    // store instruction writes 1 KiB contiguous (16 whole slots, 4 lanes per slot) instead of a
    // 16-B quarter of every slot. Swizzle: quarter j of slot r at float4 r*4 + (j ^ (r>>2 & 3)),
    // conflict-free on both the per-lane writes and the per-slot reads.
    // A wave none of whose lanes was reset now (~94 % of waves in the bench's steady state) has
    // the same 64 slots for both histories: one LDS staging pass, each transposed float4 read
    // once and stored twice (round 6; was two passes for every wave: 4 ds_write_b128 + 4
    // ds_read_b128 and two wave barriers per wave per step saved). The byte count is unchanged:
    // both histories must hold every frame for the (N, K, 15) strided view to alternate parity
    // (DESIGN.md 9 item 7).
#ifdef F16_TWO_PASS_SLOTS  // (A/B reference: round 5's two staging passes for every wave)
    const bool one_pass = false;
#else
    const bool one_pass = !ROLL && rows == EPW && __ballot(reset_now) == 0;
#endif
    if (one_pass) {
      float4* st4 = reinterpret_cast<float4*>(stg);
      const int q = lane & 3, sw = (lane >> 2) & 3;
      __builtin_amdgcn_wave_barrier();
      st4[lane * 4 + (0 ^ sw)] = make_float4(f[0], f[1], f[2], f[3]);
      st4[lane * 4 + (1 ^ sw)] = make_float4(f[4], f[5], f[6], f[7]);
      st4[lane * 4 + (2 ^ sw)] = make_float4(f[8], f[9], f[10], f[11]);
      st4[lane * 4 + (3 ^ sw)] = make_float4(f[12], f[13], f[14], 0.0f);
      __builtin_amdgcn_wave_barrier();
      const int64_t off = (int64_t)p * a.wrow + (row0 + (lane >> 2)) * a.wenv + 4 * q;
      float* const dx = a.wx + off;
      float* const dy = a.wy + off;
      float4 v[EPW / 16];
#pragma unroll
      for (int j = 0; j < EPW / 16; ++j) {
        const int r = 16 * j + (lane >> 2);
        v[j] = st4[r * 4 + (q ^ ((r >> 2) & 3))];
      }
#pragma unroll
      for (int j = 0; j < EPW / 16; ++j) st16<NT>(reinterpret_cast<float4*>(dx + (int64_t)(16 * j) * a.wenv), v[j]);
#ifndef F16_DIAG_ONE_HIST  // (timing-only bound of a single history: wrong results by design, never shipped)
#pragma unroll
      for (int j = 0; j < EPW / 16; ++j) st16<NT>(reinterpret_cast<float4*>(dy + (int64_t)(16 * j) * a.wenv), v[j]);
#endif
      __builtin_amdgcn_wave_barrier();
    } else if (rows == EPW) {
      float4* st4 = reinterpret_cast<float4*>(stg);
      const int q = lane & 3, sw = (lane >> 2) & 3;
      float* const hist[2] = {a.wx, a.wy};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float* fr = (h == 0 && reset_now) ? f0 : f;
        __builtin_amdgcn_wave_barrier();
        st4[lane * 4 + (0 ^ sw)] = make_float4(fr[0], fr[1], fr[2], fr[3]);
        st4[lane * 4 + (1 ^ sw)] = make_float4(fr[4], fr[5], fr[6], fr[7]);
        st4[lane * 4 + (2 ^ sw)] = make_float4(fr[8], fr[9], fr[10], fr[11]);
        st4[lane * 4 + (3 ^ sw)] = make_float4(fr[12], fr[13], fr[14], 0.0f);
        __builtin_amdgcn_wave_barrier();
        float* dst = hist[h] + (int64_t)p * a.wrow + (row0 + (lane >> 2)) * a.wenv + 4 * q;
#pragma unroll
        for (int j = 0; j < EPW / 16; ++j) {
          const int r = 16 * j + (lane >> 2);
          st16<NT>(reinterpret_cast<float4*>(dst + (int64_t)(16 * j) * a.wenv), st4[r * 4 + (q ^ ((r >> 2) & 3))]);
        }
        if (ROLL && h == 0 && a.r_next_frame) {
          // the rollout's frame log: the returned observation's newest frame (the next slot's
          // frame), the wave's 64 rows as 960 contiguous floats: each lane writes its 15 floats
          // at a 15-float pitch into the (now free) staging area (odd pitch: conflict-free),
          // then 240 float4 go out linearly; a log whose rows are not 16-B aligned (N % 4 != 0)
          // takes dword stores
          float* sf = reinterpret_cast<float*>(st4);
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int c = 0; c < F16_OBS_DIM; ++c) sf[lane * F16_OBS_DIM + c] = fr[c];
          __builtin_amdgcn_wave_barrier();
          float* dstf = a.r_next_frame + row0 * F16_OBS_DIM;
          if (((uintptr_t)dstf & 15) == 0) {
            for (int u = lane; u < 64 * F16_OBS_DIM / 4; u += 64)
              reinterpret_cast<float4*>(dstf)[u] = reinterpret_cast<const float4*>(sf)[u];
          } else {
            for (int u = lane; u < 64 * F16_OBS_DIM; u += 64) dstf[u] = sf[u];
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    } else if (live) {
      const int64_t off = k * a.wenv + (int64_t)p * a.wrow;
      put_slot<NT>(a.wx + off, reset_now ? f0 : f);
      put_slot<NT>(a.wy + off, f);
      if (ROLL && a.r_next_frame) {
        const float* fr = reset_now ? f0 : f;
#pragma unroll
        for (int c = 0; c < F16_OBS_DIM; ++c) a.r_next_frame[k * F16_OBS_DIM + c] = fr[c];
      }
    }
    if (FEATW && a.fwx) {
      // the feature window (f16_feature_window_kernel's invariant, written here instead of by a
      // second launch): fx[p] = fy[p] = features of wx[p]; a lane reset now also fills
      // fx[p-K+1 .. p-1] and, ahead of the next step's window fill, fy[p-K+2 .. p-1]. The
      // wave's 64 rows (64 * 17 contiguous floats per history) leave through its staging area
      // (free after the frame stores) as float4.
      const int64_t rowN = a.E.n * FEAT_OUT;
      float y[FEAT_OUT];
      if (live) frame_features(reset_now ? f0 : f, y);
      if (rows == EPW) {
        float* sf = stg;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < FEAT_OUT; ++j) sf[lane * FEAT_OUT + j] = y[j];
        __builtin_amdgcn_wave_barrier();
        float* gx = a.fwx + (int64_t)p * rowN + row0 * FEAT_OUT;
        float* gy = a.fwy + (int64_t)p * rowN + row0 * FEAT_OUT;
        if (((((uintptr_t)gx) | ((uintptr_t)gy)) & 15) == 0) {
          for (int u = lane; u < 64 * FEAT_OUT / 4; u += 64) {
            const float4 v = reinterpret_cast<const float4*>(sf)[u];
            reinterpret_cast<float4*>(gx)[u] = v;
            reinterpret_cast<float4*>(gy)[u] = v;
          }
        } else {
          for (int u = lane; u < 64 * FEAT_OUT; u += 64) {
            gx[u] = sf[u];
            gy[u] = sf[u];
          }
        }
        // the window fills of the wave's reset lanes (rare), each lane's (row, feature) pairs
        // spread over the whole wave from the staging area (as f16_feature_window_kernel)
        const uint64_t rm = __ballot(reset_now);
        if (rm && K > 1) {
          const int items = (2 * K - 3) * FEAT_OUT;  // fx rows p-K+1 .. p-1, fy rows p-K+2 .. p-1
          for (uint64_t m = rm; m; m &= m - 1) {
            const int ee = __builtin_ctzll(m);
            const int64_t kk = row0 + ee;
            for (int it = lane; it < items; it += 64) {
              const int ri = it / FEAT_OUT, j = it - ri * FEAT_OUT;
              float* d = ri < K - 1 ? a.fwx + (int64_t)(p - K + 1 + ri) * rowN
                                    : a.fwy + (int64_t)(p - K + 2 + (ri - (K - 1))) * rowN;
              d[kk * FEAT_OUT + j] = sf[ee * FEAT_OUT + j];
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
      } else if (live) {
#pragma unroll
        for (int j = 0; j < FEAT_OUT; ++j) {
          a.fwx[(int64_t)p * rowN + k * FEAT_OUT + j] = y[j];
          a.fwy[(int64_t)p * rowN + k * FEAT_OUT + j] = y[j];
        }
      }
      if (rows != EPW && reset_now && K > 1) {  // a partial wave's reset lanes: one lane each
        for (int r = p - K + 1; r < p; ++r) {
#pragma unroll
          for (int j = 0; j < FEAT_OUT; ++j) {
            a.fwx[(int64_t)r * rowN + k * FEAT_OUT + j] = y[j];
            if (r > p - K + 1) a.fwy[(int64_t)r * rowN + k * FEAT_OUT + j] = y[j];
          }
        }
      }
    }
    if ((XV & XV_X) != 0 && a.poses) {
      // the pose export (F16_STEP_POSES, f16_poses_kernel's output written here instead of by a
      // second launch): the pose of the returned observation's newest frame; the wave's 64 rows
      // (640 contiguous floats) leave through its staging area as float4
      float po[10];
      if (live) pose_of_frame(reset_now ? f0 : f, po);
      if (rows == EPW) {
        float* sp = stg;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < 10; ++j) sp[lane * 10 + j] = po[j];
        __builtin_amdgcn_wave_barrier();
        float* g = a.poses + row0 * 10;
        if (((uintptr_t)g & 15) == 0) {
          for (int u = lane; u < 64 * 10 / 4; u += 64)
            reinterpret_cast<float4*>(g)[u] = reinterpret_cast<const float4*>(sp)[u];
        } else {
          for (int u = lane; u < 64 * 10; u += 64) g[u] = sp[u];
        }
        __builtin_amdgcn_wave_barrier();
      } else if (live) {
#pragma unroll
        for (int j = 0; j < 10; ++j) a.poses[k * 10 + j] = po[j];
      }
    }
    F16_STAMP(stamps, ST_COPY);
  } else if (image) {
    // 2) splice the new frame of row r into the image at row r+1's first frame, which the
    //    shifted copy never reads: out_flat[j] = img[j + 15] for the whole block. The stack
    //    DMA landed at the prologue wait, and a wave only touches its own image, so the steps
    //    below need no workgroup barrier (a wave's LDS accesses complete in order).
    __builtin_amdgcn_wave_barrier();
    if (live) {
      float* dst = img + IMG_OFF + (size_t)(lane + 1) * KC;
#pragma unroll
      for (int j = 0; j < F16_OBS_DIM; ++j) dst[j] = f[j];
    }
    __builtin_amdgcn_wave_barrier();
    // 3) finished rows: terminal obs = the spliced row; then the row becomes K x frame 0
    if (live && done) {
      float* src = img + IMG_OFF + (size_t)lane * KC + F16_OBS_DIM;
      if (a.tobs) {
        float* t = a.tobs + k * KC;
        if ((KC & 3) == 0) {  // K % 4 == 0: the row is 16-B aligned in HBM, dwordx4 stores
          for (int c = 0; c < KC; c += 4)
            *reinterpret_cast<float4*>(t + c) = make_float4(src[c], src[c + 1], src[c + 2], src[c + 3]);
        } else {
          for (int c = 0; c < KC; ++c) t[c] = src[c];
        }
      }
      if (autoreset)  // frame by frame: f0 indexed by literals (no per-element modulo / select chain)
        for (int r = 0; r < a.E.K; ++r)
#pragma unroll
          for (int j = 0; j < F16_OBS_DIM; ++j) src[r * F16_OBS_DIM + j] = f0[j];
    }
    __builtin_amdgcn_wave_barrier();
    F16_STAMP(stamps, ST_SYNC);
    // 4) one coalesced float4 copy of the block (obs blocks are 16-B aligned per wave)
    if (rows > 0) {
      float* out = a.obs + row0 * KC;
      const int total = rows * KC, n4 = total >> 2;
      float4* out4 = reinterpret_cast<float4*>(out);
      for (int q = lane; q < n4; q += 64) {
#if (IMG_OFF + F16_OBS_DIM) % 4 == 0
        out4[q] = reinterpret_cast<const float4*>(img + IMG_OFF + F16_OBS_DIM)[q];
#else
        const float* p = img + IMG_OFF + 4 * q + F16_OBS_DIM;
        out4[q] = make_float4(p[0], p[1], p[2], p[3]);
#endif
      }
      for (int j = 4 * n4 + lane; j < total; j += 64) out[j] = img[IMG_OFF + j + F16_OBS_DIM];
    }
    F16_STAMP(stamps, ST_COPY);
  } else {
    // fallback (large K): chunked flat copy from obs_prev, frames staged in LDS
    float* sF = dynl;
    float* sR = dynl + BLOCK * FRAME_PITCH;
    if (live) {
#pragma unroll
      for (int j = 0; j < F16_OBS_DIM; ++j) sF[threadIdx.x * FRAME_PITCH + j] = f[j];
      if (done)
#pragma unroll
        for (int j = 0; j < F16_OBS_DIM; ++j) sR[threadIdx.x * FRAME_PITCH + j] = f0[j];
    }
    __syncthreads();
    F16_STAMP(stamps, ST_SYNC);
    // A wave's 64 rows are one contiguous block of 64*K*15 floats in both obs_prev and obs,
    // and out[j] = prev[j + 15] except in each row's last frame: the wave walks the block with
    // flat, coalesced indices j = lane + 64*it; loads are issued in chunks of 16 before their
    // stores, and chunks only read ahead of what earlier chunks wrote (in-place safe).
    if (rows > 0) {
      const float* prev = a.obs_prev + row0 * KC;
      float* out = a.obs + row0 * KC;
      float* tout = a.tobs ? a.tobs + row0 * KC : nullptr;
      const int total = rows * KC;
      int row = lane / KC, col = lane - (lane / KC) * KC;
#ifndef F16_FALLBACK_CH
#define F16_FALLBACK_CH 16
#endif
      constexpr int CH = F16_FALLBACK_CH;
      for (int base = 0; base < total; base += 64 * CH) {
        float v[CH];
        int rw[CH], cl[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int j = base + 64 * u + lane;
          rw[u] = row; cl[u] = col;
          float x = 0.0f;
          if (j < total) {
            const int li = wave * 64 + row;
            x = (col < HC) ? prev[j + F16_OBS_DIM] : sF[li * FRAME_PITCH + (col - HC)];
          }
          v[u] = x;
          col += 64;
          while (col >= KC) { col -= KC; ++row; }
        }
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int j = base + 64 * u + lane;
          if (j < total) {
            const int li = wave * 64 + rw[u];
            if (!sDone[li]) {
              out[j] = v[u];
            } else {
              if (tout) tout[j] = v[u];
              out[j] = autoreset ? sR[li * FRAME_PITCH + (cl[u] % F16_OBS_DIM)] : v[u];
            }
          }
        }
      }
    }
    F16_STAMP(stamps, ST_COPY);
  }
#ifdef F16_STAMPS
  if (lane == 0) {
    const int w = (blockIdx.x * BLOCK + threadIdx.x) >> 6;
    if (w < (1 << 14))
      for (int q = 0; q < ST_N; ++q) g_stamps[w][q] = stamps.acc[q];
  }
#endif
}

#define STEP_SHARED                                       \
  __shared__ __align__(16) float sT[F16_BLOB_FLOATS];   \
  __shared__ __align__(16) float4 sTmpl[NCOL + TMPL_FRAME_COLS]; \
  __shared__ int sDone[BLOCK];                            \
  extern __shared__ __align__(16) float dynl[];

// Occupancy variants. The body needs ~300 registers (VGPR + AGPR), i.e. one wave per SIMD;
// OCC = 2 caps it at 256 (a few spills) so two waves share each SIMD: slower per wave, but
// when there are more waves than SIMDs (N > 64 x 4 x CUs) the pair overlaps one wave's
// memory phases and stalls with the other's VALU work (f16env_step picks per launch).
#define STEP_PRE_ARGS const float4 *__restrict__ sc, const float *__restrict__ act, const float4 *__restrict__ tmpl, int64_t n
__global__ __launch_bounds__(BLOCK, 1) void f16_step_kernel(STEP_PRE_ARGS, StepArgs a) {
  STEP_SHARED
  const StepPre pre = {sc, act, tmpl, n};
  step_body<0>(a, sT, sTmpl, sDone, dynl, &pre);
}
template <int MODE, int OCC, bool ROLL = false>
__global__ __launch_bounds__(BLOCK, OCC) void f16_step_var_kernel(STEP_PRE_ARGS, StepArgs a) {
  STEP_SHARED
  const StepPre pre = {sc, act, tmpl, n};
  step_body<MODE, false, ROLL, OCC == 2>(a, sT, sTmpl, sDone, dynl, &pre);
}
// global-table variant (large K on the LDS-image path): no LDS table copy
template <int MODE, bool ROLL = false>
__global__ __launch_bounds__(BLOCK, 1) void f16_step_gt_kernel(STEP_PRE_ARGS, StepArgs a) {
  __shared__ __align__(16) float4 sTmpl[NCOL + TMPL_FRAME_COLS];
  __shared__ int sDone[BLOCK];
  extern __shared__ __align__(16) float dynl[];
  const StepPre pre = {sc, act, tmpl, n};
  step_body<MODE, true, ROLL>(a, nullptr, sTmpl, sDone, dynl, &pre);
}
// windowed-observation build (f16env_step_window): no stack image, LDS holds the tables and
// the per-wave frame staging
// ROLL: the rollout-slot build (f16env_window_step_rollout: in-kernel Philox or clipped policy
// actions, the slot's actions / rewards / next starts and the returned observation's newest
// frame); the plain windowed step carries none of its code.
template <int MODE, int OCC, bool ROLL = false>
__global__ __launch_bounds__(BLOCK, OCC) void f16_step_win_kernel(const float4* __restrict__ sc, const float* __restrict__ act,
                                                                  const float4* __restrict__ tmpl, int64_t n, StepArgs a) {
  STEP_SHARED
  const StepPre pre = {sc, act, tmpl, n};
  step_body<MODE, false, ROLL, OCC == 2, true>(a, sT, sTmpl, sDone, dynl, &pre);
}
// ... with non-temporal state and frame-slot stores, for grids resident in one round (st16)
template <int MODE, int OCC, bool ROLL = false>
__global__ __launch_bounds__(BLOCK, OCC) void f16_step_win_nt_kernel(const float4* __restrict__ sc,
                                                                     const float* __restrict__ act,
                                                                     const float4* __restrict__ tmpl, int64_t n,
                                                                     StepArgs a) {
  STEP_SHARED
  const StepPre pre = {sc, act, tmpl, n};
  step_body<MODE, false, ROLL, OCC == 2, true, true>(a, sT, sTmpl, sDone, dynl, &pre);
}
// the windowed plain step with extras (XV_X | XV_FEAT: the feature window in the epilogue; every
// winx build takes act == NULL as "draw the actions in-kernel"): f16env_window_step_ex. A kernel
// of its own, so the headline instances above keep their instruction stream.
template <int MODE, int OCC, bool NT, int XV>
__global__ __launch_bounds__(BLOCK, OCC) void f16_step_winx_kernel(const float4* __restrict__ sc,
                                                                   const float* __restrict__ act,
                                                                   const float4* __restrict__ tmpl, int64_t n,
                                                                   StepArgs a) {
  STEP_SHARED
  const StepPre pre = {sc, act, tmpl, n};
  step_body<MODE, false, false, OCC == 2, true, NT, false, XV>(a, sT, sTmpl, sDone, dynl, &pre);
}
// the half-populated-wave experiment (HALF above): 256-register build, two waves per SIMD
template <int MODE>
__global__ __launch_bounds__(BLOCK, 2) void f16_step_win_half_kernel(const float4* __restrict__ sc,
                                                                     const float* __restrict__ act,
                                                                     const float4* __restrict__ tmpl, int64_t n,
                                                                     StepArgs a) {
  STEP_SHARED
  const StepPre pre = {sc, act, tmpl, n};
  step_body<MODE, false, false, true, true, true, true>(a, sT, sTmpl, sDone, dynl, &pre);
}
using StepKernel = void (*)(const float4*, const float*, const float4*, int64_t, StepArgs);
using WinKernel = StepKernel;
template <bool ROLL>
static WinKernel step_win_kernel_for_r(int mode, int occ, int nt) {
  static const WinKernel table[2][2][4] = {
      {{f16_step_win_kernel<0, 1, ROLL>, f16_step_win_kernel<1, 1, ROLL>, f16_step_win_kernel<2, 1, ROLL>,
        f16_step_win_kernel<3, 1, ROLL>},
       {f16_step_win_kernel<0, 2, ROLL>, f16_step_win_kernel<1, 2, ROLL>, f16_step_win_kernel<2, 2, ROLL>,
        f16_step_win_kernel<3, 2, ROLL>}},
      {{f16_step_win_nt_kernel<0, 1, ROLL>, f16_step_win_nt_kernel<1, 1, ROLL>, f16_step_win_nt_kernel<2, 1, ROLL>,
        f16_step_win_nt_kernel<3, 1, ROLL>},
       {f16_step_win_nt_kernel<0, 2, ROLL>, f16_step_win_nt_kernel<1, 2, ROLL>, f16_step_win_nt_kernel<2, 2, ROLL>,
        f16_step_win_nt_kernel<3, 2, ROLL>}}};
  return table[nt ? 1 : 0][occ == 2 ? 1 : 0][mode & 3];
}
static WinKernel step_win_kernel_for(int mode, int occ, int nt, bool roll = false) {
  return roll ? step_win_kernel_for_r<true>(mode, occ, nt) : step_win_kernel_for_r<false>(mode, occ, nt);
}
template <int XV>
static WinKernel step_winx_kernel_for_x(int mode, int occ, int nt) {
  static const WinKernel table[2][2][4] = {
      {{f16_step_winx_kernel<0, 1, false, XV>, f16_step_winx_kernel<1, 1, false, XV>,
        f16_step_winx_kernel<2, 1, false, XV>, f16_step_winx_kernel<3, 1, false, XV>},
       {f16_step_winx_kernel<0, 2, false, XV>, f16_step_winx_kernel<1, 2, false, XV>,
        f16_step_winx_kernel<2, 2, false, XV>, f16_step_winx_kernel<3, 2, false, XV>}},
      {{f16_step_winx_kernel<0, 1, true, XV>, f16_step_winx_kernel<1, 1, true, XV>,
        f16_step_winx_kernel<2, 1, true, XV>, f16_step_winx_kernel<3, 1, true, XV>},
       {f16_step_winx_kernel<0, 2, true, XV>, f16_step_winx_kernel<1, 2, true, XV>,
        f16_step_winx_kernel<2, 2, true, XV>, f16_step_winx_kernel<3, 2, true, XV>}}};
  return table[nt ? 1 : 0][occ == 2 ? 1 : 0][mode & 3];
}
static WinKernel step_winx_kernel_for(int mode, int occ, int nt, bool feat) {
  return feat ? step_winx_kernel_for_x<XV_X | XV_FEAT>(mode, occ, nt) : step_winx_kernel_for_x<XV_X>(mode, occ, nt);
}
static constexpr size_t WIN_DYN_LDS = sizeof(float) * (BLOCK / 64) * WIN_WAVE_FLOATS;
// variant: 0 = LDS tables, 1 wave/SIMD; 1 = LDS tables, 2 waves/SIMD; 2 = global tables.
// roll: the rollout-slot build (f16env_step_rollout); the plain step carries none of its code.
static StepKernel step_kernel_for(int mode, int variant, bool roll = false) {
  static const StepKernel table[2][3][4] = {
      {{f16_step_kernel, f16_step_var_kernel<1, 1>, f16_step_var_kernel<2, 1>, f16_step_var_kernel<3, 1>},
       {f16_step_var_kernel<0, 2>, f16_step_var_kernel<1, 2>, f16_step_var_kernel<2, 2>, f16_step_var_kernel<3, 2>},
       {f16_step_gt_kernel<0>, f16_step_gt_kernel<1>, f16_step_gt_kernel<2>, f16_step_gt_kernel<3>}},
      {{f16_step_var_kernel<0, 1, true>, f16_step_var_kernel<1, 1, true>, f16_step_var_kernel<2, 1, true>,
        f16_step_var_kernel<3, 1, true>},
       {f16_step_var_kernel<0, 2, true>, f16_step_var_kernel<1, 2, true>, f16_step_var_kernel<2, 2, true>,
        f16_step_var_kernel<3, 2, true>},
       {f16_step_gt_kernel<0, true>, f16_step_gt_kernel<1, true>, f16_step_gt_kernel<2, true>,
        f16_step_gt_kernel<3, true>}}};
  return table[roll ? 1 : 0][variant < 0 || variant > 2 ? 0 : variant][mode & 3];
}

// ------------------------------------------------------------------------------------------
// Persistent rollout under the uniform random policy (f16env_rollout_random /
// f16env_window_rollout_random): T env steps of every lane in ONE launch. The actions come from
// the f16env_sample_actions Philox stream, so no step waits for a host or a policy: each lane
// keeps its state in registers across the whole rollout and per step writes only the rollout
// slot -- the action, reward and next episode start of step t, and the newest frame of the
// observation it returns, which is the frame slot t + 1 acts on (frames[0] is the newest frame
// of the observation before step 0). No frame stack is kept on chip: the final observation is
// rebuilt at the end from the frame log the lane wrote (obs[j] = F[max(T-K+1+j, s)], s the
// lane's last episode start, F[T] the last frame in registers, F[t <= 0] from the observation
// before the rollout -- rollout.py rebuild_observations), so K is not bounded by LDS (round 3's
// ring held K <= 8 frames per lane). cfg5 modes (MODE != 0): gusts per step as the step kernel,
// and a finished lane resets from the reset cache when it holds its next episode's row (the
// first reset of a lane in the rollout; f16_ic_fill_kernel fills it before the launch), else
// by its own RunIC. Same arithmetic, RNG streams and auto-reset as T launches of the fused step
// (f16env_step_rollout / f16env_window_step_rollout): bit-identical results (build.py
// -ffp-contract=on: contraction is fixed per source expression, not per kernel).
// ------------------------------------------------------------------------------------------
struct RollArgs {
  SoA s, tmpl, icc;       // icc: cfg5 reset cache (MODE != 0; c == nullptr: every reset a RunIC)
  // the observation before step 0: frame j of lane k at obs_prev + k * in_row + j * in_pitch
  // (contiguous N x K x 15: K*15, 15; a position-major window: 16, N*16)
  const float* obs_prev;
  int64_t in_row, in_pitch;
  // the observation after step T-1, written the same way to out0 and (when not NULL) out1 --
  // the two window histories -- with out_slot floats per frame (15, or 16: a 64-B slot)
  float* out0;
  float* out1;
  int64_t out_row, out_pitch;
  int32_t out_slot;
  float* frames;          // T x N x 15: frames[t] = newest frame of the observation step t acts on
  float* actions;         // T x N x 4
  float* rewards;         // T x N
  float* next_start;      // (T - 1) x N: 1.0 where the lane finished at step t < T-1
  float* last_start;      // N: the same for step T-1
  unsigned long long* nonfinite;  // [0] F16_FLAG_NAN_GUARD quarantines, [2] F16_FLAG_OBS_CHECK
  uint64_t seed, step0;
  int32_t T;
  int32_t clear_fresh;    // both output windows are whole: no lane needs a FRESH fill next step
  EnvArgs E;
  ModelConsts C;
};
template <int MODE, int OCC>
__global__ __launch_bounds__(BLOCK, OCC) void f16_rollout_kernel(RollArgs a) {
  __shared__ __align__(16) float sT[F16_BLOB_FLOATS];
  __shared__ __align__(16) float4 sTmpl[NCOL + TMPL_FRAME_COLS];
  __shared__ __align__(16) float4 sF[BLOCK * 4];  // per wave: its 64 new frames as [64][4] float4
  constexpr bool GUST = (MODE & 2) != 0;
  const int K = a.E.K, tid = threadIdx.x;
  const int64_t k = (int64_t)blockIdx.x * BLOCK + tid;
  const int64_t N = a.E.n;
  const bool live = k < N;
  stage_tables_issue(sT);
  if (MODE == 0 && tid < NCOL + TMPL_FRAME_COLS)
    dma16(reinterpret_cast<const float*>(a.tmpl.c + (tid < NCOL ? tid : tid + NCOL_ALL - NCOL)),
          reinterpret_cast<float*>(sTmpl));
  Lane L;
  float fn[F16_OBS_DIM];  // newest frame of the lane's current observation
  if (live) {
    lane_load<GUST>(a.s, k, L);
    const float* op = a.obs_prev + k * a.in_row + (int64_t)(K - 1) * a.in_pitch;
#pragma unroll
    for (int c = 0; c < F16_OBS_DIM; ++c) fn[c] = op[c];
  }
  VM_DRAIN();
  __syncthreads();
  if (!live) return;  // no barrier below
  const int wave = tid >> 6, lane = tid & 63;
  const int64_t row0 = (int64_t)blockIdx.x * BLOCK + wave * 64;
  // a full wave writes its 64 frames (3 840 contiguous bytes) as 240 float4 gathered from its
  // LDS staging, instead of fifteen 4-byte stores per lane at a 60-byte stride
  const bool coalesced = N - row0 >= 64 && (N * F16_OBS_DIM) % 4 == 0 && ((uintptr_t)a.frames & 15) == 0;
  float4* stg = sF + wave * 256;
  auto put_frame = [&](int64_t t) {  // frames[t] = fn for every lane of the wave
    if (coalesced) {
      __builtin_amdgcn_wave_barrier();
      stg[lane * 4 + 0] = make_float4(fn[0], fn[1], fn[2], fn[3]);
      stg[lane * 4 + 1] = make_float4(fn[4], fn[5], fn[6], fn[7]);
      stg[lane * 4 + 2] = make_float4(fn[8], fn[9], fn[10], fn[11]);
      stg[lane * 4 + 3] = make_float4(fn[12], fn[13], fn[14], 0.0f);
      __builtin_amdgcn_wave_barrier();
      const float* src = reinterpret_cast<const float*>(stg);
      float4* dst = reinterpret_cast<float4*>(a.frames + (t * N + row0) * F16_OBS_DIM);
      for (int q = lane; q < 64 * F16_OBS_DIM / 4; q += 64) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = 4 * q + i, r = e / F16_OBS_DIM;
          v[i] = src[r * 16 + (e - r * F16_OBS_DIM)];
        }
        dst[q] = make_float4(v[0], v[1], v[2], v[3]);
      }
    } else {
      float* fr = a.frames + (t * N + k) * F16_OBS_DIM;
#pragma unroll
      for (int c = 0; c < F16_OBS_DIM; ++c) fr[c] = fn[c];
    }
  };
  put_frame(0);
  const uint64_t gid = (uint64_t)(a.E.id_base + k);
  int last_s = -(1 << 30);  // index t of the lane's last reset frame F[t] in this rollout (none yet)
  bool cache_fresh = a.icc.c != nullptr;  // the cached row can only serve the lane's first reset
  for (int t = 0; t < a.T; ++t) {
    const float4 av = philox_action(a.seed, gid, a.step0 + (uint64_t)t);
    const float cmd[4] = {av.x, av.y, av.z, av.w};
    L.step += 1;  L.flags &= ~LANE_FLAG_FRESH;                                              // jsbsim_gym.py:215
    if (GUST) {  // cfg5 Gauss-Markov gust update, once per env step before the frames (as step_body)
      float xi[3];
      rng_normals(a.E.seed, gid, (uint32_t)(L.ep_count - 1), (uint32_t)L.step, xi);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        L.gust[j] = __builtin_fmaf(a.E.gust_a, L.gust[j], a.E.gust_b * xi[j]);
        L.wind[j] = L.wst[j] + L.gust[j];
      }
    }
    double ce, se;
    earth_angle(L.epa, ce, se);
    const AltRef A = alt_ref(L, ce, se);
#ifdef F16_STAMPS
    Stamps stamps = {};
#endif
    for (int s = 0; s < a.E.down_sample; ++s)
      frame<OCC == 2, GUST>(L, cmd, ce, se, A, sT, a.C, false F16_STAMP_PASS);  // :225-232
    float f[F16_OBS_DIM];
    make_frame(L, ce, se, A, f);                              // :234
    float r32;
    const int fl = env_reward(L, f, a.E, r32);
    const int done = fl & 3;
    if (a.E.flags & F16_FLAG_NAN_GUARD) {
      const unsigned long long qm = __ballot(fl & 4);
      if (qm && lane == 0) atomicAdd(a.nonfinite, (unsigned long long)__popcll(qm));
    }
    if (a.E.flags & F16_FLAG_OBS_CHECK) {  // jsbsim_gym.py:268-285 on the new frame
      const unsigned long long om = __ballot(obs_out_of_bounds(f));
      if (om && lane == 0) atomicAdd(a.nonfinite + 2, (unsigned long long)__popcll(om));
    }
    const int64_t row = (int64_t)t * N + k;
    reinterpret_cast<float4*>(a.actions)[row] = av;
    a.rewards[row] = r32;
    if (t + 1 < a.T) a.next_start[row] = done ? 1.0f : 0.0f;
    else a.last_start[k] = done ? 1.0f : 0.0f;
    if (done) {  // dummy_vec_env.py:68-71: the next observation is K x the reset frame
      if (MODE == 0) {
        lane_reset_template(L, sTmpl, a.E, k, fn);
      } else if (cache_fresh && __float_as_int(a.icc.c[(int64_t)15 * a.icc.n + k].w) == L.ep_count + 1) {
        lane_load<GUST>(a.icc, k, L);  // the lane's next reset, evaluated ahead (f16_ic_fill_kernel)
#pragma unroll
        for (int j = 0; j < TMPL_FRAME_COLS; ++j) {
          const float4 v = a.icc.c[(int64_t)(NCOL_ALL + j) * a.icc.n + k];
          fn[4 * j] = v.x; fn[4 * j + 1] = v.y; fn[4 * j + 2] = v.z; fn[4 * j + 3] = v.w;
        }
        fn[12] = L.goal[0]; fn[13] = L.goal[1]; fn[14] = L.goal[2];
        cache_fresh = false;
      } else {
        lane_reset_mode<MODE, OCC == 2>(L, a.E, k, sT, a.C, fn);
        cache_fresh = false;
      }
      last_s = t + 1;
    } else {
#pragma unroll
      for (int c = 0; c < F16_OBS_DIM; ++c) fn[c] = f[c];
    }
    if (t + 1 < a.T) put_frame(t + 1);
  }
  if (a.clear_fresh) L.flags &= ~LANE_FLAG_FRESH;
  lane_store<GUST>(a.s, k, L);
  // the final observation, oldest frame first: F[max(T-K+1+j, last_s)]; F[T] = fn, F[1..T-1] from
  // this wave's own frame-log rows (made visible to the reads by the fence), F[t <= 0] from the
  // observation before the rollout (F[0] is also frames[0])
  __threadfence();
  const int T = a.T;
  for (int j = 0; j < K; ++j) {
    const int idx = max(T - K + 1 + j, last_s);
    float v[F16_OBS_DIM];
    if (idx == T) {
#pragma unroll
      for (int c = 0; c < F16_OBS_DIM; ++c) v[c] = fn[c];
    } else if (idx >= 1) {
      const float* src = a.frames + ((int64_t)idx * N + k) * F16_OBS_DIM;
#pragma unroll
      for (int c = 0; c < F16_OBS_DIM; ++c) v[c] = __builtin_nontemporal_load(src + c);
    } else {
      const float* src = a.obs_prev + k * a.in_row + (int64_t)(idx + K - 1) * a.in_pitch;
#pragma unroll
      for (int c = 0; c < F16_OBS_DIM; ++c) v[c] = src[c];
    }
    F16_CHECK(idx >= 1 - K && idx <= T, DBG_RING_SLOT);
    for (int b = 0; b < 2; ++b) {
      float* o = (b == 0 ? a.out0 : a.out1);
      if (!o) continue;
      o += k * a.out_row + (int64_t)j * a.out_pitch;
#pragma unroll
      for (int c = 0; c < F16_OBS_DIM; ++c) o[c] = v[c];
      if (a.out_slot > F16_OBS_DIM) o[F16_OBS_DIM] = 0.0f;
    }
  }
}

// cfg5 auto-reset of the lanes a deferred-mode step finished (done list from its ballot
// compaction): full RunIC (random IC box, gust start) and K x frame 0 into their obs rows.
struct ResetDoneArgs {
  SoA s, tmpl;
  const int32_t* done_idx;
  const int32_t* n_done;
  float* obs;       // frame r of env k at obs + k * obs_row + obs_off + r * obs_pitch, obs_slot
                    // floats written per frame (contiguous: K*15, 0, 15, 15; window:
                    // 16, (p-K+1)*N*16, N*16, 16)
  int64_t obs_row, obs_off, obs_pitch;
  int32_t obs_slot;
  int32_t* zero_next;  // the handle's other done counter (the next step's): zeroed here, so a
                       // step needs no memset of its counter
  EnvArgs E;
  ModelConsts C;
};
__global__ __launch_bounds__(BLOCK) void f16_reset_done_kernel(ResetDoneArgs a) {
  __shared__ __align__(16) float sT[F16_BLOB_FLOATS];
  if (a.zero_next && blockIdx.x == 0 && threadIdx.x == 0) *a.zero_next = 0;
  // one round trip before the work: the table DMA, the done count and this thread's first list
  // entry in flight together (the list holds N entries, so the speculative read is in bounds)
  stage_tables_issue(sT);
  const int64_t i0 = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  const int nd = *a.n_done;
  const int32_t k0 = i0 < a.E.n ? a.done_idx[i0] : -1;
  VM_DRAIN();
  __syncthreads();
  if ((int64_t)blockIdx.x * BLOCK >= nd) return;  // after the only barrier
  for (int64_t i = i0; i < nd; i += (int64_t)gridDim.x * BLOCK) {
    const int64_t k = i == i0 ? k0 : a.done_idx[i];
    F16_CHECK(k >= 0 && k < a.E.n, DBG_RESET_INDEX);
    if (k < 0 || k >= a.E.n) continue;
    Lane L;
    lane_load<true>(a.s, k, L);
    float f0[F16_OBS_DIM];
    lane_reset(L, a.tmpl, nullptr, nullptr, a.E, k, sT, a.C, f0);
    lane_store<true>(a.s, k, L);
    float* o = a.obs + k * a.obs_row + a.obs_off;
    for (int r = 0; r < a.E.K; ++r)
      for (int j = 0; j < a.obs_slot; ++j) o[r * a.obs_pitch + j] = j < F16_OBS_DIM ? f0[j] : 0.0f;
  }
}

// cfg5 reset cache (windowed layout): a lane's next reset -- RunIC of its random IC, gust
// start, goal, frame 0 -- is a pure function of (seed, global env id, episode), so it is
// evaluated ahead, here, for every lane whose cached row is not the one of its next episode
// (tag: the row's episode count = the lane's + 1), and the windowed step copies it into a
// finished lane like MODE 0's template reset. Run every ICC_PERIOD windowed steps (and at the
// first): the lanes that reset since the last fill are refilled; a lane that finishes again
// before that runs its RunIC inside the step. Columns: NCOL_ALL state columns, then frame 0
// without the goal (TMPL_FRAME_COLS).
enum { ICC_COLS = NCOL_ALL + TMPL_FRAME_COLS };
template <int MODE>
__global__ __launch_bounds__(BLOCK) void f16_ic_fill_kernel(SoA s, SoA cache, EnvArgs E, ModelConsts C) {
  __shared__ __align__(16) float sT[F16_BLOB_FLOATS];
  stage_tables(sT);
  const int64_t k = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (k >= E.n) return;
  const int32_t ep = __float_as_int(s.c[(int64_t)15 * s.n + k].w);
  if (__float_as_int(cache.c[(int64_t)15 * cache.n + k].w) == ep + 1) return;
  Lane L;
  L.ep_count = ep;
  L.flags = 0;
  float f0[F16_OBS_DIM];
  lane_reset_mode<MODE>(L, E, k, sT, C, f0);
  lane_store<true>(cache, k, L);
  for (int j = 0; j < TMPL_FRAME_COLS; ++j)
    cache.c[(int64_t)(NCOL_ALL + j) * cache.n + k] = make_float4(f0[4 * j], f0[4 * j + 1], f0[4 * j + 2], f0[4 * j + 3]);
}

struct ResetArgs {
  SoA s, tmpl;
  const uint8_t* mask;
  const float* goals;
  const double* ic;
  float* obs;       // frame addressing as ResetDoneArgs
  int64_t obs_row, obs_off, obs_pitch;
  int32_t obs_slot;
  int* wind_any;    // per-lane IC given: set if a lane got wind (the handle needs the wind kernels)
  EnvArgs E;
  ModelConsts C;
};
__global__ __launch_bounds__(BLOCK) void f16_reset_kernel(ResetArgs a) {
  __shared__ __align__(16) float sT[F16_BLOB_FLOATS];
  stage_tables(sT);
  const int64_t k = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (k >= a.E.n) return;
  if (a.mask && !a.mask[k]) return;
  Lane L;
  lane_load<true>(a.s, k, L);
  float f0[F16_OBS_DIM];
  // a goal row whose x is NaN draws the lane's goal from the device stream (mixed seeded /
  // unseeded resets in ONE call: the episode counter advances once per reset)
  const float* g = a.goals ? a.goals + 3 * k : nullptr;
  if (g && isnan(g[0])) g = nullptr;
  lane_reset(L, a.tmpl, a.ic ? a.ic + (int64_t)F16_IC_N * k : nullptr, g, a.E, k, sT, a.C, f0);
  lane_store<true>(a.s, k, L);
  if (a.wind_any && (L.wst[0] != 0.0f || L.wst[1] != 0.0f || L.wst[2] != 0.0f)) atomicOr(a.wind_any, 1);
  if (a.obs) {
    float* o = a.obs + k * a.obs_row + a.obs_off;
    for (int r = 0; r < a.E.K; ++r)
      for (int j = 0; j < a.obs_slot; ++j) o[r * a.obs_pitch + j] = j < F16_OBS_DIM ? f0[j] : 0.0f;
  }
}

// windowed observations: the histories' last K-1 frame positions (p_old-K+2 .. p_old) move to
// the front (0 .. K-2) of both histories, so the next step writes its frame at K-1. One lane
// per float4 of a slot; (wenv, wpos) as StepArgs (wrow, wenv).
__global__ void f16_window_restart_kernel(int64_t n, int32_t K, int64_t wenv, int64_t wpos, int32_t p_src, float* h0,
                                          float* h1) {
  const int64_t per = (int64_t)(K - 1) * n * 4;  // float4 per history
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * per) return;
  const int64_t b = i >= per, t = i - b * per;
  F16_CHECK(p_src >= 1, DBG_WINDOW_POS);
  float* h = b ? h1 : h0;
  if (wenv == 4 * 4 && wpos == n * 16) {  // position-major: the K-1 positions are one block
    float4* h4 = reinterpret_cast<float4*>(h);
    h4[t] = h4[(int64_t)p_src * n * 4 + t];
    return;
  }
  const int64_t q = t & 3, u = t >> 2;
  const int64_t k = u % n, r = u / n;
  float* d = h + k * wenv + r * wpos + 4 * q;
  *reinterpret_cast<float4*>(d) = *reinterpret_cast<const float4*>(d + (int64_t)p_src * wpos);
}

// IC -> state (used once at create to build the reset template, n = 1)
__global__ void f16_ic_kernel(SoA dst, const double* ic, ModelConsts C) {
  __shared__ __align__(16) float sT[F16_BLOB_FLOATS];
  stage_tables(sT);
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Lane L;
  memset(&L, 0, sizeof L);
  apply_ic(L, ic, sT, C);
  L.ep_ret = 0.0; L.step = 0; L.ep_count = 0; L.last_d = 0.0f;
  L.goal[0] = L.goal[1] = L.goal[2] = 0.0f;
  lane_store<true>(dst, 0, L);  // with the config IC's wind columns (read by wind-kernel resets)
  // frame 0 of the template (goal excluded): what every template auto-reset would evaluate
  float f[F16_OBS_DIM];
  make_frame(L, 1.0, 0.0, alt_ref(L, 1.0, 0.0), f);
  for (int j = 0; j < TMPL_FRAME_COLS; ++j)
    dst.c[NCOL_ALL + j] = make_float4(f[4 * j], f[4 * j + 1], f[4 * j + 2], f[4 * j + 3]);
}

__global__ void f16_get_state_kernel(SoA s, double* c, ModelConsts C) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= s.n) return;
  Lane L;
  lane_load<true>(s, k, L);
  double* o = c + (int64_t)F16C_N * k;
  for (int j = 0; j < 3; ++j) {
    o[F16C_RI + j] = L.rI[j]; o[F16C_VI + j] = L.vI[j];
    o[F16C_VIH1 + j] = L.vI[j] - (double)L.ndv1[j];  // vI + dv1
    o[F16C_VIH2 + j] = L.vI[j] + (double)L.dv2[j];
    o[F16C_AI + j] = L.aI[j]; o[F16C_AIP + j] = L.aIp[j]; o[F16C_WI + j] = L.wI[j];
    o[F16C_WID + j] = L.wId[j]; o[F16C_BA + j] = L.ba[j]; o[F16C_GOAL + j] = L.goal[j];
    o[F16C_WIND + j] = L.wst[j];
    o[F16C_GUST + j] = L.gust[j];
  }
  for (int j = 0; j < 4; ++j) { o[F16C_Q + j] = L.q[j]; o[F16C_CMD + j] = 0.0; }
  o[F16C_EPA_C] = cos(L.epa); o[F16C_EPA_S] = sin(L.epa);
  o[F16C_TEF] = L.tef; o[F16C_AIL] = L.ail; o[F16C_ELE] = L.ele; o[F16C_RUD] = L.rud;
  o[F16C_LEF] = L.lef; o[F16C_SB] = L.sb;
  o[F16C_PID_R_I] = L.pri; o[F16C_PID_R_P] = L.prp; o[F16C_PID_P_I] = L.ppi;
  o[F16C_PID_P_P] = L.ppp; o[F16C_PID_Y_I] = L.pyi; o[F16C_PID_Y_P] = L.pyp;
  o[F16C_N1] = L.n1; o[F16C_N2] = L.n2; o[F16C_AUG] = (L.flags & LANE_FLAG_AUG) ? 1.0 : 0.0;
  for (int j = 0; j < F16L_N; ++j) o[F16C_LX + j] = L.lx[j];
  o[F16C_LX + F16L_VC_KTS] = vcas_from_qc(L.lx[F16L_VC_KTS], C);  // the latch holds qc
  o[F16C_LAST_D] = L.last_d; o[F16C_STEP] = L.step; o[F16C_EP_RET] = L.ep_ret;
  o[F16C_EP_COUNT] = (double)(uint32_t)L.ep_count;
}

__global__ void f16_set_state_kernel(SoA s, const double* c, ModelConsts C, int* wind_any) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= s.n) return;
  Lane L;
  const double* o = c + (int64_t)F16C_N * k;
  for (int j = 0; j < 3; ++j) {
    L.rI[j] = o[F16C_RI + j]; L.vI[j] = o[F16C_VI + j];
    L.ndv1[j] = -(float)(o[F16C_VIH1 + j] - o[F16C_VI + j]);
    L.dv2[j] = (float)(o[F16C_VIH2 + j] - o[F16C_VI + j]);
    L.aI[j] = (float)o[F16C_AI + j]; L.aIp[j] = (float)o[F16C_AIP + j]; L.wI[j] = (float)o[F16C_WI + j];
    L.wId[j] = (float)o[F16C_WID + j]; L.ba[j] = (float)o[F16C_BA + j]; L.goal[j] = (float)o[F16C_GOAL + j];
    L.wst[j] = (float)o[F16C_WIND + j];
    L.gust[j] = (float)o[F16C_GUST + j];
    L.wind[j] = L.wst[j] + L.gust[j];
  }
  for (int j = 0; j < 4; ++j) L.q[j] = (float)o[F16C_Q + j];
  L.epa = atan2(o[F16C_EPA_S], o[F16C_EPA_C]);
  L.tef = (float)o[F16C_TEF]; L.ail = (float)o[F16C_AIL]; L.ele = (float)o[F16C_ELE];
  L.rud = (float)o[F16C_RUD]; L.lef = (float)o[F16C_LEF]; L.sb = (float)o[F16C_SB];
  L.pri = (float)o[F16C_PID_R_I]; L.prp = (float)o[F16C_PID_R_P]; L.ppi = (float)o[F16C_PID_P_I];
  L.ppp = (float)o[F16C_PID_P_P]; L.pyi = (float)o[F16C_PID_Y_I]; L.pyp = (float)o[F16C_PID_Y_P];
  L.n1 = (float)o[F16C_N1]; L.n2 = (float)o[F16C_N2];
  // FRESH (the lane's other window history still lacks its reset frames) describes the
  // handle's observation histories, not the physics state, so it survives a set_state: a
  // reset -> set_state -> step sequence still fills the new window from the reset frame
  // (f16env_window_clear_fresh drops it once the caller has written whole windows)
  const bool fresh = sign_flag(s.c[(int64_t)14 * s.n + k].x);
  L.flags = (o[F16C_AUG] != 0.0 ? LANE_FLAG_AUG : 0) | (fresh ? LANE_FLAG_FRESH : 0);
  for (int j = 0; j < F16L_N; ++j) L.lx[j] = (float)o[F16C_LX + j];
  L.lx[F16L_VC_KTS] = qc_from_vcas(o[F16C_LX + F16L_VC_KTS], C);
  L.last_d = (float)o[F16C_LAST_D]; L.step = (int32_t)o[F16C_STEP]; L.ep_ret = o[F16C_EP_RET];
  L.ep_count = (int32_t)(uint32_t)o[F16C_EP_COUNT];
  lane_store<true>(s, k, L);
  // a lane with wind needs the wind kernels (f16env_set_state switches the handle)
  bool w = false;
  for (int j = 0; j < 3; ++j) w = w || L.wst[j] != 0.0f || L.gust[j] != 0.0f;
  if (w) atomicOr(wind_any, 1);
}

// the caller wrote whole observation windows into both histories (F16Envs.set_obs): no lane
// needs its window filled from a reset frame any more (the FRESH sign bit of column 14's x)
__global__ void f16_clear_fresh_kernel(SoA s) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= s.n) return;
  float* y = &s.c[(int64_t)14 * s.n + k].x;
  *y = without_sign_flag(*y);
}

// Trim: Newton on (alpha, elevator cmd, throttle cmd), mirrors oracle trim_one()
__device__ void trim_residual(const double* icb, const float* x, const float* T, const ModelConsts& C,
                              float* res) {
  double ic[F16_IC_N];
  for (int j = 0; j < F16_IC_N; ++j) ic[j] = icb[j];
  const double vt = icb[F16_IC_U_FPS];
  ic[F16_IC_U_FPS] = vt * cos((double)x[0]);
  ic[F16_IC_V_FPS] = 0.0;
  ic[F16_IC_W_FPS] = vt * sin((double)x[0]);
  ic[F16_IC_THETA_RAD] = x[0];
  ic[F16_IC_PHI_RAD] = 0.0;
  ic[F16_IC_P_RPS] = ic[F16_IC_Q_RPS] = ic[F16_IC_R_RPS] = 0.0;
  ic[F16_IC_CMD_AIL] = 0.0; ic[F16_IC_CMD_RUD] = 0.0;
  ic[F16_IC_CMD_ELE] = x[1];
  ic[F16_IC_CMD_THR] = x[2];
  Lane L;
  L.gust[0] = L.gust[1] = L.gust[2] = 0.0f;
  apply_ic(L, ic, T, C);
  // FGAccelerations::CalculateUVWdot: specific force + gravity - (pqr + 2 w_b) x uvw
  // - Ti2b (w x (w x rI))
  Derived d;
  derive(L, 1.0, 0.0, alt_ref(L, 1.0, 0.0), d);
  float gb[3];
  mvec(d.Ti2b, d.gI, gb);
  const float we = (float)OMEGA_E;
  const float wb[3] = {d.Ti2b[2] * we, d.Ti2b[5] * we, d.Ti2b[8] * we};
  const float t[3] = {d.pqr[0] + 2.0f * wb[0], d.pqr[1] + 2.0f * wb[1], d.pqr[2] + 2.0f * wb[2]};
  float c1[3];
  crossf(t, d.uvw, c1);
  const double w2 = OMEGA_E * OMEGA_E;
  const float wxwxr[3] = {(float)(-w2 * L.rI[0]), (float)(-w2 * L.rI[1]), 0.0f};
  float cent[3];
  mvec(d.Ti2b, wxwxr, cent);
  res[0] = L.ba[0] + gb[0] - c1[0] - cent[0];
  res[1] = L.ba[2] + gb[2] - c1[2] - cent[2];
  res[2] = L.wId[1];
}
__device__ void inv3f(const float* M, float* I, bool& ok) {
  const float a = M[0], b = M[1], c = M[2], d = M[3], e = M[4], f = M[5], g = M[6], h = M[7], k = M[8];
  const float A = e * k - f * h, B = -(d * k - f * g), Cc = d * h - e * g;
  const float det = a * A + b * B + c * Cc;
  ok = det != 0.0f;
  const float r = ok ? 1.0f / det : 0.0f;
  I[0] = A * r; I[1] = -(b * k - c * h) * r; I[2] = (b * f - c * e) * r;
  I[3] = B * r; I[4] = (a * k - c * g) * r; I[5] = -(a * f - c * d) * r;
  I[6] = Cc * r; I[7] = -(a * h - b * g) * r; I[8] = (a * e - b * d) * r;
}
__global__ __launch_bounds__(BLOCK) void f16_trim_kernel(int64_t n, const double* ic_in, double* ic_out,
                                                         double* resid, ModelConsts C) {
  __shared__ __align__(16) float sT[F16_BLOB_FLOATS];
  stage_tables(sT);
  const int64_t k = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (k >= n) return;
  const double* icb = ic_in + (int64_t)F16_IC_N * k;
  // Newton on x = (alpha, elevator cmd, throttle cmd) as the oracle's trim_one, with what the
  // fp32 residual needs to converge to its own noise floor (~1e-4 ft/s^2): central differences
  // (the forward ones of the fp64 oracle carry an O(h) bias at the step size fp32 allows), up
  // to 24 iterations, and the iterate with the smallest residual kept (fp32 noise can make the
  // last step a slightly worse one)
  float x[3] = {0.05f, 0.0f, 0.5f};
  const float hs[3] = {2e-3f, 2e-3f, 2e-3f};
  float r[3], best[3] = {x[0], x[1], x[2]}, best_r = 3.4e38f;
  for (int it = 0;; ++it) {
    trim_residual(icb, x, sT, C, r);
    const float rmax = fmaxf(fabsf(r[0]), fmaxf(fabsf(r[1]), fabsf(r[2])));
    if (rmax < best_r) { best_r = rmax; best[0] = x[0]; best[1] = x[1]; best[2] = x[2]; }
    if (rmax < 2e-5f || it == 24) break;
    float Jm[9], Ji[9];
    for (int j = 0; j < 3; ++j) {
      float xp[3] = {x[0], x[1], x[2]}, xm[3] = {x[0], x[1], x[2]}, rp[3], rm[3];
      xp[j] += hs[j];
      xm[j] -= hs[j];
      trim_residual(icb, xp, sT, C, rp);
      trim_residual(icb, xm, sT, C, rm);
      for (int i = 0; i < 3; ++i) Jm[3 * i + j] = (rp[i] - rm[i]) / (2.0f * hs[j]);
    }
    bool ok;
    inv3f(Jm, Ji, ok);
    if (!ok) break;
    float dx[3];
    mvec(Ji, r, dx);
    for (int i = 0; i < 3; ++i) x[i] -= dx[i];
    x[0] = clipf(x[0], -0.3f, 0.6f);
    x[1] = clipf(x[1], -1.0f, 0.44f);
    x[2] = clipf(x[2], 0.0f, 1.0f);
  }
  x[0] = best[0]; x[1] = best[1]; x[2] = best[2];
  trim_residual(icb, x, sT, C, r);
  double* o = ic_out + (int64_t)F16_IC_N * k;
  for (int j = 0; j < F16_IC_N; ++j) o[j] = icb[j];
  const double vt = icb[F16_IC_U_FPS];
  o[F16_IC_U_FPS] = vt * cos((double)x[0]);
  o[F16_IC_V_FPS] = 0.0;
  o[F16_IC_W_FPS] = vt * sin((double)x[0]);
  o[F16_IC_THETA_RAD] = x[0];
  o[F16_IC_PHI_RAD] = 0.0;
  o[F16_IC_P_RPS] = o[F16_IC_Q_RPS] = o[F16_IC_R_RPS] = 0.0;
  o[F16_IC_CMD_AIL] = 0.0; o[F16_IC_CMD_RUD] = 0.0;
  o[F16_IC_CMD_ELE] = x[1];
  o[F16_IC_CMD_THR] = x[2];
  if (resid)
    for (int i = 0; i < 3; ++i) resid[3 * k + i] = fabsf(r[i]);
}

__global__ void f16_sample_actions_kernel(int64_t n, int64_t id_base, uint64_t seed, uint64_t step, float* act) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  reinterpret_cast<float4*>(act)[k] = philox_action(seed, (uint64_t)(id_base + k), step);
}
// T steps' actions in one launch (f16env_sample_actions_steps, ABI 6): act[t][k] for t < T, the
// same draws as T calls of f16env_sample_actions. One 1-MB batch per launch (65 536 envs) is a
// launch-latency-bound kernel (~0.8 us over an empty launch, at 1 wave per SIMD); here each lane
// draws SA_PER_LANE float4 at a grid stride, so the whole T x N block fills the chip and streams
// out as coalesced 1-KiB wave stores.
constexpr int SA_PER_LANE = 4;
__global__ __launch_bounds__(BLOCK) void f16_sample_actions_steps_kernel(int64_t n, int64_t total, int64_t id_base,
                                                                        uint64_t seed, uint64_t step0, float* act) {
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
#pragma unroll
  for (int u = 0; u < SA_PER_LANE; ++u, i += stride) {
    if (i < total) {
      const int64_t t = i / n, k = i - t * n;
      st16<true>(reinterpret_cast<float4*>(act) + i, philox_action(seed, (uint64_t)(id_base + k), step0 + (uint64_t)t));
    }
  }
}

// GAE(lambda) over a [n_steps][n_envs] rollout, one lane per env, backward in time.
// Restates stable_baselines3/common/buffers.py:403-438 (RolloutBuffer.
// compute_returns_and_advantage) with numpy's float32 per-operation rounding: every product
// and sum is rounded separately (no FMA), gamma and gamma*lambda are rounded to float32
// exactly as numpy casts a Python float against a float32 array.
// The recurrence is serial per env (bit-exactness forbids reassociating it into a scan), and at
// cfg4's 32 768 envs one lane per env is only 512 waves, each walking 2 048 steps. Its loads do
// not depend on the chain, so they are software-pipelined: the rewards / values / starts of the
// next block of U steps are issued before the current block is computed, keeping ~2U steps of
// loads in flight per lane (round 3's loop waited on each step's three loads in turn: 0.13 of
// HBM peak). LPW lanes of each 64-lane wave carry an env (64: full waves, f16env_gae below).
// Streaming data: non-temporal loads and stores.
template <int U>
__device__ __forceinline__ void gae_load(int64_t s0, int64_t n_envs, int64_t e, const float* __restrict__ rewards,
                                         const float* __restrict__ values, const float* __restrict__ ep_starts,
                                         float (&r)[U], float (&v)[U], float (&st)[U]) {
#pragma unroll
  for (int i = 0; i < U; ++i) {
    const int64_t idx = (s0 + i) * n_envs + e;
    r[i] = __builtin_nontemporal_load(rewards + idx);
    v[i] = __builtin_nontemporal_load(values + idx);
    st[i] = __builtin_nontemporal_load(ep_starts + idx);
  }
}
template <int U, int LPW>
__global__ __launch_bounds__(64) void f16_gae_kernel(int64_t n_steps, int64_t n_envs, const float* __restrict__ rewards,
                                                     const float* __restrict__ values, const float* __restrict__ ep_starts,
                                                     const float* __restrict__ last_values, const uint8_t* __restrict__ dones,
                                                     float g, float gl, float* __restrict__ adv, float* __restrict__ ret) {
  // float32 per-op rounding as numpy (no FMA contraction; __f*_rn still contract under -O3)
#pragma clang fp contract(off)
  if ((int)threadIdx.x >= LPW) return;
  const int64_t e = (int64_t)blockIdx.x * LPW + threadIdx.x;
  if (e >= n_envs) return;
  float lgl = 0.0f;
  float nv = last_values[e];
  float nnt = 1.0f - (dones[e] ? 1.0f : 0.0f);
  // one backward step of buffers.py:425-436 at step s
  auto step = [&](int64_t s, float r, float v, float st) {
#pragma clang fp contract(off)
    const int64_t i = s * n_envs + e;
    const float t2 = (g * nv) * nnt;
    const float delta = (r + t2) - v;
    lgl = delta + (gl * nnt) * lgl;
    __builtin_nontemporal_store(lgl, adv + i);
    __builtin_nontemporal_store(lgl + v, ret + i);
    nv = v;
    nnt = 1.0f - st;
  };
  const int64_t nb = n_steps / U;  // whole blocks [b U, b U + U); the n_steps % U last steps first
  for (int64_t s = n_steps - 1; s >= nb * U; --s) {
    const int64_t i = s * n_envs + e;
    step(s, rewards[i], values[i], ep_starts[i]);
  }
  if (nb == 0) return;
  float r0[U], v0[U], s0[U];
  gae_load<U>((nb - 1) * U, n_envs, e, rewards, values, ep_starts, r0, v0, s0);
  for (int64_t b = nb - 1; b >= 0; --b) {
    float r1[U], v1[U], s1[U];
    if (b > 0) gae_load<U>((b - 1) * U, n_envs, e, rewards, values, ep_starts, r1, v1, s1);  // next block in flight
#pragma unroll
    for (int i = U - 1; i >= 0; --i) step(b * U + i, r0[i], v0[i], s0[i]);
    if (b > 0) {
#pragma unroll
      for (int i = 0; i < U; ++i) { r0[i] = r1[i]; v0[i] = v1[i]; s0[i] = s1[i]; }
    }
  }
}

// Per-frame policy features: jsbsim_gym/features.py:37-67
// JSBSimFeatureExtractor.forward, 15 observation floats -> 17 features, float32 throughout
// (torch float32 semantics: IEEE division / sqrt, ~1-ulp atan2 / cos / sin), applied to every
// frame of a (..., 15) block, e.g. the (N, K, 15) stack as the first stage of
// LMA_features.py:744-776 StackedLMAFeaturesExtractor does. HBM-bound (60 B in, 68 B out per
// frame): each 256-thread block moves its 256 frames as coalesced float4 through LDS (frame
// strides 15 and 17 are odd, so the per-thread LDS reads/writes are bank-conflict free).
__global__ __launch_bounds__(256) void f16_features_kernel(int64_t n_frames, const float* __restrict__ obs,
                                                           float* __restrict__ feat) {
  __shared__ __align__(16) float sIn[256 * FEAT_IN];
  __shared__ __align__(16) float sOut[256 * FEAT_OUT];
  const int64_t f0 = (int64_t)blockIdx.x * 256;
  const int nf = (int)(n_frames - f0 < 256 ? n_frames - f0 : 256);
  const int t = threadIdx.x;
  const float* gin = obs + f0 * FEAT_IN;
  float* gout = feat + f0 * FEAT_OUT;
  // whole-block float4 moves need 16-byte alignment of the block's slice (base % 16 == 0 and
  // a full block: 256 * 15 * 4 and 256 * 17 * 4 bytes are multiples of 16)
  const bool vin = nf == 256 && (((uintptr_t)gin) & 15) == 0;
  const bool vout = nf == 256 && (((uintptr_t)gout) & 15) == 0;
  if (vin) {
    for (int q = t; q < 256 * FEAT_IN / 4; q += 256)
      reinterpret_cast<float4*>(sIn)[q] = reinterpret_cast<const float4*>(gin)[q];
  } else {
    for (int q = t; q < nf * FEAT_IN; q += 256) sIn[q] = gin[q];
  }
  __syncthreads();
  if (t < nf) frame_features(sIn + t * FEAT_IN, sOut + t * FEAT_OUT);
  __syncthreads();
  if (vout) {
    for (int q = t; q < 256 * FEAT_OUT / 4; q += 256)
      reinterpret_cast<float4*>(gout)[q] = reinterpret_cast<const float4*>(sOut)[q];
  } else {
    for (int q = t; q < nf * FEAT_OUT; q += 256) gout[q] = sOut[q];
  }
}

// The same per-frame transform on a strided (B, K, 15) block -- e.g. a windowed observation
// (env rows 16 floats apart, frames N*16 apart: position-major 64-B slots) read in place, no
// copy to a contiguous stack.
// One lane per frame (16-B vector reads of its slot when the strides allow); the (B, K, 17)
// output leaves through LDS as coalesced float4, as in f16_features_kernel.
__global__ __launch_bounds__(256) void f16_features_strided_kernel(int64_t n_rows, int32_t K, const float* __restrict__ obs,
                                                                   int64_t row_stride, int64_t frame_stride,
                                                                   float* __restrict__ feat) {
  __shared__ __align__(16) float sOut[256 * FEAT_OUT];
  const int64_t n_frames = n_rows * K;
  const int64_t f0 = (int64_t)blockIdx.x * 256;
  const int nf = (int)(n_frames - f0 < 256 ? n_frames - f0 : 256);
  const int t = threadIdx.x;
  if (t < nf) {
    const int64_t i = f0 + t;
    const int64_t r = i / K, kk = i - r * K;
    F16_CHECK(i < n_frames && r < n_rows && kk < K, DBG_FRAME_INDEX);
    const float* o = obs + r * row_stride + kk * frame_stride;
    float x[FEAT_IN];
    if ((frame_stride & 3) == 0 && (row_stride & 3) == 0 && ((uintptr_t)obs & 15) == 0) {  // 16-B aligned frames
      const float4* q = reinterpret_cast<const float4*>(o);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const float4 v = q[j];
        x[4 * j] = v.x; x[4 * j + 1] = v.y; x[4 * j + 2] = v.z; x[4 * j + 3] = v.w;
      }
      const float2 v2 = *reinterpret_cast<const float2*>(o + 12);
      x[12] = v2.x; x[13] = v2.y; x[14] = o[14];
    } else {
#pragma unroll
      for (int j = 0; j < FEAT_IN; ++j) x[j] = o[j];
    }
    frame_features(x, sOut + t * FEAT_OUT);
  }
  __syncthreads();
  float* gout = feat + f0 * FEAT_OUT;
  if (nf == 256 && (((uintptr_t)gout) & 15) == 0) {
    for (int q = t; q < 256 * FEAT_OUT / 4; q += 256)
      reinterpret_cast<float4*>(gout)[q] = reinterpret_cast<const float4*>(sOut)[q];
  } else {
    for (int q = t; q < nf * FEAT_OUT; q += 256) gout[q] = sOut[q];
  }
}

// Feature window (windowed layout): the policy features of both frame histories kept beside
// them, position-major [T][N][17], so that after a windowed step only the frame the step wrote
// needs transforming -- the features of a K-frame observation cost one frame per step instead
// of K (f16env_features_strided over the view). The step wrote position p of both histories:
// wx[p] = the new frame, or the reset frame of a lane reset by the step (which also fills
// wx[p-K+1 .. p-1] with it), wy[p] = the new frame (the reset lane's final frame). Here
// fx[p] = fy[p] = y = feat(wx[p]), and a reset lane writes y over fx[p-K+1 .. p-1] too -- and
// over fy[p-K+2 .. p]: the window fill the NEXT step will make of that lane (FRESH: wx' = wy
// gets wx[p] at positions p-K+2 .. p, step_body) applied ahead, so no call needs the previous
// step's resets or a second transform; fy's window then holds the next step's view, not the
// terminal observation's (whose features nobody asks for). No dependent load. 64 envs per
// 256-thread block: the block's 64 frame slots come in as one float4 per thread (coalesced),
// then each of the 4 waves computes one quarter of every env's 17 features from LDS
// (frame_features_part: the work per wave a quarter, four waves per SIMD at 65 536 envs instead
// of one -- the one-lane-per-env form was latency-bound at 6.2 us, gpurun fw r04), and the
// block's rows p (64 * 17 contiguous floats in each history) leave as float4. transform = 0:
// only the ahead fills of the step's reset lanes, y read from fx[p] (after both windows were
// transformed whole following a step).
struct FeatWinArgs {
  const float* wx;
  int64_t wrow, wenv;  // frame-history strides (floats) between positions, between envs
  float* fx;
  float* fy;           // [T][N][17]
  int64_t n;
  int32_t K, p, autoreset, transform;
  const uint8_t* term;
  const uint8_t* trunc;
};
static constexpr int FW_ENVS = 64;     // envs per block
static constexpr int FW_IN = 17;       // LDS pitch of a frame (odd: conflict-free per-env reads)
__global__ __launch_bounds__(256) void f16_feature_window_kernel(FeatWinArgs a) {
  __shared__ __align__(16) float sIn[FW_ENVS * FW_IN];
  __shared__ __align__(16) float sY[FW_ENVS * FEAT_OUT];
  const int t = threadIdx.x, w = t >> 6, e = t & 63;
  const int64_t k0 = (int64_t)blockIdx.x * FW_ENVS, k = k0 + e;
  const int nb = (int)(a.n - k0 < FW_ENVS ? a.n - k0 : FW_ENVS);
  const int64_t rowN = a.n * FEAT_OUT;  // floats between feature positions
  F16_CHECK(nb > 0 && a.p >= a.K - 1, DBG_FRAME_INDEX);
  const bool done = e < nb && a.autoreset && (a.term[k] | a.trunc[k]) != 0;
  if (a.transform) {
    const int le = t >> 2, qq = t & 3;  // the block's slots: thread t loads quarter qq of env le
    if (le < nb) {
      const float4 v = *reinterpret_cast<const float4*>(a.wx + (k0 + le) * a.wenv + (int64_t)a.p * a.wrow + 4 * qq);
      float* d = sIn + le * FW_IN + 4 * qq;
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
    __syncthreads();
    if (e < nb) frame_features_part(sIn + e * FW_IN, sY + e * FEAT_OUT, w);
    __syncthreads();
  }
  // rare: the window fills of the block's reset envs (rows below p in fx, ahead in fy). Every
  // wave sees the same done mask (env e = lane); wave w takes every 4th reset env and spreads
  // its (row, feature) pairs over its 64 lanes: whole-wave stores, not one lane per env walking
  // 2K-2 rows a page apart (gpurun fw r04: +3.3 us at K = 10 for 0.13 % of lanes reset)
  const uint64_t dm = __ballot(done);
  if (dm && a.K > 1) {
    const int nrx = a.K - 1;                          // fx rows p-K+1 .. p-1
    const int nry = a.transform ? a.K - 2 : a.K - 1;  // fy rows p-K+2 .. p-1 (.. p without transform)
    const int items = (nrx + nry) * FEAT_OUT;
    int idx = 0;
    for (uint64_t m = dm; m; m &= m - 1, ++idx) {
      if ((idx & 3) != w) continue;
      const int ee = __builtin_ctzll(m);
      const int64_t kk = k0 + ee;
      for (int it = e; it < items; it += 64) {
        const int ri = it / FEAT_OUT, j = it - ri * FEAT_OUT;
        const float v = a.transform ? sY[ee * FEAT_OUT + j] : a.fx[(int64_t)a.p * rowN + kk * FEAT_OUT + j];
        float* d = ri < nrx ? a.fx + (int64_t)(a.p - a.K + 1 + ri) * rowN
                            : a.fy + (int64_t)(a.p - a.K + 2 + (ri - nrx)) * rowN;
        d[kk * FEAT_OUT + j] = v;
      }
    }
  }
  if (!a.transform) return;
  float* gx = a.fx + (int64_t)a.p * rowN + k0 * FEAT_OUT;
  float* gy = a.fy + (int64_t)a.p * rowN + k0 * FEAT_OUT;
  if (nb == FW_ENVS && ((((uintptr_t)gx) | ((uintptr_t)gy)) & 15) == 0) {
    for (int q = t; q < FW_ENVS * FEAT_OUT / 4; q += 256) {
      const float4 v = reinterpret_cast<const float4*>(sY)[q];
      reinterpret_cast<float4*>(gx)[q] = v;
      reinterpret_cast<float4*>(gy)[q] = v;
    }
  } else {
    for (int q = t; q < nb * FEAT_OUT; q += 256) {
      gx[q] = sY[q];
      gy[q] = sY[q];
    }
  }
}

// Render/telemetry poses of one frame per env (pose_of_frame above). One
// lane per env; frames are read with a caller stride so obs[:, -1, :] of a (N, K, 15) stack needs
// no copy.
// 256 envs per block; 16-B aligned frames (the windowed layout's 64-B slots) are read as
// 3 x float4 + float2 + float, and the block's 256 x 10 poses leave through LDS as contiguous
// float4 (a 40-B row per lane would be 10 partial-line dword stores)
__global__ __launch_bounds__(256) void f16_poses_kernel(int64_t n, const float* __restrict__ frames, int64_t stride,
                                                        float* __restrict__ out) {
#pragma clang fp contract(off)
  __shared__ __align__(16) float sOut[256 * 10];
  const int t = threadIdx.x;
  const int64_t k0 = (int64_t)blockIdx.x * 256, k = k0 + t;
  const int nb = (int)(n - k0 < 256 ? n - k0 : 256);
  if (t < nb) {
    const float* f = frames + k * stride;
    float x[F16_OBS_DIM];
    if ((stride & 3) == 0 && ((uintptr_t)frames & 15) == 0) {
      const float4* q4 = reinterpret_cast<const float4*>(f);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const float4 v = q4[j];
        x[4 * j] = v.x; x[4 * j + 1] = v.y; x[4 * j + 2] = v.z; x[4 * j + 3] = v.w;
      }
      const float2 v2 = *reinterpret_cast<const float2*>(f + 12);
      x[12] = v2.x; x[13] = v2.y; x[14] = f[14];
    } else {
#pragma unroll
      for (int j = 0; j < F16_OBS_DIM; ++j) x[j] = f[j];
    }
    pose_of_frame(x, sOut + t * 10);
  }
  __syncthreads();
  float* g = out + k0 * 10;
  if (nb == 256 && ((uintptr_t)g & 15) == 0) {
    for (int q = t; q < 256 * 10 / 4; q += 256)
      reinterpret_cast<float4*>(g)[q] = reinterpret_cast<const float4*>(sOut)[q];
  } else {
    for (int q = t; q < nb * 10; q += 256) g[q] = sOut[q];
  }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
struct f16env {
  f16env_config cfg;
  int device;
  void* mem;       // state SoA
  void* tmem;      // template SoA (n = 1)
  double* ic_dev;  // default IC, RANDOM_IC box lo, hi (3 x F16_IC_N)
  int32_t* done_buf;  // deferred modes: own done list (N) + two counts, when the caller gives none
  int done_par;       // which of the two counts the next step uses
  unsigned long long* nonfinite;  // F16_FLAG_NAN_GUARD quarantine counter (device, 8 B) + a
                                  // scratch word (set_state's wind detection)
  int mode;           // step kernel variant: bit 0 RANDOM_IC, bit 1 wind (GUSTS, or lanes with
                      // steady wind: config / random-IC box / set_state)
  int occ;            // waves per SIMD the step kernel is compiled for (1 or 2)
  int win_occ;        // the same for the windowed-observation step kernel
  int win_env_major;  // window histories [N][T][16] (1) instead of the default [T][N][16] (0)
  int win_nt;         // windowed step: non-temporal output stores
  int win_half;       // experiment (F16ENV_HALF=1): 32 envs per wave, f16_step_win_half_kernel
  int half_delay;     // ... and the second half of its grid starting this many cycles late
  float* fw[2];       // f16env_window_feature_bind: the feature histories (parity 0, 1)
  float* poses;       // f16env_window_poses_bind: N x 10 pose export of F16_STEP_POSES steps
  struct {            // f16env_window_bind: the buffers of f16env_window_step_bound
    float* hist[2];
    int64_t T;
    float* rew;
    uint8_t *term, *trunc;
    double* ep_ret;
    int32_t* ep_len;
  } wb;
  SoA soa, tmpl;
  // cfg5 modes: reset cache (f16_ic_fill_kernel), allocated at create (or at the first use by a
  // handle that gained wind later); refilled every icc_period windowed steps, and at the next
  // one after anything that changes the lanes' episode counters (icc_steps = 0)
  SoA icc;
  int64_t icc_steps;
  int icc_period;
  ModelConsts C;
  size_t bytes;
  int lds_image;   // step kernel stack-rebuild mode (LDS image when it fits)
  int gt;          // 1: the global-table step kernel (the image needs all of LDS, large K)
  size_t dyn_lds;  // dynamic LDS bytes per step-kernel block
  // kernel timing (f16env_profile_begin/end): start/stop events recorded by the step
  // kernel's own dispatch (hipExtLaunchKernel), one pair per launch
  std::vector<hipEvent_t> prof_ev;
  int prof_next = 0;
};

static void soa_carve(void* base, int64_t n, SoA& s) {
  s.n = n;
  s.c = (float4*)base;
}
static size_t soa_bytes(int64_t n) { return (size_t)n * NCOL_ALL * 16; }

// Same constants derivation as oracle init_consts() (f16.xml:37-83,245-300); the mass
// properties are compile-time constants (f16_device.h f16_mass_props, shared with the kernels).
static void build_consts(const f16env_config& cfg, ModelConsts& C) {
  C.inv_gref = (float)((WGS_A * WGS_A) / GM_E);
  // US-76 sea level in JSBSim units
  const double R = 8.31432 / 0.0289644;
  C.rho_sl = (float)(101325.0 / (R * 288.15) / 515.3788183931961);
  C.a_sl = (float)(sqrt(1.4 * R * 288.15) / 0.3048);
  C.p_sl = (float)(101325.0 / 47.88025898033584);
  C.inv_rho_sl = (float)(1.0 / (101325.0 / (R * 288.15) / 515.3788183931961));
  C.inv_p_sl = (float)(47.88025898033584 / 101325.0);
  C.kts_per_fps = (float)(1.0 / (1852.0 / (3600.0 * 0.3048)));
  // impact pressure at the FCS's calibrated-airspeed thresholds (f16.xml: TEF switch, PID
  // triggers), subsonic pitot (all four are far below calibrated Mach 1)
  const double a_sl = sqrt(1.4 * R * 288.15) / 0.3048, p_sl = 101325.0 / 47.88025898033584;
  auto qc_at = [&](double kts) {
    const double m = kts * (1852.0 / (3600.0 * 0.3048)) / a_sl;
    return (float)(p_sl * (pow(1.0 + 0.2 * m * m, 3.5) - 1.0));
  };
  C.qc_vc250 = qc_at(250.0); C.qc_vc20 = qc_at(20.0); C.qc_vc10 = qc_at(10.0); C.qc_vc5 = qc_at(5.0);
  C.dt = cfg.dt;
  C.cos_dE = cos(OMEGA_E * cfg.dt);
  C.sin_dE = sin(OMEGA_E * cfg.dt);
  C.epa_dt = OMEGA_E * cfg.dt;
  // fp32 products the frames formerly formed per frame (f16_device.h kin2 / pidf / frame): the
  // same single fp32 roundings, here in host IEEE arithmetic
  const float dt = (float)cfg.dt;
  C.dt_f = dt;
  C.half_dt = 0.5f * dt;
  C.dt_12 = dt * (1.0f / 12.0f);
  C.lim_ail = dt * (2.0f / 0.3f);
  C.lim_rud = dt * (2.0f / 0.4f);
  C.lim_lef = dt * (2.0f / 3.0f);
  C.lim_sb = dt * 60.0f;
  C.kidt_roll = 0.0005f * dt;
  C.kidt_pitch = 0.025f * dt;
  C.kidt_yaw = 0.00001f * dt;
}

static EnvArgs env_args(const f16env* h) {
  EnvArgs E;
  E.n = h->cfg.n_envs;
  E.K = h->cfg.stack_k;
  E.down_sample = h->cfg.down_sample;
  E.max_steps = h->cfg.max_steps;
  E.flags = h->cfg.flags;
  E.dg = (float)h->cfg.dg_m;
  E.crash = (float)h->cfg.crash_alt_m;
  E.gain = h->cfg.goal_gain;
  E.seed = h->cfg.seed;
  E.id_base = h->cfg.env_id_base;
  E.ic_cfg = h->ic_dev;
  E.ic_lo = h->ic_dev + F16_IC_N;
  E.ic_hi = h->ic_dev + 2 * F16_IC_N;
  // a = exp(-T/tau), b = sigma sqrt(1 - a^2) over the env step T = down_sample dt (oracle gust_coeffs)
  const double ga = h->cfg.gust_tau_s > 0.0 ? exp(-(double)h->cfg.down_sample * h->cfg.dt / h->cfg.gust_tau_s) : 0.0;
  E.gust_a = (float)ga;
  E.gust_b = (float)(h->cfg.gust_sigma_fps * sqrt(1.0 - ga * ga));
  E.gust_sigma = (float)h->cfg.gust_sigma_fps;
  if (!(h->cfg.flags & F16_FLAG_GUSTS)) {  // wind kernels without gusts: the gust term holds still
    E.gust_a = 1.0f; E.gust_b = 0.0f; E.gust_sigma = 0.0f;
  }
  return E;
}

extern "C" {

int f16env_config_default(f16env_config* c) {
  if (!c) return set_err(-1, "null config");
  memset(c, 0, sizeof *c);
  c->n_envs = 1;
  c->stack_k = 10;
  c->down_sample = 4;
  c->max_steps = 1200;
  c->dt = 1.0 / 120.0;
  c->dg_m = 100.0;
  c->goal_gain = 1e-2;
  c->crash_alt_m = 10.0;
  c->ic[F16_IC_H_SL_FT] = 5000.0;
  c->ic[F16_IC_U_FPS] = 900.0;
  for (int j = 0; j < F16_IC_N; ++j) c->ic_lo[j] = c->ic_hi[j] = c->ic[j];
  c->gust_sigma_fps = 0.0;
  c->gust_tau_s = 2.0;
  return 0;
}

int f16env_config_cfg5(f16env_config* c) {
  if (!c) return set_err(-1, "null config");
  c->flags |= F16_FLAG_RANDOM_IC | F16_FLAG_GUSTS;
  for (int j = 0; j < F16_IC_N; ++j) c->ic_lo[j] = c->ic_hi[j] = c->ic[j];
  const double deg10 = 0.17453292519943295;
  c->ic_lo[F16_IC_H_SL_FT] = 3000.0;  c->ic_hi[F16_IC_H_SL_FT] = 30000.0;
  c->ic_lo[F16_IC_U_FPS] = 600.0;     c->ic_hi[F16_IC_U_FPS] = 1200.0;
  c->ic_lo[F16_IC_PHI_RAD] = -deg10;  c->ic_hi[F16_IC_PHI_RAD] = deg10;
  c->ic_lo[F16_IC_THETA_RAD] = -deg10; c->ic_hi[F16_IC_THETA_RAD] = deg10;
  c->ic_lo[F16_IC_PSI_RAD] = 0.0;     c->ic_hi[F16_IC_PSI_RAD] = 6.283185307179586;
  c->ic_lo[F16_IC_CMD_THR] = 0.3;     c->ic_hi[F16_IC_CMD_THR] = 1.0;
  c->ic_lo[F16_IC_WIND_N_FPS] = -30.0; c->ic_hi[F16_IC_WIND_N_FPS] = 30.0;
  c->ic_lo[F16_IC_WIND_E_FPS] = -30.0; c->ic_hi[F16_IC_WIND_E_FPS] = 30.0;
  c->gust_sigma_fps = 10.0;
  c->gust_tau_s = 2.0;
  return 0;
}

int f16env_create(const f16env_config* cfg, int device, f16env_t* out) {
  if (!cfg || !out) return set_err(-1, "null argument");
  if (cfg->n_envs <= 0) return set_err(-1, "n_envs must be > 0");
  if (cfg->stack_k < 1 || cfg->stack_k > 64) return set_err(-1, "stack_k must be in [1, 64]");
  if (cfg->down_sample < 0) return set_err(-1, "down_sample must be >= 0");
  if (!(cfg->dt > 0.0)) return set_err(-1, "dt must be > 0");
  if ((cfg->flags & F16_FLAG_GUSTS) && !(cfg->gust_sigma_fps >= 0.0 && cfg->gust_tau_s > 0.0))
    return set_err(-1, "gusts need gust_sigma_fps >= 0 and gust_tau_s > 0");
  HIPCHK(hipSetDevice(device));
  f16env* h = new f16env();
  h->cfg = *cfg;
  h->device = device;
  build_consts(*cfg, h->C);
  h->bytes = soa_bytes(cfg->n_envs);
  hipError_t e = hipMalloc(&h->mem, h->bytes);
  if (e != hipSuccess) { delete h; return set_err(-3, "hipMalloc(state) failed"); }
  hipMemset(h->mem, 0, h->bytes);
  soa_carve(h->mem, cfg->n_envs, h->soa);
  bool wind = false;  // can any lane carry wind? (then the wind kernels: MODE bit 1)
  for (int j = F16_IC_WIND_N_FPS; j <= F16_IC_WIND_D_FPS; ++j)
    wind = wind || cfg->ic[j] != 0.0 ||
           ((cfg->flags & F16_FLAG_RANDOM_IC) && (cfg->ic_lo[j] != 0.0 || cfg->ic_hi[j] != 0.0));
  h->mode = ((cfg->flags & F16_FLAG_RANDOM_IC) ? 1 : 0) | (((cfg->flags & F16_FLAG_GUSTS) || wind) ? 2 : 0);
  h->done_buf = nullptr;
  h->icc.c = nullptr; h->icc.n = cfg->n_envs;
  h->icc_steps = 0;
  h->icc_period = 64;  // same-box sweep, 2 048 cfg5 steps: 27.5 / 27.0 / 27.0 / 26.8 / 27.7 us at 32..512
  if (getenv("F16ENV_ICC_PERIOD")) h->icc_period = atoi(getenv("F16ENV_ICC_PERIOD"));
  if (hipMalloc(&h->tmem, (size_t)TMPL_COLS * 16) != hipSuccess ||
      hipMalloc((void**)&h->ic_dev, sizeof(double) * 3 * F16_IC_N) != hipSuccess ||
      hipMalloc((void**)&h->done_buf, sizeof(int32_t) * ((size_t)cfg->n_envs + 2)) != hipSuccess) {
    hipFree(h->mem); hipFree(h->tmem); hipFree(h->ic_dev); delete h;
    return set_err(-3, "hipMalloc(template) failed");
  }
  soa_carve(h->tmem, 1, h->tmpl);
  hipMemset(h->done_buf + cfg->n_envs, 0, 2 * sizeof(int32_t));
  h->done_par = 0;
  if (hipMalloc((void**)&h->nonfinite, 4 * sizeof(unsigned long long)) != hipSuccess) {
    hipFree(h->mem); hipFree(h->tmem); hipFree(h->ic_dev); hipFree(h->done_buf); delete h;
    return set_err(-3, "hipMalloc(counter) failed");
  }
  hipMemset(h->nonfinite, 0, 4 * sizeof(unsigned long long));
  {
    const int KC = cfg->stack_k * F16_OBS_DIM;
    const size_t img = sizeof(float) * (BLOCK / 64) * ((size_t)64 * KC + 16);
    const size_t fallback = sizeof(float) * 2 * BLOCK * FRAME_PITCH;
    const size_t static_gt = 16 * (NCOL + TMPL_FRAME_COLS) + sizeof(int) * BLOCK + 64;
    const size_t static_lds = sizeof(float) * F16_BLOB_FLOATS + static_gt;
    // the stack image with LDS tables if both fit, else with global tables, else the
    // chunked flat copy (LDS tables)
    h->lds_image = (img + static_lds <= 160 * 1024) ? 1 : (img + static_gt <= 160 * 1024 ? 1 : 0);
    h->gt = (h->lds_image && img + static_lds > 160 * 1024) ? 1 : 0;
    if (getenv("F16ENV_GT") && h->lds_image) h->gt = atoi(getenv("F16ENV_GT")) ? 1 : 0;
    h->dyn_lds = h->lds_image ? img : fallback;
    // two waves per SIMD only pay when there are more waves than SIMDs and two workgroups'
    // LDS (tables + stack image) fit in one CU
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
      cus = 256;
    const int64_t waves = ((int64_t)cfg->n_envs + 63) / 64;
    h->occ = (!h->gt && waves > 4 * (int64_t)cus && 2 * (static_lds + h->dyn_lds) <= 160 * 1024) ? 2 : 1;
    if (getenv("F16ENV_OCC")) h->occ = atoi(getenv("F16ENV_OCC")) == 2 ? 2 : 1;
    h->win_occ = (waves > 4 * (int64_t)cus && 2 * (static_lds + WIN_DYN_LDS) <= 160 * 1024) ? 2 : 1;
    if (getenv("F16ENV_OCC")) h->win_occ = atoi(getenv("F16ENV_OCC")) == 2 ? 2 : 1;
    // non-temporal output stores pay in the windowed step when its whole grid is resident at
    // once (one round of waves); with more rounds they cost (st16)
    h->win_nt = waves <= (int64_t)h->win_occ * 4 * cus ? 1 : 0;
    if (getenv("F16ENV_WIN_NT")) h->win_nt = atoi(getenv("F16ENV_WIN_NT")) ? 1 : 0;
    h->win_half = getenv("F16ENV_HALF") ? (atoi(getenv("F16ENV_HALF")) ? 1 : 0) : 0;
    h->half_delay = getenv("F16ENV_HALF_DELAY") ? atoi(getenv("F16ENV_HALF_DELAY")) : 0;
    for (int v = 0; v <= 2; ++v) {
      const size_t st_v = v == 2 ? static_gt : static_lds;
      for (int m = 0; m < 8; ++m) {
        const size_t dyn = h->dyn_lds;
        if (st_v + dyn > 160 * 1024) continue;  // not launchable in this configuration
        if (hipFuncSetAttribute((const void*)step_kernel_for(m & 3, v, m >= 4), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)dyn) != hipSuccess) {
          (void)hipGetLastError();
          hipFree(h->mem); hipFree(h->tmem); hipFree(h->ic_dev); hipFree(h->done_buf); hipFree(h->nonfinite);
          delete h;
          return set_err(-2, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
        }
      }
    }
  }
  // cfg5 modes: the reset cache up front (its bytes are part of f16env_state_bytes); a handle
  // that only gains wind later (set_state / a per-lane IC) allocates it at its first use
  if (h->mode && !(cfg->flags & F16_FLAG_NO_AUTORESET)) {
    const size_t b = (size_t)ICC_COLS * 16 * (size_t)cfg->n_envs;
    if (hipMalloc((void**)&h->icc.c, b) != hipSuccess) {
      h->icc.c = nullptr;
      hipFree(h->mem); hipFree(h->tmem); hipFree(h->ic_dev); hipFree(h->done_buf); hipFree(h->nonfinite); delete h;
      return set_err(-3, "hipMalloc(reset cache) failed");
    }
    hipMemset(h->icc.c, 0, b);  // tag 0: no row valid yet
    h->bytes += b;
  }
  hipMemcpy(h->ic_dev, cfg->ic, sizeof(double) * F16_IC_N, hipMemcpyHostToDevice);
  hipMemcpy(h->ic_dev + F16_IC_N, cfg->ic_lo, sizeof(double) * F16_IC_N, hipMemcpyHostToDevice);
  hipMemcpy(h->ic_dev + 2 * F16_IC_N, cfg->ic_hi, sizeof(double) * F16_IC_N, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(f16_ic_kernel, dim3(1), dim3(BLOCK), 0, 0, h->tmpl, (const double*)h->ic_dev, h->C);
  e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) {
    hipFree(h->mem); hipFree(h->tmem); hipFree(h->ic_dev); hipFree(h->done_buf); hipFree(h->nonfinite);
    if (h->icc.c) hipFree(h->icc.c);
    delete h;
    return set_err(-2, hipGetErrorString(e));
  }
  *out = h;
  return 0;
}

static void prof_free(f16env* h) {
  for (hipEvent_t e : h->prof_ev) hipEventDestroy(e);
  h->prof_ev.clear();
  h->prof_next = 0;
}

int f16env_profile_begin(f16env_t h, int max_launches) {
  if (!h || max_launches <= 0 || max_launches > 100000) return set_err(-1, "max_launches must be in [1, 100000]");
  prof_free(h);
  h->prof_ev.resize((size_t)2 * max_launches);
  for (auto& e : h->prof_ev) HIPCHK(hipEventCreate(&e));
  return 0;
}

int f16env_profile_end(f16env_t h, double* avg_ms, double* min_ms, int* launches) {
  if (!h) return set_err(-1, "null handle");
  const int n = h->prof_next;
  double sum = 0.0, mn = 0.0;
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipEventSynchronize(h->prof_ev[2 * i + 1]));
    float ms = 0.0f;
    HIPCHK(hipEventElapsedTime(&ms, h->prof_ev[2 * i], h->prof_ev[2 * i + 1]));
    sum += ms;
    mn = (i == 0 || ms < mn) ? ms : mn;
  }
  if (avg_ms) *avg_ms = n ? sum / n : 0.0;
  if (min_ms) *min_ms = mn;
  if (launches) *launches = n;
  prof_free(h);
  return 0;
}

int f16env_profile_times(f16env_t h, double* t_ms, int max_launches) {
  if (!h || !t_ms) return set_err(-1, "null argument");
  const int n = h->prof_next < max_launches ? h->prof_next : max_launches;
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipEventSynchronize(h->prof_ev[2 * i + 1]));
    float a = 0.0f, b = 0.0f;
    HIPCHK(hipEventElapsedTime(&a, h->prof_ev[0], h->prof_ev[2 * i]));
    HIPCHK(hipEventElapsedTime(&b, h->prof_ev[0], h->prof_ev[2 * i + 1]));
    t_ms[2 * i] = a;
    t_ms[2 * i + 1] = b;
  }
  return n;
}

int f16env_destroy(f16env_t h) {
  if (!h) return 0;
  hipSetDevice(h->device);
  hipFree(h->mem);
  hipFree(h->tmem);
  hipFree(h->ic_dev);
  if (h->done_buf) hipFree(h->done_buf);
  if (h->icc.c) hipFree(h->icc.c);
  hipFree(h->nonfinite);
  prof_free(h);
  delete h;
  return 0;
}

size_t f16env_state_bytes(f16env_t h) { return h ? h->bytes : 0; }
int f16env_state_bytes_per_env(void) { return STATE_BYTES; }

static inline unsigned nblocks(int64_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }

// reset launch shared by f16env_reset / f16env_reset_window. A per-lane IC may carry wind:
// then the handle reads back (waits for the stream) whether any lane got some, and switches to
// the wind kernels if so (the caller's IC is not hot-path).
static int reset_launch(f16env_t h, hipStream_t st, ResetArgs& a) {
  h->icc_steps = 0;  // the lanes' episode counters move: the next windowed step refills the reset cache
  a.wind_any = nullptr;
  if (a.ic && !(h->mode & 2)) {
    a.wind_any = reinterpret_cast<int*>(h->nonfinite + 1);
    HIPCHK(hipMemsetAsync(a.wind_any, 0, sizeof(int), st));
  }
  hipLaunchKernelGGL(f16_reset_kernel, dim3(nblocks(a.E.n)), dim3(BLOCK), 0, st, a);
  HIPCHK(hipGetLastError());
  if (a.wind_any) {
    int w = 0;
    HIPCHK(hipMemcpyAsync(&w, a.wind_any, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (w) h->mode |= 2;
  }
  return 0;
}

int f16env_reset(f16env_t h, void* stream, const uint8_t* mask, const float* goals, const double* ic, float* obs) {
  if (!h) return set_err(-1, "null handle");
  ResetArgs a;
  a.s = h->soa; a.tmpl = h->tmpl; a.mask = mask; a.goals = goals; a.ic = ic; a.obs = obs;
  a.obs_row = (int64_t)h->cfg.stack_k * F16_OBS_DIM; a.obs_off = 0; a.obs_pitch = F16_OBS_DIM;
  a.obs_slot = F16_OBS_DIM;
  a.E = env_args(h);
  a.C = h->C;
  return reset_launch(h, (hipStream_t)stream, a);
}

// The done list of a step: the caller's (its count zeroed here), else, in deferred modes, the
// handle's own with two alternating counts -- the step's deferred-reset kernel zeroes the one
// the next step uses, so an auto-resetting step issues no memset (one GPU operation fewer).
static int done_counter(f16env_t h, int32_t* done_idx, int32_t*& list, int32_t*& count, int32_t*& zero_next,
                        hipStream_t st) {
  zero_next = nullptr;
  if (h->mode && !done_idx) {  // deferred resets need the done list
    list = h->done_buf;
    count = h->done_buf + h->cfg.n_envs + h->done_par;
    if (!(h->cfg.flags & F16_FLAG_NO_AUTORESET)) {  // the reset kernel follows: it zeroes the other
      zero_next = h->done_buf + h->cfg.n_envs + (h->done_par ^ 1);
      h->done_par ^= 1;
      return 0;
    }
  }
  if (count) HIPCHK(hipMemsetAsync(count, 0, sizeof(int32_t), st));
  return 0;
}

static int step_impl(f16env_t h, void* stream, const f16env_rollout_slot* slot, const float* act,
                     const float* obs_prev, float* obs, float* rew, uint8_t* terminated, uint8_t* truncated,
                     float* terminal_obs, double* ep_return, int32_t* ep_len, int32_t* done_idx, int32_t* n_done) {
  if (!h) return set_err(-1, "null handle");
  if ((!act && !slot) || !obs_prev || !obs || !rew || !terminated || !truncated)
    return set_err(-1, "act (or a rollout slot)/obs_prev/obs/rew/terminated/truncated are required");
  if (done_idx && !n_done) return set_err(-1, "done_idx requires n_done");
  if (act && ((uintptr_t)act & 15) != 0) return set_err(-1, "act must be 16-byte aligned");
  StepArgs a;
  a.s = h->soa; a.tmpl = h->tmpl; a.act = act; a.obs_prev = obs_prev; a.obs = obs; a.rew = rew;
  a.term = terminated; a.trunc = truncated; a.tobs = terminal_obs; a.ep_ret = ep_return; a.ep_len = ep_len;
  a.done_idx = done_idx; a.n_done = n_done;
  a.nonfinite = h->nonfinite;
  a.sample_act = act ? 0 : 1;
  a.clip_act = (slot && (slot->flags & F16_SLOT_CLIP)) ? 1 : 0;
  a.act_seed = slot ? slot->act_seed : 0; a.act_step = slot ? slot->act_step : 0;
  a.r_frame = slot ? slot->frame : nullptr;
  a.r_next_frame = nullptr;
  a.r_act = slot ? slot->actions : nullptr;
  a.r_rew = slot ? slot->rewards : nullptr;
  a.r_next_start = slot ? slot->next_start : nullptr;
  float* feat = slot ? slot->features : nullptr;
  if (slot && slot->next_frame)
    return set_err(-1, "rollout slot next_frame is the windowed layout's (f16env_window_step_rollout); "
                       "the contiguous layout writes frame");
  if ((a.r_frame && ((uintptr_t)a.r_frame & 15) != 0) || (a.r_act && ((uintptr_t)a.r_act & 15) != 0))
    return set_err(-1, "rollout slot frame/actions must be 16-byte aligned");
  a.wx = a.wy = nullptr; a.wrow = a.wenv = 0; a.wpos = 0;
  a.icc.c = nullptr; a.icc.n = 0;
  a.E = env_args(h);
  a.C = h->C;
  a.lds_image = h->lds_image;
  if (((uintptr_t)obs & 15) != 0 || ((uintptr_t)obs_prev & 15) != 0)
    return set_err(-1, "obs and obs_prev must be 16-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  int32_t* zero_next = nullptr;
  if (int e = done_counter(h, done_idx, a.done_idx, a.n_done, zero_next, st)) return e;
  const dim3 grid(nblocks(a.E.n)), blk(BLOCK);
  const StepKernel kern = step_kernel_for(h->mode, h->gt ? 2 : (h->occ == 2 ? 1 : 0), slot != nullptr);
  if (h->prof_next < (int)h->prof_ev.size() / 2) {  // profiling: events from the dispatch packet itself
    const int i = h->prof_next++;
    hipExtLaunchKernelGGL(kern, grid, blk, (std::uint32_t)h->dyn_lds, st, h->prof_ev[2 * i], h->prof_ev[2 * i + 1], 0u,
                          (const float4*)a.s.c, a.act, (const float4*)a.tmpl.c, a.E.n, a);
  } else {
    hipLaunchKernelGGL(kern, grid, blk, h->dyn_lds, st, (const float4*)a.s.c, a.act, (const float4*)a.tmpl.c, a.E.n, a);
  }
  HIPCHK(hipGetLastError());
  if (h->mode && !(h->cfg.flags & F16_FLAG_NO_AUTORESET)) {
    ResetDoneArgs r;
    r.s = h->soa; r.tmpl = h->tmpl; r.done_idx = a.done_idx; r.n_done = a.n_done; r.obs = obs;
    r.obs_row = (int64_t)a.E.K * F16_OBS_DIM; r.obs_off = 0; r.obs_pitch = F16_OBS_DIM; r.obs_slot = F16_OBS_DIM;
    r.zero_next = zero_next;
    r.E = a.E; r.C = h->C;
    const unsigned g = nblocks(a.E.n) < 64u ? nblocks(a.E.n) : 64u;
    hipLaunchKernelGGL(f16_reset_done_kernel, dim3(g), blk, 0, st, r);
    HIPCHK(hipGetLastError());
  }
  if (feat) {  // policy features of the returned obs (after any deferred reset rewrote rows)
    const int64_t nf = (int64_t)a.E.n * a.E.K;
    hipLaunchKernelGGL(f16_features_kernel, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, st, nf,
                       (const float*)obs, feat);
    HIPCHK(hipGetLastError());
  }
  return 0;
}

int f16env_step(f16env_t h, void* stream, const float* act, const float* obs_prev, float* obs, float* rew,
                uint8_t* terminated, uint8_t* truncated, float* terminal_obs, double* ep_return, int32_t* ep_len,
                int32_t* done_idx, int32_t* n_done) {
  return step_impl(h, stream, nullptr, act, obs_prev, obs, rew, terminated, truncated, terminal_obs, ep_return,
                   ep_len, done_idx, n_done);
}

// (floats between positions, floats between envs) of the handle's window history order
static void window_strides(f16env_t h, int64_t T, int64_t& wpos, int64_t& wenv) {
  if (h->win_env_major) { wpos = WPITCH; wenv = T * WPITCH; }
  else { wpos = (int64_t)h->cfg.n_envs * WPITCH; wenv = WPITCH; }
}

int f16env_set_window_order(f16env_t h, int env_major) {
  if (!h) return set_err(-1, "null handle");
  h->win_env_major = env_major ? 1 : 0;
  return 0;
}

// cfg5 modes: the reset cache, allocated if this handle has none yet (it gained wind after
// create), refilled now if `fill` (f16_ic_fill_kernel: every lane whose cached row is not its
// next episode's)
static int icc_prepare(f16env_t h, hipStream_t st, bool fill) {
  const int64_t n = h->cfg.n_envs;
  if (!h->icc.c) {
    const size_t b = (size_t)ICC_COLS * 16 * (size_t)n;
    if (hipMalloc((void**)&h->icc.c, b) != hipSuccess) { h->icc.c = nullptr; return set_err(-3, "hipMalloc(reset cache) failed"); }
    HIPCHK(hipMemsetAsync(h->icc.c, 0, b, st));  // tag 0: no row valid yet
    h->bytes += b;
    fill = true;
  }
  h->icc.n = n;
  if (fill) {
    using FillKernel = void (*)(SoA, SoA, EnvArgs, ModelConsts);
    static const FillKernel fills[4] = {f16_ic_fill_kernel<0>, f16_ic_fill_kernel<1>, f16_ic_fill_kernel<2>,
                                        f16_ic_fill_kernel<3>};
    hipLaunchKernelGGL(fills[h->mode & 3], dim3(nblocks(n)), dim3(BLOCK), 0, st, h->soa, h->icc, env_args(h), h->C);
    HIPCHK(hipGetLastError());
  }
  return 0;
}

static int window_check(f16env_t h, const float* hist_cur, const float* hist_other, int64_t T, int32_t pos) {
  const int K = h->cfg.stack_k;
  if (!hist_cur || (hist_other == nullptr && hist_cur == nullptr)) return set_err(-1, "null history");
  if (((uintptr_t)hist_cur & 15) != 0 || ((uintptr_t)hist_other & 15) != 0)
    return set_err(-1, "histories must be 16-byte aligned");
  if (T < 2 * (int64_t)K) return set_err(-1, "history length T must be >= 2K");
  if (pos < K - 1 || (int64_t)pos >= T) return set_err(-1, "window position must be in [K-1, T-1]");
  return 0;
}

static int step_window_impl(f16env_t h, void* stream, const f16env_rollout_slot* slot, const float* act,
                            float* hist_cur, float* hist_other, int64_t T, int32_t pos, float* rew,
                            uint8_t* terminated, uint8_t* truncated, double* ep_return, int32_t* ep_len,
                            int32_t* done_idx, int32_t* n_done, bool ex = false, uint32_t xflags = 0,
                            uint64_t act_seed = 0, uint64_t act_step = 0) {
  if (!h) return set_err(-1, "null handle");
  if ((!act && !slot && !ex) || !hist_other || !rew || !terminated || !truncated)
    return set_err(-1, "act (or a rollout slot)/hist_cur/hist_other/rew/terminated/truncated are required");
  if (int e = window_check(h, hist_cur, hist_other, T, pos)) return e;
  if (hist_cur == hist_other) return set_err(-1, "the two histories must be distinct buffers");
  if (done_idx && !n_done) return set_err(-1, "done_idx requires n_done");
  if (act && ((uintptr_t)act & 15) != 0) return set_err(-1, "act must be 16-byte aligned");
  StepArgs a;
  memset(&a, 0, sizeof a);
  a.s = h->soa; a.tmpl = h->tmpl; a.act = act; a.rew = rew;
  a.term = terminated; a.trunc = truncated; a.ep_ret = ep_return; a.ep_len = ep_len;
  a.done_idx = done_idx; a.n_done = n_done;
  a.nonfinite = h->nonfinite;
  float* feat = nullptr;
  if (slot) {
    if (slot->frame)
      return set_err(-1, "rollout slot frame is the contiguous layout's; the windowed layout writes next_frame "
                         "(the newest frame of the returned observation)");
    a.sample_act = act ? 0 : 1;
    a.clip_act = (slot->flags & F16_SLOT_CLIP) ? 1 : 0;
    a.act_seed = slot->act_seed; a.act_step = slot->act_step;
    a.r_next_frame = slot->next_frame; a.r_act = slot->actions; a.r_rew = slot->rewards;
    a.r_next_start = slot->next_start;
    feat = slot->features;
    if ((a.r_next_frame && ((uintptr_t)a.r_next_frame & 3) != 0) || (a.r_act && ((uintptr_t)a.r_act & 15) != 0))
      return set_err(-1, "rollout slot next_frame must be 4-byte and actions 16-byte aligned");
    if (slot->flags & F16_SLOT_FEATURE_WINDOW) {
      if (!h->fw[0] || !h->fw[1]) return set_err(-1, "F16_SLOT_FEATURE_WINDOW: f16env_window_feature_bind first");
      if (hist_cur != h->wb.hist[0] && hist_cur != h->wb.hist[1])
        return set_err(-1, "F16_SLOT_FEATURE_WINDOW: the step's histories must be the bound ones");
      if (h->mode && !(h->cfg.flags & F16_FLAG_NO_AUTORESET) && h->icc_period <= 0)
        return set_err(-1, "F16_SLOT_FEATURE_WINDOW: not with the deferred-reset step (F16ENV_ICC_PERIOD=0)");
      const int b = hist_cur == h->wb.hist[0] ? 0 : 1;
      a.fwx = h->fw[b]; a.fwy = h->fw[b ^ 1];
    }
  } else if (ex) {  // f16env_window_step_ex: the winx build (in-kernel actions, feature window)
    a.sample_act = act ? 0 : 1;
    a.act_seed = act_seed; a.act_step = act_step;
    if (xflags & ~(uint32_t)(F16_STEP_FEATURE_WINDOW | F16_STEP_POSES))
      return set_err(-1, "unknown f16env_window_step_ex flags");
    if (xflags & F16_STEP_POSES) {
      if (!h->poses) return set_err(-1, "F16_STEP_POSES: f16env_window_poses_bind first");
      if (h->mode && !(h->cfg.flags & F16_FLAG_NO_AUTORESET) && h->icc_period <= 0)
        return set_err(-1, "F16_STEP_POSES: not with the deferred-reset step (F16ENV_ICC_PERIOD=0)");
      a.poses = h->poses;
    }
    if (xflags & F16_STEP_FEATURE_WINDOW) {
      if (!h->fw[0] || !h->fw[1]) return set_err(-1, "F16_STEP_FEATURE_WINDOW: f16env_window_feature_bind first");
      if (hist_cur != h->wb.hist[0] && hist_cur != h->wb.hist[1])
        return set_err(-1, "F16_STEP_FEATURE_WINDOW: the step's histories must be the bound ones");
      if (h->mode && !(h->cfg.flags & F16_FLAG_NO_AUTORESET) && h->icc_period <= 0)
        return set_err(-1, "F16_STEP_FEATURE_WINDOW: not with the deferred-reset step (F16ENV_ICC_PERIOD=0)");
      const int b = hist_cur == h->wb.hist[0] ? 0 : 1;
      a.fwx = h->fw[b]; a.fwy = h->fw[b ^ 1];
    }
  }
  // cfg5 modes: finished lanes are reset inside the step from the reset cache (period 0 or
  // F16ENV_ICC_PERIOD=0: the deferred f16_reset_done_kernel instead)
  const bool cache = h->mode && !(h->cfg.flags & F16_FLAG_NO_AUTORESET) && h->icc_period > 0;
  const bool deferred = h->mode && !(h->cfg.flags & F16_FLAG_NO_AUTORESET) && !cache;
  // the deferred reset rewrites finished lanes' windows after the step kernel, so a slot frame or
  // features written by the step would describe the pre-reset window: rejected here, before any
  // launch, so that a refused call leaves the device state untouched
  if (deferred && slot && (slot->next_frame || feat))
    return set_err(-1, "the deferred-reset windowed step (F16ENV_ICC_PERIOD=0) writes no next_frame / features");
  int64_t P, Q;  // floats between positions, between envs
  window_strides(h, T, P, Q);
  a.wx = hist_cur; a.wy = hist_other; a.wrow = P; a.wenv = Q; a.wpos = pos;
  a.E = env_args(h);
  a.C = h->C;
  a.lds_image = 0;
  hipStream_t st = (hipStream_t)stream;
  int32_t* zero_next = nullptr;
  const dim3 blk(BLOCK);
  a.icc.c = nullptr; a.icc.n = a.E.n;
  if (cache) {
    if (int e = icc_prepare(h, st, h->icc_steps % h->icc_period == 0)) return e;
    ++h->icc_steps;
    a.icc = h->icc;
    if (n_done) HIPCHK(hipMemsetAsync(n_done, 0, sizeof(int32_t), st));  // the caller's done list only
  } else if (int e = done_counter(h, done_idx, a.done_idx, a.n_done, zero_next, st)) {
    return e;
  }
  WinKernel kern = ex ? step_winx_kernel_for(h->mode, h->win_occ, h->win_nt, a.fwx != nullptr)
                      : step_win_kernel_for(h->mode, h->win_occ, h->win_nt, slot != nullptr);
  dim3 grid(nblocks(a.E.n));
  if (h->win_half && !slot && !ex) {  // the half-populated-wave experiment: 128 envs per block
    static const WinKernel half[4] = {f16_step_win_half_kernel<0>, f16_step_win_half_kernel<1>,
                                      f16_step_win_half_kernel<2>, f16_step_win_half_kernel<3>};
    kern = half[h->mode & 3];
    grid = dim3((unsigned)((a.E.n + 127) / 128));
    a.half_delay = h->half_delay;
  }
  const float4* sc = a.s.c;
  const float4* tc = a.tmpl.c;
  const int64_t n = a.E.n;
  if (h->prof_next < (int)h->prof_ev.size() / 2) {
    const int i = h->prof_next++;
    hipExtLaunchKernelGGL(kern, grid, blk, (std::uint32_t)WIN_DYN_LDS, st, h->prof_ev[2 * i], h->prof_ev[2 * i + 1], 0u,
                          sc, a.act, tc, n, a);
  } else {
    hipLaunchKernelGGL(kern, grid, blk, WIN_DYN_LDS, st, sc, a.act, tc, n, a);
  }
  HIPCHK(hipGetLastError());
  if (deferred) {
    ResetDoneArgs r;
    r.s = h->soa; r.tmpl = h->tmpl; r.done_idx = a.done_idx; r.n_done = a.n_done; r.obs = hist_cur;
    r.obs_row = Q; r.obs_off = (int64_t)(pos - a.E.K + 1) * P; r.obs_pitch = P; r.obs_slot = WPITCH;
    r.zero_next = zero_next;
    r.E = a.E; r.C = h->C;
    const unsigned g = nblocks(a.E.n) < 64u ? nblocks(a.E.n) : 64u;
    hipLaunchKernelGGL(f16_reset_done_kernel, dim3(g), blk, 0, st, r);
    HIPCHK(hipGetLastError());
  }
  if (feat) {  // policy features of the returned observation, read in place from the window
    const int64_t blocks = ((int64_t)a.E.n * a.E.K + 255) / 256;
    hipLaunchKernelGGL(f16_features_strided_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (int64_t)a.E.n,
                       (int32_t)a.E.K, (const float*)(hist_cur + (int64_t)(pos - a.E.K + 1) * P), Q, P, feat);
    HIPCHK(hipGetLastError());
  }
  return 0;
}

int f16env_step_window(f16env_t h, void* stream, const float* act, float* hist_cur, float* hist_other, int64_t T,
                       int32_t pos, float* rew, uint8_t* terminated, uint8_t* truncated, double* ep_return,
                       int32_t* ep_len, int32_t* done_idx, int32_t* n_done) {
  if (!act) return set_err(-1, "act is required");
  return step_window_impl(h, stream, nullptr, act, hist_cur, hist_other, T, pos, rew, terminated, truncated,
                          ep_return, ep_len, done_idx, n_done);
}

int f16env_window_bind(f16env_t h, float* hist0, float* hist1, int64_t T, float* rew, uint8_t* terminated,
                       uint8_t* truncated, double* ep_return, int32_t* ep_len) {
  if (!h) return set_err(-1, "null handle");
  if (!hist0 || !hist1 || hist0 == hist1 || !rew || !terminated || !truncated)
    return set_err(-1, "two distinct histories and rew/terminated/truncated are required");
  if (int e = window_check(h, hist0, hist1, T, h->cfg.stack_k - 1)) return e;
  h->wb.hist[0] = hist0; h->wb.hist[1] = hist1; h->wb.T = T;
  h->wb.rew = rew; h->wb.term = terminated; h->wb.trunc = truncated;
  h->wb.ep_ret = ep_return; h->wb.ep_len = ep_len;
  return 0;
}

int f16env_window_feature_bind(f16env_t h, float* feat0, float* feat1) {
  if (!h) return set_err(-1, "null handle");
  if ((!feat0) != (!feat1) || (feat0 && feat0 == feat1)) return set_err(-1, "two distinct feature histories (or none)");
  if (((((uintptr_t)feat0) | ((uintptr_t)feat1)) & 3) != 0) return set_err(-1, "feature histories must be float-aligned");
  h->fw[0] = feat0; h->fw[1] = feat1;
  return 0;
}

int f16env_window_poses_bind(f16env_t h, float* poses) {
  if (!h) return set_err(-1, "null handle");
  if (((uintptr_t)poses & 3) != 0) return set_err(-1, "poses must be float-aligned");
  h->poses = poses;
  return 0;
}

int f16env_window_step_bound(f16env_t h, void* stream, const float* act, int32_t parity, int32_t pos) {
  if (!h) return set_err(-1, "null handle");
  if (!h->wb.hist[0]) return set_err(-1, "f16env_window_bind first");
  const int b = parity & 1;
  return f16env_step_window(h, stream, act, h->wb.hist[b], h->wb.hist[b ^ 1], h->wb.T, pos, h->wb.rew, h->wb.term,
                            h->wb.trunc, h->wb.ep_ret, h->wb.ep_len, nullptr, nullptr);
}

int f16env_window_step_ex(f16env_t h, void* stream, const float* act, int32_t parity, int32_t pos, uint32_t flags,
                          uint64_t act_seed, uint64_t act_step) {
  if (!h) return set_err(-1, "null handle");
  if (!h->wb.hist[0]) return set_err(-1, "f16env_window_bind first");
  const int b = parity & 1;
  if (act && !flags)  // nothing extra: the plain windowed step (the headline instance)
    return f16env_step_window(h, stream, act, h->wb.hist[b], h->wb.hist[b ^ 1], h->wb.T, pos, h->wb.rew, h->wb.term,
                              h->wb.trunc, h->wb.ep_ret, h->wb.ep_len, nullptr, nullptr);
  // (rew/terminated/truncated are required by the impl; act may be NULL here)
  return step_window_impl(h, stream, nullptr, act, h->wb.hist[b], h->wb.hist[b ^ 1], h->wb.T, pos, h->wb.rew,
                          h->wb.term, h->wb.trunc, h->wb.ep_ret, h->wb.ep_len, nullptr, nullptr, true, flags, act_seed,
                          act_step);
}

const char* f16env_window_step_ex_kernel_name(f16env_t h, uint32_t flags) {
  static thread_local char buf[64];
  if (!h) return "";
  snprintf(buf, sizeof buf, "f16_step_winx_kernel<%d, %d, %s, %d>", h->mode & 3, h->win_occ, h->win_nt ? "true" : "false",
           (flags & F16_STEP_FEATURE_WINDOW) ? (XV_X | XV_FEAT) : XV_X);
  return buf;
}

int f16env_window_step_rollout(f16env_t h, void* stream, const f16env_rollout_slot* slot, const float* act,
                               int32_t parity, int32_t pos) {
  if (!h) return set_err(-1, "null handle");
  if (!slot) return set_err(-1, "null rollout slot");
  if (!h->wb.hist[0]) return set_err(-1, "f16env_window_bind first");
  const int b = parity & 1;
  return step_window_impl(h, stream, slot, act, h->wb.hist[b], h->wb.hist[b ^ 1], h->wb.T, pos, h->wb.rew,
                          h->wb.term, h->wb.trunc, h->wb.ep_ret, h->wb.ep_len, nullptr, nullptr);
}

int f16env_reset_window(f16env_t h, void* stream, const uint8_t* mask, const float* goals, const double* ic,
                        float* hist_cur, int64_t T, int32_t pos) {
  if (!h) return set_err(-1, "null handle");
  if (int e = window_check(h, hist_cur, nullptr, T, pos)) return e;
  ResetArgs a;
  a.s = h->soa; a.tmpl = h->tmpl; a.mask = mask; a.goals = goals; a.ic = ic; a.obs = hist_cur;
  int64_t P, Q;
  window_strides(h, T, P, Q);
  a.obs_row = Q; a.obs_off = (int64_t)(pos - h->cfg.stack_k + 1) * P; a.obs_pitch = P; a.obs_slot = WPITCH;
  a.E = env_args(h);
  a.C = h->C;
  return reset_launch(h, (hipStream_t)stream, a);
}

int f16env_window_restart(f16env_t h, void* stream, float* hist0, float* hist1, int64_t T, int32_t pos_old) {
  if (!h) return set_err(-1, "null handle");
  if (!hist1) return set_err(-1, "null history");
  if (int e = window_check(h, hist0, hist1, T, pos_old)) return e;
  const int K = h->cfg.stack_k;
  if (K < 2) return 0;
  if (pos_old - K + 2 <= K - 2) return set_err(-1, "restart source and destination overlap (pos_old < 2K-3)");
  int64_t P, Q;
  window_strides(h, T, P, Q);
  const int64_t blocks = (2 * (int64_t)(K - 1) * h->cfg.n_envs * 4 + 255) / 256;
  if (blocks > 0x7fffffffLL) return set_err(-1, "history too large for one restart launch");
  hipLaunchKernelGGL(f16_window_restart_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     (int64_t)h->cfg.n_envs, (int32_t)K, Q, P, pos_old - K + 2, hist0, hist1);
  HIPCHK(hipGetLastError());
  return 0;
}

int f16env_step_window_waves_per_simd(f16env_t h) { return h ? h->win_occ : 0; }
int f16env_step_window_nt(f16env_t h) { return h ? h->win_nt : -1; }

int f16env_step_rollout(f16env_t h, void* stream, const f16env_rollout_slot* slot, const float* act,
                        const float* obs_prev, float* obs, float* rew, uint8_t* terminated, uint8_t* truncated,
                        float* terminal_obs, double* ep_return, int32_t* ep_len, int32_t* done_idx,
                        int32_t* n_done) {
  if (!slot) return set_err(-1, "null rollout slot");
  return step_impl(h, stream, slot, act, obs_prev, obs, rew, terminated, truncated, terminal_obs, ep_return,
                   ep_len, done_idx, n_done);
}

int f16env_nonfinite_count(f16env_t h, void* stream, uint64_t* count) {
  if (!h || !count) return set_err(-1, "null argument");
  unsigned long long v = 0;
  HIPCHK(hipMemcpyAsync(&v, h->nonfinite, sizeof v, hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  *count = (uint64_t)v;
  return 0;
}

int f16env_debug_checks(f16env_t h, void* stream, uint32_t* violations) {
  if (!h || !violations) return set_err(-1, "null argument");
#ifdef F16_DEBUG_CHECKS
  unsigned int v = 0;
  HIPCHK(hipMemcpyFromSymbolAsync(&v, HIP_SYMBOL(g_f16_violations), sizeof v, 0, hipMemcpyDeviceToHost,
                                  (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  *violations = v;
  return 1;
#else
  (void)stream;
  *violations = 0;
  return 0;
#endif
}

int f16env_obs_bounds_count(f16env_t h, void* stream, uint64_t* count) {
  if (!h || !count) return set_err(-1, "null argument");
  unsigned long long v = 0;
  HIPCHK(hipMemcpyAsync(&v, h->nonfinite + 2, sizeof v, hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  *count = (uint64_t)v;
  return 0;
}

// persistent rollout launch shared by the contiguous and windowed entry points
static int rollout_launch(f16env_t h, hipStream_t st, RollArgs& a) {
  if (a.T < 1) return set_err(-1, "T must be >= 1");
  if (!a.frames || !a.actions || !a.rewards || !a.last_start || (a.T > 1 && !a.next_start))
    return set_err(-1, "frames/actions/rewards/last_start (and next_start for T > 1) are required");
  if (((uintptr_t)a.actions & 15) != 0) return set_err(-1, "actions must be 16-byte aligned");
  if (h->cfg.flags & F16_FLAG_NO_AUTORESET) return set_err(-1, "rollout_random needs auto-reset");
  a.s = h->soa; a.tmpl = h->tmpl; a.nonfinite = h->nonfinite;
  a.E = env_args(h);
  a.C = h->C;
  a.icc.c = nullptr; a.icc.n = a.E.n;
  if (h->mode) {  // cfg5 modes: every lane's next reset cached before the launch (its first reset in it)
    if (int e = icc_prepare(h, st, true)) return e;
    a.icc = h->icc;
    h->icc_steps = 0;  // the rollout consumed rows: the next windowed step refills
  }
  // two waves per SIMD when there are more waves than SIMDs (the 256-register build)
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || cus <= 0) cus = 256;
  int occ = ((int64_t)a.E.n + 63) / 64 > 4 * (int64_t)cus ? 2 : 1;
  if (getenv("F16ENV_ROLL_OCC")) occ = atoi(getenv("F16ENV_ROLL_OCC")) == 2 ? 2 : 1;
  using RollKernel = void (*)(RollArgs);
  static const RollKernel table[2][4] = {
      {f16_rollout_kernel<0, 1>, f16_rollout_kernel<1, 1>, f16_rollout_kernel<2, 1>, f16_rollout_kernel<3, 1>},
      {f16_rollout_kernel<0, 2>, f16_rollout_kernel<1, 2>, f16_rollout_kernel<2, 2>, f16_rollout_kernel<3, 2>}};
  hipLaunchKernelGGL(table[occ == 2 ? 1 : 0][h->mode & 3], dim3(nblocks(a.E.n)), dim3(BLOCK), 0, st, a);
  HIPCHK(hipGetLastError());
  return 0;
}

int f16env_rollout_random(f16env_t h, void* stream, uint64_t seed, uint64_t step0, int32_t T, const float* obs_prev,
                          float* obs, float* frames, float* actions, float* rewards, float* next_start,
                          float* last_start) {
  if (!h) return set_err(-1, "null handle");
  if (!obs_prev || !obs) return set_err(-1, "obs_prev/obs are required");
  const int K = h->cfg.stack_k;
  RollArgs a;
  memset(&a, 0, sizeof a);
  a.obs_prev = obs_prev; a.in_row = (int64_t)K * F16_OBS_DIM; a.in_pitch = F16_OBS_DIM;
  a.out0 = obs; a.out1 = nullptr; a.out_row = (int64_t)K * F16_OBS_DIM; a.out_pitch = F16_OBS_DIM;
  a.out_slot = F16_OBS_DIM;
  a.frames = frames; a.actions = actions; a.rewards = rewards; a.next_start = next_start; a.last_start = last_start;
  a.seed = seed; a.step0 = step0; a.T = T;
  a.clear_fresh = 0;
  return rollout_launch(h, (hipStream_t)stream, a);
}

int f16env_window_rollout_random(f16env_t h, void* stream, uint64_t seed, uint64_t step0, int32_t T, int32_t parity,
                                 int32_t pos, int32_t pos_out, float* frames, float* actions, float* rewards,
                                 float* next_start, float* last_start) {
  if (!h) return set_err(-1, "null handle");
  if (!h->wb.hist[0]) return set_err(-1, "f16env_window_bind first");
  const int K = h->cfg.stack_k;
  const int64_t Th = h->wb.T;
  if (pos < K - 1 || pos >= Th || pos_out < K - 1 || pos_out >= Th)
    return set_err(-1, "window positions must be in [K-1, T-1]");
  if (pos_out - K + 1 <= pos && pos - K + 1 <= pos_out)
    return set_err(-1, "the output window must not overlap the input window");
  int64_t P, Q;
  window_strides(h, Th, P, Q);
  const int b = parity & 1;
  RollArgs a;
  memset(&a, 0, sizeof a);
  a.obs_prev = h->wb.hist[b] + (int64_t)(pos - K + 1) * P; a.in_row = Q; a.in_pitch = P;
  a.out0 = h->wb.hist[0] + (int64_t)(pos_out - K + 1) * P;
  a.out1 = h->wb.hist[1] + (int64_t)(pos_out - K + 1) * P;
  a.out_row = Q; a.out_pitch = P; a.out_slot = WPITCH;
  a.frames = frames; a.actions = actions; a.rewards = rewards; a.next_start = next_start; a.last_start = last_start;
  a.seed = seed; a.step0 = step0; a.T = T;
  a.clear_fresh = 1;  // both histories hold the whole final window
  return rollout_launch(h, (hipStream_t)stream, a);
}

// on_policy_algorithm.py:236-245 over a device batch: rewards[i] += gamma * terminal_values[i]
// where the lane's episode ended by truncation only (TimeLimit.truncated), float32 per-op
// rounding as SB3 (gamma rounded to float32, the product, then the sum; no FMA)
__global__ void f16_bootstrap_kernel(int64_t n, float* __restrict__ rew, const uint8_t* __restrict__ term,
                                     const uint8_t* __restrict__ trunc, const float* __restrict__ tv, float g) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (trunc[i] && !term[i]) rew[i] = rew[i] + g * tv[i];
}

int f16env_bootstrap_timeouts(void* stream, int64_t n, float* rewards, const uint8_t* terminated,
                              const uint8_t* truncated, const float* terminal_values, double gamma) {
  if (n < 0) return set_err(-1, "n must be >= 0");
  if (n == 0) return 0;
  if (!rewards || !terminated || !truncated || !terminal_values) return set_err(-1, "null argument");
  hipLaunchKernelGGL(f16_bootstrap_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n,
                     rewards, terminated, truncated, terminal_values, (float)gamma);
  HIPCHK(hipGetLastError());
  return 0;
}

// The deferred timeout bootstrap (include/f16env.h): per step, the terminal observations of the
// lanes that ended by truncation alone are appended to a stash (one atomic per wave, ballot
// compaction as the step kernel's done list); after the rollout one value evaluation over the
// stash and a scatter of gamma * V into the rewards.
__global__ __launch_bounds__(256) void f16_bootstrap_stash_kernel(int64_t n, int32_t K, const float* __restrict__ tobs,
                                                                  int64_t row_stride, int64_t frame_stride,
                                                                  const uint8_t* __restrict__ term,
                                                                  const uint8_t* __restrict__ trunc, int64_t flat_base,
                                                                  float* __restrict__ stash, int64_t* __restrict__ idx,
                                                                  int32_t* count, int64_t cap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const bool take = i < n && trunc[i] && !term[i];
  const unsigned long long m = __ballot(take);
  if (!m) return;  // wave-uniform
  int base = 0;
  if (lane == 0) base = atomicAdd(count, __popcll(m));
  base = __shfl(base, 0);
  if (!take) return;
  const int64_t slot = (int64_t)base + __popcll(m & ((1ull << lane) - 1ull));
  F16_CHECK(slot >= 0, DBG_DONE_LIST);
  if (slot >= cap) return;
  float* dst = stash + slot * (int64_t)K * F16_OBS_DIM;
  for (int j = 0; j < K; ++j) {
    const float* src = tobs + i * row_stride + (int64_t)j * frame_stride;
#pragma unroll
    for (int c = 0; c < F16_OBS_DIM; ++c) dst[j * F16_OBS_DIM + c] = src[c];
  }
  idx[slot] = flat_base + i;
}

__global__ void f16_bootstrap_apply_kernel(int64_t m, float* __restrict__ rew, const int64_t* __restrict__ idx,
                                           const float* __restrict__ v, float g) {
#pragma clang fp contract(off)
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const int64_t r = idx[j];
  rew[r] = rew[r] + g * v[j];
}

int f16env_bootstrap_stash(void* stream, int64_t n, int32_t K, const float* tobs, int64_t row_stride,
                           int64_t frame_stride, const uint8_t* terminated, const uint8_t* truncated,
                           int64_t flat_base, float* stash_obs, int64_t* stash_idx, int32_t* count,
                           int64_t capacity) {
  if (n < 0 || K < 1 || capacity < 0) return set_err(-1, "n >= 0, K >= 1 and capacity >= 0 required");
  if (n == 0) return 0;
  if (!tobs || !terminated || !truncated || !stash_idx || !count || (capacity > 0 && !stash_obs))
    return set_err(-1, "null argument");
  hipLaunchKernelGGL(f16_bootstrap_stash_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     n, K, tobs, row_stride, frame_stride, terminated, truncated, flat_base, stash_obs, stash_idx,
                     count, capacity);
  HIPCHK(hipGetLastError());
  return 0;
}

int f16env_bootstrap_apply(void* stream, int64_t m, float* rewards, const int64_t* idx, const float* values,
                           double gamma) {
  if (m < 0) return set_err(-1, "m must be >= 0");
  if (m == 0) return 0;
  if (!rewards || !idx || !values) return set_err(-1, "null argument");
  hipLaunchKernelGGL(f16_bootstrap_apply_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     m, rewards, idx, values, (float)gamma);
  HIPCHK(hipGetLastError());
  return 0;
}

int f16env_abi_version(void) { return F16ENV_ABI_VERSION; }

int f16env_get_state(f16env_t h, void* stream, double* canon) {
  if (!h || !canon) return set_err(-1, "null argument");
  hipLaunchKernelGGL(f16_get_state_kernel, dim3(nblocks(h->soa.n)), dim3(BLOCK), 0, (hipStream_t)stream, h->soa, canon, h->C);
  HIPCHK(hipGetLastError());
  return 0;
}

int f16env_set_state(f16env_t h, void* stream, const double* canon) {
  if (!h || !canon) return set_err(-1, "null argument");
  hipStream_t st = (hipStream_t)stream;
  h->icc_steps = 0;  // episode counters may change: the next windowed step refills the reset cache
  int* wind_any = reinterpret_cast<int*>(h->nonfinite + 1);
  HIPCHK(hipMemsetAsync(wind_any, 0, sizeof(int), st));
  hipLaunchKernelGGL(f16_set_state_kernel, dim3(nblocks(h->soa.n)), dim3(BLOCK), 0, st, h->soa, canon, h->C, wind_any);
  HIPCHK(hipGetLastError());
  int w = 0;
  HIPCHK(hipMemcpyAsync(&w, wind_any, sizeof(int), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (w) h->mode |= 2;  // lanes with wind: the wind kernels from now on
  return 0;
}

int f16env_window_clear_fresh(f16env_t h, void* stream) {
  if (!h) return set_err(-1, "null handle");
  hipLaunchKernelGGL(f16_clear_fresh_kernel, dim3(nblocks(h->soa.n)), dim3(BLOCK), 0, (hipStream_t)stream, h->soa);
  HIPCHK(hipGetLastError());
  return 0;
}

int f16env_trim(f16env_t h, void* stream, const double* ic_in, double* ic_out, double* residual_out) {
  if (!h || !ic_in || !ic_out) return set_err(-1, "null argument");
  hipLaunchKernelGGL(f16_trim_kernel, dim3(nblocks(h->soa.n)), dim3(BLOCK), 0, (hipStream_t)stream,
                     (int64_t)h->soa.n, ic_in, ic_out, residual_out, h->C);
  HIPCHK(hipGetLastError());
  return 0;
}

int f16env_sample_actions(f16env_t h, void* stream, uint64_t seed, uint64_t step, float* act) {
  if (!h || !act) return set_err(-1, "null argument");
  if (((uintptr_t)act & 15) != 0) return set_err(-1, "act must be 16-byte aligned");
  hipLaunchKernelGGL(f16_sample_actions_kernel, dim3(nblocks(h->soa.n)), dim3(BLOCK), 0, (hipStream_t)stream,
                     (int64_t)h->soa.n, (int64_t)h->cfg.env_id_base, seed, step, act);
  HIPCHK(hipGetLastError());
  return 0;
}

int f16env_sample_actions_steps(f16env_t h, void* stream, uint64_t seed, uint64_t step0, int32_t T, float* act) {
  if (!h || !act) return set_err(-1, "null argument");
  if (T <= 0) return set_err(-1, "T must be > 0");
  if (((uintptr_t)act & 15) != 0) return set_err(-1, "act must be 16-byte aligned");
  const int64_t total = (int64_t)T * h->soa.n;
  const int64_t per_block = (int64_t)BLOCK * SA_PER_LANE;
  const int64_t blocks = (total + per_block - 1) / per_block;
  if (blocks > 0x7fffffff) return set_err(-1, "T x N too large");
  hipLaunchKernelGGL(f16_sample_actions_steps_kernel, dim3((unsigned)blocks), dim3(BLOCK), 0, (hipStream_t)stream,
                     (int64_t)h->soa.n, total, (int64_t)h->cfg.env_id_base, seed, step0, act);
  HIPCHK(hipGetLastError());
  return 0;
}

int f16env_window_resets_deferred(f16env_t h) {
  if (!h) return set_err(-1, "null handle");
  // cfg5 modes with F16ENV_ICC_PERIOD=0: finished lanes are reset by f16_reset_done_kernel after
  // the step kernel (the same condition f16env_step_window tests: `deferred`)
  return (h->mode && !(h->cfg.flags & F16_FLAG_NO_AUTORESET) && h->icc_period <= 0) ? 1 : 0;
}

int f16env_gae(void* stream, int64_t n_steps, int64_t n_envs, const float* rewards, const float* values,
               const float* episode_starts, const float* last_values, const uint8_t* dones, double gamma,
               double gae_lambda, float* advantages, float* returns) {
  if (n_steps <= 0 || n_envs <= 0) return set_err(-1, "n_steps and n_envs must be > 0");
  if (!rewards || !values || !episode_starts || !last_values || !dones || !advantages || !returns)
    return set_err(-1, "null argument");
  const float g = (float)gamma, gl = (float)(gamma * gae_lambda);
  // full waves and 32-step load blocks: at cfg4's 2 048 x 32 768, 0.236 ms (5.69 TB/s) against
  // 0.266 with half-populated waves (1 024 waves, round 4's first version) and 0.29-0.30 with two
  // envs per lane by float2 moves (tools/gae_sweep.py, profiles/r04_gae_sweep.json: per load
  // instruction the full wave moves two 128-B lines instead of one). F16ENV_GAE_LPW=16|32|64 and
  // F16ENV_GAE_U=8|16|32 select the others (A/B only).
  static const int lpw_env = getenv("F16ENV_GAE_LPW") ? atoi(getenv("F16ENV_GAE_LPW")) : 64;
  static const int u_env = getenv("F16ENV_GAE_U") ? atoi(getenv("F16ENV_GAE_U")) : 32;
  const int lpw = lpw_env == 32 || lpw_env == 16 ? lpw_env : 64;
  const int64_t blocks = (n_envs + lpw - 1) / lpw;
  if (blocks > 0x7fffffffLL) return set_err(-1, "n_envs too large");
  using GaeKernel = void (*)(int64_t, int64_t, const float*, const float*, const float*, const float*, const uint8_t*,
                             float, float, float*, float*);
  static const GaeKernel table[3][3] = {
      {f16_gae_kernel<8, 16>, f16_gae_kernel<8, 32>, f16_gae_kernel<8, 64>},
      {f16_gae_kernel<16, 16>, f16_gae_kernel<16, 32>, f16_gae_kernel<16, 64>},
      {f16_gae_kernel<32, 16>, f16_gae_kernel<32, 32>, f16_gae_kernel<32, 64>}};
  const GaeKernel kern = table[u_env == 8 ? 0 : (u_env == 16 ? 1 : 2)][lpw == 16 ? 0 : (lpw == 32 ? 1 : 2)];
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(64), 0, (hipStream_t)stream, n_steps, n_envs, rewards, values,
                     episode_starts, last_values, dones, g, gl, advantages, returns);
  HIPCHK(hipGetLastError());
  return 0;
}

int f16env_features(void* stream, int64_t n_frames, const float* obs, float* feat) {
  if (n_frames < 0) return set_err(-1, "n_frames must be >= 0");
  if (n_frames == 0) return 0;
  if (!obs || !feat) return set_err(-1, "null argument");
  if (((uintptr_t)obs & 3) != 0 || ((uintptr_t)feat & 3) != 0) return set_err(-1, "obs and feat must be float-aligned");
  const int64_t blocks = (n_frames + 255) / 256;
  if (blocks > 0x7fffffffLL) return set_err(-1, "n_frames too large");
  hipLaunchKernelGGL(f16_features_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n_frames, obs,
                     feat);
  HIPCHK(hipGetLastError());
  return 0;
}

int f16env_features_strided(void* stream, int64_t n_rows, int32_t K, const float* obs, int64_t row_stride,
                            int64_t frame_stride, float* feat) {
  if (n_rows < 0 || K < 1) return set_err(-1, "n_rows >= 0 and K >= 1 required");
  if (n_rows == 0) return 0;
  if (!obs || !feat) return set_err(-1, "null argument");
  if (frame_stride < 0 || row_stride < 0) return set_err(-1, "strides must be non-negative");
  if (((uintptr_t)obs & 3) != 0 || ((uintptr_t)feat & 3) != 0) return set_err(-1, "obs and feat must be float-aligned");
  const int64_t blocks = (n_rows * K + 255) / 256;
  if (blocks > 0x7fffffffLL) return set_err(-1, "too many frames");
  hipLaunchKernelGGL(f16_features_strided_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n_rows, K,
                     obs, row_stride, frame_stride, feat);
  HIPCHK(hipGetLastError());
  return 0;
}

int f16env_features_window_step(void* stream, int64_t n, int32_t K, int32_t pos, const float* hist_cur,
                                int64_t pos_stride, int64_t env_stride, float* feat_cur, float* feat_other,
                                const uint8_t* terminated, const uint8_t* truncated, int32_t autoreset,
                                int32_t transform) {
  if (n < 0 || K < 1 || pos < K - 1) return set_err(-1, "n >= 0, K >= 1 and pos >= K - 1 required");
  if (n == 0) return 0;
  if (!hist_cur || !feat_cur || !feat_other || !terminated || !truncated) return set_err(-1, "null argument");
  if ((pos_stride & 15) || (env_stride & 15) || pos_stride < 16 || env_stride < 16 || (((uintptr_t)hist_cur) & 15) != 0)
    return set_err(-1, "frame history must be 16-byte aligned with 16-float slots");
  if (((((uintptr_t)feat_cur) | ((uintptr_t)feat_other)) & 3) != 0) return set_err(-1, "feature histories must be float-aligned");
  FeatWinArgs a;
  a.wx = hist_cur; a.wrow = pos_stride; a.wenv = env_stride;
  a.fx = feat_cur; a.fy = feat_other; a.n = n; a.K = K; a.p = pos;
  a.autoreset = autoreset ? 1 : 0; a.transform = transform ? 1 : 0;
  a.term = terminated; a.trunc = truncated;
  const int64_t blocks = (n + FW_ENVS - 1) / FW_ENVS;
  if (blocks > 0x7fffffffLL) return set_err(-1, "too many envs");
  hipLaunchKernelGGL(f16_feature_window_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a);
  HIPCHK(hipGetLastError());
  return 0;
}

int f16env_poses(void* stream, int64_t n, const float* frames, int64_t frame_stride, float* out) {
  if (n < 0 || frame_stride < F16_OBS_DIM) return set_err(-1, "n >= 0 and frame_stride >= 15 required");
  if (n == 0) return 0;
  if (!frames || !out) return set_err(-1, "null argument");
  hipLaunchKernelGGL(f16_poses_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n, frames,
                     frame_stride, out);
  HIPCHK(hipGetLastError());
  return 0;
}

// The step kernel instance a handle launches in its observation layout: the windowed one once
// f16env_window_bind has been called, else the contiguous one (step_kernel_for's table).
const char* f16env_step_kernel_name(f16env_t h) {
  static thread_local char buf[64];
  if (!h) return "";
  if (h->wb.hist[0]) {
    // (as rocprofv3 demangles it: the plain step, not the rollout-slot build <.., true>)
    snprintf(buf, sizeof buf, "f16_step_win%s_kernel<%d, %d, false>", h->win_nt ? "_nt" : "", h->mode & 3, h->win_occ);
  } else if (h->gt) {
    snprintf(buf, sizeof buf, "f16_step_gt_kernel<%d, false>", h->mode & 3);  // as rocprofv3 demangles it
  } else if ((h->mode & 3) == 0 && h->occ == 1) {
    snprintf(buf, sizeof buf, "f16_step_kernel");
  } else {
    snprintf(buf, sizeof buf, "f16_step_var_kernel<%d, %d, false>", h->mode & 3, h->occ);
  }
  return buf;
}
int f16env_step_waves_per_simd(f16env_t h) { return h ? h->occ : 0; }
int f16env_step_mode(f16env_t h) { return h ? h->mode : -1; }
int f16env_step_variant(f16env_t h) { return h ? (h->gt ? 2 : (h->occ == 2 ? 1 : 0)) : -1; }

double f16env_algorithmic_bytes_per_env_step(int stack_k) {
  return 16.0 + 60.0 * stack_k + 60.0 * (stack_k - 1) + 4.0 + 2.0 + 2.0 * STATE_BYTES;
}

const char* f16env_last_error(void) { return g_err.c_str(); }

#ifdef F16_STAMPS
// diagnostic build only: copy per-wave section cycle totals (waves x ST_N u64) to host
int f16env_diag_stamps(unsigned long long* host, int max_waves) {
  const int n = max_waves < (1 << 14) ? max_waves : (1 << 14);
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * ST_N * n, 0,
                             hipMemcpyDeviceToHost));
  return ST_N;
}
#endif

}  // extern "C"
