/*
 * f16ref.c -- CPU fp64 restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY
 * (the oracle / CPU baseline; never linked into libf16env.so).
 *
 * What it restates, and from where:
 *   env layer      jsbsim_gym/jsbsim_gym.py:60-78 (angle normalisation), :172-197 (obs frame),
 *                  :199-287 (step), :289-331 (reset), :470-519 (PositionReward), gymnasium
 *                  TimeLimit(1200) (:537-545), common/monitor.py:85-111 (episode stats),
 *                  common/vec_env/dummy_vec_env.py:56-83 (auto-reset, terminal obs).
 *   FDM data       aircraft/f16/f16.xml (tables via tools/gen_tables.py -> f16ref_tables.h),
 *                  aircraft/f16/Engines/F100-PW-229.xml, Engines/direct.xml.
 *   FDM semantics  JSBSim (external, requirements.txt:4, unpinned): FGFDMExec::Run model
 *                  order, FGPropagate integrators (rect-Euler rotation, AB2 translational
 *                  rate, AB3 translational position), FGInertial WGS84+J2, FGStandardAtmosphere
 *                  (US-1976), FGAuxiliary, FGFCS components (switch/pure_gain/scheduled_gain/
 *                  summer/pid/kinematic/aerosurface_scale/fcs_function), FGTurbine,
 *                  FGAerodynamics (wind-axis lift/drag), FGMassBalance, FGAccelerations.
 *                  These are restated from JSBSim's public design; JSBSim's source is not in
 *                  this environment, so JSBSim parity is UNPINNED.
 *
 * Deliberate, documented choices where the reference/JSBSim behaviour is undefined or
 * unavailable here (DESIGN.md "Model choices"):
 *   - RunIC = three evaluation passes without integration; FCS actuators settle on their
 *     commanded value (FGKinematic trim-mode semantics), PID derivative history primed,
 *     engine N2 at its target; then the integrator histories are filled
 *     (FGPropagate::InitializeDerivatives). Every reset is a full lane reset.
 *   - Ground reactions are not modelled (gear retracted by the per-substep pins,
 *     jsbsim_gym.py:230-231; the env terminates at 10 m AGL).
 *   - Mass, CG and inertia are constant (tanks pinned to 1000 lb before every run(),
 *     jsbsim_gym.py:227-228).
 */
#include "f16ref.h"
#include "f16ref_tables.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------------
 * constants
 * ---------------------------------------------------------------------------------------- */
#define PI 3.14159265358979323846
#define FT2M 0.3048
#define INCH2FT (1.0 / 12.0)
#define SLUG2LB 32.174049
#define KTS2FPS (1852.0 / (3600.0 * 0.3048))
#define RAD2DEG (180.0 / PI)
/* WGS84 / FGInertial defaults */
#define WGS_A 20925646.32546
#define WGS_B 20855486.5951
#define GM_E 14.0764417572e15
#define J2_E 1.08262982e-03
#define OMEGA_E 0.00007292115
/* env constants (jsbsim_gym.py) */
#define RADIUS_M 6.3781e6 /* :56 */

/* aircraft (f16.xml:37-83,245-300) */
static const double S_W = 300.0, B_W = 30.0, CBAR = 11.32;

typedef struct {
  double mass;           /* slug */
  double cg[3];          /* structural, in */
  double J[9], Jinv[9];  /* body, slug ft^2 */
  double rp[3];          /* AERORP rel. CG, body ft */
  double eye[3];         /* EYEPOINT rel. CG, body ft */
  double eng[3];         /* thruster rel. CG, body ft */
  double gref;           /* FGInertial gAccelReference = GM/a^2 */
  double e2, ec, ec2, c; /* ellipse constants */
} consts_t;
static consts_t K;
static int K_ready = 0;

/* Test-only physics switch (f16ref_set_physics_mask, default 0 = the full model): drops the
 * aerodynamic forces and moments, the thrust, gravity, or J2 (central gravity only), so CPU
 * tests can check the equations of motion against analytic invariants
 * (tests/test_oracle_physics.py); F16REF_TEST_SHAPING_2D is a deliberate defect -- the
 * PositionReward distance over (x, y) only instead of jsbsim_gym.py:496-500's 3-D norm -- that
 * the reward parity tests must reject (tests/reward_bound.py). Process-wide; tests set it
 * around their own runs. */
static int g_phys_mask = 0;
void f16ref_set_physics_mask(int mask) { g_phys_mask = mask; }
static void init_consts(void);
/* body inertia (slug ft^2, incl. pilot and the pinned tanks) and mass (slug), for tests */
void f16ref_mass_props(double J[9], double* mass) {
  init_consts();
  memcpy(J, K.J, sizeof K.J);
  *mass = K.mass;
}
int f16ref_get_physics_mask(void) { return g_phys_mask; }

/* ------------------------------------------------------------------------------------------
 * small linear algebra (row-major 3x3)
 * ---------------------------------------------------------------------------------------- */
static void mv(const double* M, const double* v, double* o) {
  double a = M[0] * v[0] + M[1] * v[1] + M[2] * v[2];
  double b = M[3] * v[0] + M[4] * v[1] + M[5] * v[2];
  double c = M[6] * v[0] + M[7] * v[1] + M[8] * v[2];
  o[0] = a; o[1] = b; o[2] = c;
}
static void mtv(const double* M, const double* v, double* o) { /* M^T v */
  double a = M[0] * v[0] + M[3] * v[1] + M[6] * v[2];
  double b = M[1] * v[0] + M[4] * v[1] + M[7] * v[2];
  double c = M[2] * v[0] + M[5] * v[1] + M[8] * v[2];
  o[0] = a; o[1] = b; o[2] = c;
}
static void mm(const double* A, const double* B, double* C) {
  double T[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      T[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
  memcpy(C, T, sizeof T);
}
static void mT(const double* A, double* B) {
  double T[9] = {A[0], A[3], A[6], A[1], A[4], A[7], A[2], A[5], A[8]};
  memcpy(B, T, sizeof T);
}
static void cross(const double* a, const double* b, double* o) {
  double x = a[1] * b[2] - a[2] * b[1];
  double y = a[2] * b[0] - a[0] * b[2];
  double z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}
static int inv3(const double* M, double* I) {
  double a = M[0], b = M[1], c = M[2], d = M[3], e = M[4], f = M[5], g = M[6], h = M[7], k = M[8];
  double A = e * k - f * h, B = -(d * k - f * g), C = d * h - e * g;
  double det = a * A + b * B + c * C;
  if (det == 0.0) return -1;
  double r = 1.0 / det;
  I[0] = A * r; I[1] = -(b * k - c * h) * r; I[2] = (b * f - c * e) * r;
  I[3] = B * r; I[4] = (a * k - c * g) * r; I[5] = -(a * f - c * d) * r;
  I[6] = C * r; I[7] = -(a * h - b * g) * r; I[8] = (a * e - b * d) * r;
  return 0;
}

/* StructuralToBody (FGMassBalance): structural inches -> body feet relative to the CG */
static void s2b(const double* cg, const double* r, double* o) {
  o[0] = INCH2FT * (cg[0] - r[0]);
  o[1] = INCH2FT * (r[1] - cg[1]);
  o[2] = INCH2FT * (cg[2] - r[2]);
}
/* FGMassBalance::GetPointmassInertia */
static void pm_inertia(double m, const double* v, double* J) {
  double sv[3] = {m * v[0], m * v[1], m * v[2]};
  double xx = sv[0] * v[0], yy = sv[1] * v[1], zz = sv[2] * v[2];
  double xy = -sv[0] * v[1], xz = -sv[0] * v[2], yz = -sv[1] * v[2];
  J[0] += yy + zz; J[1] += xy; J[2] += xz;
  J[3] += xy; J[4] += xx + zz; J[5] += yz;
  J[6] += xz; J[7] += yz; J[8] += xx + yy;
}

/* Mass balance (f16.xml:62-83; tanks f16.xml:264-299 pinned per jsbsim_gym.py:227-228). */
static void init_consts(void) {
  if (K_ready) return;
  const double empty = 17400.0, cg_e[3] = {-193.0, 0.0, -5.1};
  const double pilot = 230.0, pilot_loc[3] = {-336.2, 0.0, 0.0};
  const double tank_w[4] = {1000.0, 1000.0, 0.0, 0.0};
  const double tank_loc[4][3] = {{-174.4, 65.0, 5.0}, {-174.4, -65.0, 5.0},
                                 {-174.4, 65.0, -15.0}, {-174.4, -65.0, -15.0}};
  double W = empty + pilot, m[3];
  for (int i = 0; i < 3; i++) m[i] = empty * cg_e[i] + pilot * pilot_loc[i];
  for (int t = 0; t < 4; t++) {
    W += tank_w[t];
    for (int i = 0; i < 3; i++) m[i] += tank_w[t] * tank_loc[t][i];
  }
  for (int i = 0; i < 3; i++) K.cg[i] = m[i] / W;
  K.mass = W / SLUG2LB;
  /* negated_crossproduct_inertia="true": J = [ixx,-ixy,ixz; -ixy,iyy,-iyz; ixz,-iyz,izz] */
  const double ixx = 9496, iyy = 55814, izz = 63100, ixy = 0, ixz = -982, iyz = 0;
  double J[9] = {ixx, -ixy, ixz, -ixy, iyy, -iyz, ixz, -iyz, izz};
  double v[3];
  s2b(K.cg, pilot_loc, v);
  pm_inertia(pilot / SLUG2LB, v, J);
  for (int t = 0; t < 4; t++) {
    s2b(K.cg, tank_loc[t], v);
    pm_inertia(tank_w[t] / SLUG2LB, v, J);
  }
  memcpy(K.J, J, sizeof J);
  inv3(K.J, K.Jinv);
  const double aerorp[3] = {-189.5, 0.0, 3.9}, eye[3] = {-336.2, 0.0, 29.5}, eng[3] = {0, 0, 0};
  s2b(K.cg, aerorp, K.rp);
  s2b(K.cg, eye, K.eye);
  s2b(K.cg, eng, K.eng);
  K.gref = GM_E / (WGS_A * WGS_A);
  K.e2 = 1.0 - (WGS_B * WGS_B) / (WGS_A * WGS_A);
  K.ec2 = 1.0 - K.e2;
  K.ec = sqrt(K.ec2);
  K.c = WGS_A * K.e2;
  K_ready = 1;
}

/* ------------------------------------------------------------------------------------------
 * tables (FGTable::GetValue: clamped linear / bilinear, no extrapolation, f16.xml:536-537)
 * ---------------------------------------------------------------------------------------- */
static double tab1(const ref_table* t, double x) {
  const int n = t->nrows;
  const double* r = t->rows;
  const double* d = t->data;
  if (x <= r[0]) return d[0];
  if (x >= r[n - 1]) return d[n - 1];
  int i = 1;
  while (i < n - 1 && r[i] < x) i++;
  double span = r[i] - r[i - 1];
  double f = span != 0.0 ? (x - r[i - 1]) / span : 1.0;
  if (f > 1.0) f = 1.0;
  return f * (d[i] - d[i - 1]) + d[i - 1];
}
static double tab2(const ref_table* t, double x, double y) {
  if (t->ncols == 0) return tab1(t, x);
  const int nr = t->nrows, nc = t->ncols;
  int i = 1, j = 1;
  while (i < nr - 1 && t->rows[i] < x) i++;
  while (j < nc - 1 && t->cols[j] < y) j++;
  double rf = (x - t->rows[i - 1]) / (t->rows[i] - t->rows[i - 1]);
  double cf = (y - t->cols[j - 1]) / (t->cols[j] - t->cols[j - 1]);
  if (rf > 1.0) rf = 1.0; else if (rf < 0.0) rf = 0.0;
  if (cf > 1.0) cf = 1.0; else if (cf < 0.0) cf = 0.0;
  const double* d = t->data;
  double c1 = rf * (d[i * nc + j - 1] - d[(i - 1) * nc + j - 1]) + d[(i - 1) * nc + j - 1];
  double c2 = rf * (d[i * nc + j] - d[(i - 1) * nc + j]) + d[(i - 1) * nc + j];
  return c1 + cf * (c2 - c1);
}

/* ------------------------------------------------------------------------------------------
 * US-1976 standard atmosphere (FGStandardAtmosphere), SI internally, geopotential altitude
 * ---------------------------------------------------------------------------------------- */
void f16ref_atmosphere(double h_ft, double out[4]) {
  static const double Hb[8] = {0.0, 11000.0, 20000.0, 32000.0, 47000.0, 51000.0, 71000.0, 84852.0};
  static const double Lb[7] = {-0.0065, 0.0, 0.001, 0.0028, 0.0, -0.0028, -0.002};
  static double Tb[8], Pb[8];
  static int init = 0;
  const double g0 = 9.80665, Rstar = 8.31432, M = 0.0289644, r0 = 6356766.0;
  const double GMR = g0 * M / Rstar;
  if (!init) {
    Tb[0] = 288.15; Pb[0] = 101325.0;
    for (int i = 0; i < 7; i++) {
      double dh = Hb[i + 1] - Hb[i];
      Tb[i + 1] = Tb[i] + Lb[i] * dh;
      if (Lb[i] != 0.0) Pb[i + 1] = Pb[i] * pow(Tb[i] / Tb[i + 1], GMR / Lb[i]);
      else Pb[i + 1] = Pb[i] * exp(-GMR * dh / Tb[i]);
    }
    init = 1;
  }
  double z = h_ft * FT2M;
  double H = r0 * z / (r0 + z); /* geopotential */
  int b = 0;
  while (b < 6 && H >= Hb[b + 1]) b++;
  double T, P;
  if (Lb[b] != 0.0) {
    T = Tb[b] + Lb[b] * (H - Hb[b]);
    P = Pb[b] * pow(Tb[b] / T, GMR / Lb[b]);
  } else {
    T = Tb[b];
    P = Pb[b] * exp(-GMR * (H - Hb[b]) / Tb[b]);
  }
  double R = Rstar / M;
  double rho = P / (R * T);
  double a = sqrt(1.4 * R * T);
  /* SI -> JSBSim English units */
  out[0] = T * 1.8;                        /* Rankine */
  out[1] = P / 47.88025898033584;          /* psf     */
  out[2] = rho / 515.3788183931961;        /* slug/ft^3 */
  out[3] = a / FT2M;                       /* ft/s    */
}
static double atm_rho_sl(void) {
  static double r = 0.0;
  if (r == 0.0) { double o[4]; f16ref_atmosphere(0.0, o); r = o[2]; }
  return r;
}
static double atm_p_sl(void) { return 101325.0 / 47.88025898033584; }
static double atm_a_sl(void) {
  static double a = 0.0;
  if (a == 0.0) { double o[4]; f16ref_atmosphere(0.0, o); a = o[3]; }
  return a;
}

/* FGAuxiliary::PitotTotalPressure / MachFromImpactPressure / VcalibratedFromMach */
static double pitot_total(double mach, double p) {
  if (mach < 0) return p;
  if (mach < 1) return p * pow(1.0 + 0.2 * mach * mach, 3.5);
  return p * 166.92158009316827 * pow(mach, 7.0) / pow(7.0 * mach * mach - 1.0, 2.5);
}
static double mach_from_qc(double qc, double p) {
  double A = qc / p + 1.0;
  double M = sqrt(5.0 * (pow(A, 1.0 / 3.5) - 1.0));
  if (M > 1.0)
    for (int i = 0; i < 10; i++) M = 0.8812848543473311 * sqrt(A * pow(1.0 - 1.0 / (7.0 * M * M), 2.5));
  return M;
}
double f16ref_vcas_kts(double mach, double p) {
  if (!(fabs(mach) > 0.0)) return 0.0;
  double qc = pitot_total(mach, p) - p;
  return atm_a_sl() * mach_from_qc(qc, atm_p_sl()) / KTS2FPS;
}

/* ------------------------------------------------------------------------------------------
 * WGS84 (FGLocation): geodetic -> ECEF, ECEF -> geodetic altitude (Fukushima 2006, one
 * Halley iteration, as FGLocation::ComputeDerivedUnconditional)
 * ---------------------------------------------------------------------------------------- */
void f16ref_geodetic_to_ecef(double lat, double lon, double h, double e[3]) {
  init_consts();
  double sl = sin(lat), cl = cos(lat);
  double N = WGS_A / sqrt(1.0 - K.e2 * sl * sl);
  e[0] = (N + h) * cl * cos(lon);
  e[1] = (N + h) * cl * sin(lon);
  e[2] = (K.ec2 * N + h) * sl;
}
double f16ref_geodetic_altitude(const double e[3]) {
  init_consts();
  double rxy = sqrt(e[0] * e[0] + e[1] * e[1]);
  double s0 = fabs(e[2]);
  double zc = K.ec * s0, c0 = K.ec * rxy;
  double c02 = c0 * c0, s02 = s0 * s0;
  double a02 = c02 + s02, a0 = sqrt(a02), a03 = a02 * a0;
  double s1 = zc * a03 + K.c * s02 * s0;
  double c1 = rxy * a03 - K.c * c02 * c0;
  double cs0c0 = K.c * c0 * s0;
  double b0 = 1.5 * cs0c0 * ((rxy * s0 - zc * c0) * a0 - cs0c0);
  s1 = s1 * a03 - b0 * s0;
  double cc = K.ec * (c1 * a03 - b0 * c0);
  double s12 = s1 * s1, cc2 = cc * cc;
  double norm = sqrt(s12 + cc2);
  return (rxy * cc + s0 * s1 - WGS_A * sqrt(K.ec2 * s12 + cc2)) / norm;
}

/* ------------------------------------------------------------------------------------------
 * quaternion helpers (FGQuaternion)
 * ---------------------------------------------------------------------------------------- */
static void quat_T(const double* q, double* T) { /* FGQuaternion::GetT: from-frame -> body */
  double q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
  double q0q0 = q0 * q0, q1q1 = q1 * q1, q2q2 = q2 * q2, q3q3 = q3 * q3;
  T[0] = q0q0 + q1q1 - q2q2 - q3q3;
  T[1] = 2.0 * (q1 * q2 + q0 * q3);
  T[2] = 2.0 * (q1 * q3 - q0 * q2);
  T[3] = 2.0 * (q1 * q2 - q0 * q3);
  T[4] = q0q0 - q1q1 + q2q2 - q3q3;
  T[5] = 2.0 * (q2 * q3 + q0 * q1);
  T[6] = 2.0 * (q1 * q3 + q0 * q2);
  T[7] = 2.0 * (q2 * q3 - q0 * q1);
  T[8] = q0q0 - q1q1 - q2q2 + q3q3;
}
static void mat_quat(const double* T, double* q) { /* FGMatrix33::GetQuaternion */
  double t[4] = {1.0 + T[0] + T[4] + T[8], 1.0 + T[0] - T[4] - T[8],
                 1.0 - T[0] + T[4] - T[8], 1.0 - T[0] - T[4] + T[8]};
  int idx = 0;
  for (int i = 1; i < 4; i++)
    if (t[i] > t[idx]) idx = i;
  switch (idx) {
    case 0:
      q[0] = 0.5 * sqrt(t[0]);
      q[1] = 0.25 * (T[5] - T[7]) / q[0];
      q[2] = 0.25 * (T[6] - T[2]) / q[0];
      q[3] = 0.25 * (T[1] - T[3]) / q[0];
      break;
    case 1:
      q[1] = 0.5 * sqrt(t[1]);
      q[0] = 0.25 * (T[5] - T[7]) / q[1];
      q[2] = 0.25 * (T[1] + T[3]) / q[1];
      q[3] = 0.25 * (T[2] + T[6]) / q[1];
      break;
    case 2:
      q[2] = 0.5 * sqrt(t[2]);
      q[0] = 0.25 * (T[6] - T[2]) / q[2];
      q[1] = 0.25 * (T[1] + T[3]) / q[2];
      q[3] = 0.25 * (T[5] + T[7]) / q[2];
      break;
    default:
      q[3] = 0.5 * sqrt(t[3]);
      q[0] = 0.25 * (T[1] - T[3]) / q[3];
      q[1] = 0.25 * (T[2] + T[6]) / q[3];
      q[2] = 0.25 * (T[5] + T[7]) / q[3];
  }
  if (q[0] < 0) for (int i = 0; i < 4; i++) q[i] = -q[i];
}
static void euler_T(double phi, double tht, double psi, double* T) { /* Tl2b from Euler 3-2-1 */
  double cp = cos(phi), sp = sin(phi), ct = cos(tht), st = sin(tht), cs = cos(psi), ss = sin(psi);
  T[0] = ct * cs;                 T[1] = ct * ss;                 T[2] = -st;
  T[3] = sp * st * cs - cp * ss;  T[4] = sp * st * ss + cp * cs;  T[5] = sp * ct;
  T[6] = cp * st * cs + sp * ss;  T[7] = cp * st * ss - sp * cs;  T[8] = cp * ct;
}
static void T_euler(const double* T, double* e) { /* FGMatrix33::GetEuler -> phi, theta, psi */
  if (T[2] <= -1.0) {
    e[1] = 0.5 * PI; e[0] = atan2(-T[7], T[4]); e[2] = 0.0;
  } else if (T[2] >= 1.0) {
    e[1] = -0.5 * PI; e[0] = atan2(-T[7], T[4]); e[2] = 0.0;
  } else {
    e[1] = asin(-T[2]);
    e[0] = atan2(T[5], T[8]);
    double psi = atan2(T[1], T[0]);
    if (psi < 0.0) psi += 2.0 * PI;
    e[2] = psi;
  }
}

/* ------------------------------------------------------------------------------------------
 * per-env state
 * ---------------------------------------------------------------------------------------- */
typedef struct {
  double rI[3], vI[3], vIh1[3], vIh2[3], aI[3], aIp[3];
  double q[4], wI[3], wId[3], ba[3];
  double epa_c, epa_s, epa;
  double tef, ail, ele, rud, lef, sb;
  double pid_r_i, pid_r_p, pid_p_i, pid_p_p, pid_y_i, pid_y_p;
  double n1, n2, aug;
  double lx[F16L_N];
  double cmd[4];
  double wind[3];
  double gust[3]; /* cfg5 Gauss-Markov gust, NED fps (F16_FLAG_GUSTS) */
  float goal[3];
  float last_d;
  int32_t step;
  double ep_ret;
  uint64_t ep_count;
  float* stack; /* K x 15 ring, oldest first at (head) */
  int head;
} env_t;

typedef struct { /* quantities derived from the propagated state (FGPropagate getters) */
  double rE[3], r, rxy, slat, clat, slon, clon, lat_gc, lon, h_ft;
  double Ti2b[9], Tb2i[9], Tec2b[9], Tl2b[9], Tb2l[9], Tec2l[9];
  double uvw[3], pqr[3], vned[3], eul[3];
} derived_t;

struct f16ref {
  f16env_config cfg;
  int n;
  env_t* env;
  float* stacks;
  uint64_t obs_oob; /* F16_FLAG_OBS_CHECK: lane-steps with a finite out-of-bounds new frame */
};

/* jsbsim_gym.py:268-285: observation_space.contains(obs) fails on a FINITE value outside
 * SINGLE_OBS_LOW / SINGLE_OBS_HIGH (:28-53, float32 arrays); checked on the new frame */
static int obs_out_of_bounds(const float* f) {
  static const float pe = (float)(3.14159265358979323846 + 1e-5), he = (float)(1.5707963267948966 + 1e-5);
  const float lo[F16_OBS_DIM] = {-INFINITY, -INFINITY, -INFINITY, 0.0f, -pe, -pe, -INFINITY, -INFINITY, -INFINITY,
                                 -pe, -he, -pe, -INFINITY, -INFINITY, 0.0f};
  const float hi[F16_OBS_DIM] = {INFINITY, INFINITY, INFINITY, INFINITY, pe, pe, INFINITY, INFINITY, INFINITY,
                                 pe, he, pe, INFINITY, INFINITY, INFINITY};
  for (int j = 0; j < F16_OBS_DIM; j++)
    if (isfinite(f[j]) && (f[j] < lo[j] || f[j] > hi[j])) return 1;
  return 0;
}

static void derive(const env_t* e, derived_t* d) {
  /* Ti2ec (FGLocation) and vLocation = Ti2ec * vInertialPosition */
  double c = e->epa_c, s = e->epa_s;
  d->rE[0] = c * e->rI[0] + s * e->rI[1];
  d->rE[1] = -s * e->rI[0] + c * e->rI[1];
  d->rE[2] = e->rI[2];
  d->rxy = sqrt(d->rE[0] * d->rE[0] + d->rE[1] * d->rE[1]);
  d->r = sqrt(d->rxy * d->rxy + d->rE[2] * d->rE[2]);
  if (d->rxy == 0.0) { d->slon = 0.0; d->clon = 1.0; d->lon = 0.0; }
  else { d->slon = d->rE[1] / d->rxy; d->clon = d->rE[0] / d->rxy; d->lon = atan2(d->rE[1], d->rE[0]); }
  d->lat_gc = atan2(d->rE[2], d->rxy);
  d->slat = d->rE[2] / d->r;
  d->clat = d->rxy / d->r;
  d->h_ft = f16ref_geodetic_altitude(d->rE);
  double* L = d->Tec2l;
  L[0] = -d->clon * d->slat; L[1] = -d->slon * d->slat; L[2] = d->clat;
  L[3] = -d->slon;           L[4] = d->clon;            L[5] = 0.0;
  L[6] = -d->clon * d->clat; L[7] = -d->slon * d->clat; L[8] = -d->slat;
  double Tec2i[9] = {c, -s, 0, s, c, 0, 0, 0, 1}; /* transpose of Ti2ec */
  quat_T(e->q, d->Ti2b);
  mT(d->Ti2b, d->Tb2i);
  mm(d->Ti2b, Tec2i, d->Tec2b);
  double Tl2ec[9];
  mT(L, Tl2ec);
  mm(d->Tec2b, Tl2ec, d->Tl2b);
  mT(d->Tl2b, d->Tb2l);
  /* CalculateUVW: vUVW = Ti2b * (vInertialVelocity - omega x r) */
  double v[3] = {e->vI[0] + OMEGA_E * e->rI[1], e->vI[1] - OMEGA_E * e->rI[0], e->vI[2]};
  mv(d->Ti2b, v, d->uvw);
  /* vPQR = vPQRi - Ti2b * omega */
  double w[3] = {0, 0, OMEGA_E}, wb[3];
  mv(d->Ti2b, w, wb);
  for (int i = 0; i < 3; i++) d->pqr[i] = e->wI[i] - wb[i];
  mv(d->Tb2l, d->uvw, d->vned);
  T_euler(d->Tl2b, d->eul);
}

/* FGInertial::GetGravityJ2 (ECEF) */
static void gravity_j2(const derived_t* d, double* g) {
  double r = d->r, sl = d->slat;
  double adivr = WGS_A / r;
  double pre = (g_phys_mask & F16REF_PHYS_NO_J2) ? 0.0 : 1.5 * J2_E * adivr * adivr;
  double xy = 1.0 - 5.0 * sl * sl, z = 3.0 - 5.0 * sl * sl;
  double gm = GM_E / (r * r);
  g[0] = -gm * (1.0 + pre * xy) * d->rE[0] / r;
  g[1] = -gm * (1.0 + pre * xy) * d->rE[1] / r;
  g[2] = -gm * (1.0 + pre * z) * d->rE[2] / r;
}

/* ------------------------------------------------------------------------------------------
 * FCS components (FGFCSComponent family)
 * ---------------------------------------------------------------------------------------- */
static double clip(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
static int eq_roundoff(double a, double b) {
  double m = fabs(a) > fabs(b) ? fabs(a) : fabs(b);
  return fabs(a - b) <= 2.0 * 2.220446049250313e-16 * m;
}
/* FGKinematic::Run: rate-limited traverse between detents (input clamped to the detent
 * range; ic => trim-mode: output = input). */
static double kinematic(double out, double in, const double* det, const double* tim, int n,
                        double dt, int ic) {
  if (in < det[0]) in = det[0];
  else if (in > det[n - 1]) in = det[n - 1];
  if (ic) return in;
  double dt0 = dt;
  for (int guard = 0; guard < 2 * n + 2 && dt0 > 0.0 && !eq_roundoff(in, out); guard++) {
    int ind = 1;
    if (in < out) { while (ind < n - 1 && det[ind] < out) ind++; }
    else          { while (ind < n - 1 && det[ind] <= out) ind++; }
    if (tim[ind] <= 0.0) { out = in; break; }
    double rate = (det[ind] - det[ind - 1]) / tim[ind];
    double tin = in;
    if (tin < det[ind - 1]) tin = det[ind - 1];
    if (det[ind] < tin) tin = det[ind];
    double tdt = fabs((tin - out) / rate);
    if (dt0 < tdt) {
      tdt = dt0;
      if (out < in) out += tdt * rate; else out -= tdt * rate;
    } else {
      out = tin;
    }
    dt0 -= tdt;
  }
  return out;
}
/* FGPID::Run (rect integrator, non-"standard" form); trigger != 0 holds the integrator,
 * trigger < 0 resets it. ic => no integration, derivative 0. */
static double pid(double in, double* itot, double* prev, double trig, double kp, double ki,
                  double kd, double dt, int ic) {
  double dval = ic ? 0.0 : (in - *prev) / dt;
  double delta = (!ic && fabs(trig) < 0.000001) ? in : 0.0;
  if (trig < 0.0) *itot = 0.0;
  *itot += ki * dt * delta;
  double out = kp * in + *itot + kd * dval;
  *prev = in;
  return out;
}
/* aerosurface_scale, zero_centered (FGGain) */
static double aero_scale(double in, double inmin, double inmax, double outmin, double outmax) {
  if (in == 0.0) return 0.0;
  if (in > 0.0) return (in / inmax) * outmax;
  return (in / inmin) * outmin;
}

/* the FCS / engine components as stand-alone entry points for unit tests */
double f16ref_kinematic(double out, double in, const double* detents, const double* times, int n, double dt,
                        int ic) {
  return kinematic(out, in, detents, times, n, dt, ic);
}
double f16ref_pid(double in, double* integral, double* prev, double trigger, double kp, double ki, double kd,
                  double dt, int ic) {
  return pid(in, integral, prev, trigger, kp, ki, kd, dt, ic);
}
double f16ref_aero_scale(double in, double inmin, double inmax, double outmin, double outmax) {
  return aero_scale(in, inmin, inmax, outmin, outmax);
}

typedef struct { double de, da, dr, dlef, flap_mix, dsb, throttle; } fcs_out_t;

/* flight_control "F-16 FC", f16.xml:309-984, channels and components in document order.
 * Reads the previous frame's auxiliary latch (Systems run before Auxiliary in
 * FGFDMExec::Run) and current propagate outputs (theta, phi, v-fps). */
static void fcs_run(env_t* e, const derived_t* d, double dt, int ic, fcs_out_t* o) {
  const double alpha = e->lx[F16L_ALPHA], mach = e->lx[F16L_MACH], vc = e->lx[F16L_VC_KTS];
  const double vg = e->lx[F16L_VG_FPS];
  const double cmd_ail = e->cmd[0], cmd_ele = e->cmd[1], cmd_rud = e->cmd[2], cmd_thr = e->cmd[3];
  static const double d2[2] = {-1.0, 1.0};
  /* -- Flaps (:317-352) -- */
  double tef_rad = 0.0;
  if (vc < 250.0) tef_rad = 0.349;
  else if (mach > 0.9) tef_rad = -0.0349;
  double tef_norm = tef_rad * 2.864789;
  { static const double det[3] = {-1.0, 0.0, 1.0}, tim[3] = {3.0, 0.0, 3.0};
    e->tef = kinematic(e->tef, tef_norm, det, tim, 3, dt, ic); }
  /* -- Roll (:354-491) -- */
  double roll_rate_norm = e->lx[F16L_P_AERO] * 0.31821;
  double roll_err = cmd_ail - roll_rate_norm;
  double ail_trig = (vc < 20.0) ? 0.0 : 1.0;
  double roll_pid = pid(roll_err, &e->pid_r_i, &e->pid_r_p, ail_trig, 3.0, 0.0005, -0.00125, dt, ic);
  double roll_cmd = clip(roll_pid + cmd_ail, -1.0, 1.0);
  o->da = aero_scale(roll_cmd, -1.0, 1.0, -0.375, 0.375);           /* fcs/aileron-pos-rad */
  { static const double tim[2] = {0.3, 0.3};
    e->ail = kinematic(e->ail, roll_cmd, d2, tim, 2, dt, ic); }       /* left-aileron-pos-norm */
  double asc = e->ail * tab1(&T_aileron_speed_compensated, mach);
  double lflap = clip(-e->tef - asc, -1.0, 1.0);
  double rflap = clip(e->tef - asc, -1.0, 1.0);
  o->flap_mix = (lflap + rflap) * 1.4324;
  /* -- Pitch (:493-672) -- */
  double nz_corr = cos(d->eul[1]) * cos(d->eul[0]);
  double g_corr = e->lx[F16L_NPZ] - nz_corr;
  double ele_lim = clip(cmd_ele + 0.0 /* pitch-trim-cmd-norm */, -1.0, 0.44);
  double ele_sched = ele_lim * tab1(&T_elevator_scheduler, alpha);
  double alpha_lim = alpha * 1.0472;
  double q_norm = e->lx[F16L_Q_AERO] * 6.2;
  double g_norm = g_corr * 0.020;
  double pitch_err = ele_sched + q_norm - g_norm;
  double ele_trig = (vc < 5.0) ? 0.0 : 1.0;
  double gpid = clip(pid(pitch_err, &e->pid_p_i, &e->pid_p_p, ele_trig, 0.3, 0.025, 0.0, dt, ic), -1.0, 1.0);
  double pitch_sched = clip(ele_sched + alpha_lim + gpid, -1.0, 1.0);
  { static const double tim[2] = {0.3, 0.3};
    e->ele = kinematic(e->ele, pitch_sched, d2, tim, 2, dt, ic); }    /* elevator-pos-norm */
  o->de = aero_scale(e->ele, -1.0, 1.0, -0.436, 0.436);               /* elevator-pos-rad */
  /* -- Yaw (:674-763) -- */
  double yaw_rate_norm = e->lx[F16L_R_AERO] * tab1(&T_yaw_rate_norm, vg);
  double yaw_load_norm = e->lx[F16L_NPY] * 0.25;
  double yaw_err = cmd_rud + yaw_rate_norm + yaw_load_norm;
  double rud_trig = (vc < 10.0) ? 0.0 : 1.0;
  double ypid = clip(pid(yaw_err, &e->pid_y_i, &e->pid_y_p, rud_trig, 0.1055, 0.00001, 0.00005, dt, ic), -1.0, 1.0);
  double yaw_sched = clip(cmd_rud + 0.0 /* yaw-trim-cmd-norm */ + ypid, -1.0, 1.0);
  { static const double tim[2] = {0.4, 0.4};
    e->rud = kinematic(e->rud, yaw_sched, d2, tim, 2, dt, ic); }      /* rudder-pos-norm */
  o->dr = aero_scale(e->rud, -1.0, 1.0, -0.524, 0.524);               /* rudder-pos-rad */
  /* -- Landing Gear (:765-803): gear-cmd/pos pinned to 0 (jsbsim_gym.py:230-231), no WOW -- */
  const double gear_wow = 0.0, gear_pos = 0.0;
  /* -- Leading Edge Flap (:805-857) -- */
  double lef_rad = 0.0;
  if (gear_wow == 1.0 && gear_pos > 0.0) lef_rad = -0.0349;
  else if (gear_pos == 0.0 && alpha > 0.2618) lef_rad = 0.436;
  else if (gear_wow == 0.0 && alpha > 0.0873) lef_rad = 0.262;
  else if (mach > 0.9) lef_rad = -0.0349;
  o->dlef = lef_rad;                                                  /* fcs/lef-pos-rad */
  { static const double tim[2] = {3.0, 3.0};
    e->lef = kinematic(e->lef, lef_rad * 2.293578, d2, tim, 2, dt, ic); }
  /* -- Throttle (:859-867) -- */
  o->throttle = cmd_thr * 2.0;
  /* -- Speedbrake (:869-937) -- */
  double sb_lim = (alpha * RAD2DEG >= 53.0 && d->uvw[1] <= 18.0) ? 1.0 : 0.0;
  double sb_init = (sb_lim == 1.0 || 0.0 /* speedbrake-cmd-norm */ == 1.0) ? 1.0 : 0.0;
  double sb_sched = sb_init * tab1(&T_speedbrake_scheduler, 0.0 /* gear-cmd-norm */);
  { static const double det[2] = {0.0, 60.0}, tim[2] = {0.0, 1.0};
    e->sb = kinematic(e->sb, sb_sched * 60.0 /* scaled by last detent */, det, tim, 2, dt, ic); }
  o->dsb = e->sb / RAD2DEG;                                           /* speedbrake-pos-rad */
  /* Hook / Canopy (:939-982): inputs are 0 in flight -> inert. */
}

/* ------------------------------------------------------------------------------------------
 * FGTurbine (F100-PW-229.xml: milthrust 17800, maxthrust 29000, bpr 0.36, bleed 0.03,
 * idle N1/N2 30/60, max 100/100, augmented, augmethod 2), tpRun phase.
 * ---------------------------------------------------------------------------------------- */
static double seek(double v, double target, double accel, double decel, double dt) {
  if (v > target) { v -= dt * decel; if (v < target) v = target; }
  else if (v < target) { v += dt * accel; if (v > target) v = target; }
  return v;
}
double f16ref_seek(double v, double target, double accel, double decel, double dt) {
  return seek(v, target, accel, decel, dt);
}
static double engine_run(env_t* e, double throttle_pos, double mach, double h_rho, double sigma,
                         double dt, int ic) {
  const double milthrust = 17800.0, maxthrust = 29000.0, bleed = 0.03;
  const double idle_n1 = 30.0, idle_n2 = 60.0, n1f = 70.0, n2f = 40.0;
  const double delay = 90.0 / (0.36 + 3.0);
  double tp = throttle_pos, aug_cmd = 0.0;
  if (tp > 1.0) { aug_cmd = tp - 1.0; tp -= aug_cmd; }
  double idle = milthrust * tab2(&T_IdleThrust, mach, h_rho);
  double mil = (milthrust - idle) * tab2(&T_MilThrust, mach, h_rho);
  if (ic) {
    e->n2 = idle_n2 + tp * n2f;
    e->n1 = idle_n1 + tp * n1f;
    e->aug = aug_cmd > 0.0 ? 1.0 : 0.0;
  } else {
    double n2norm_prev = (e->n2 - idle_n2) / n2f;
    double nn = n2norm_prev + 0.1;
    if (nn > 1.0) nn = 1.0;
    double spool = delay / (1.0 + 3.0 * (1.0 - nn) * (1.0 - nn) * (1.0 - nn) + (1.0 - sigma));
    e->n2 = seek(e->n2, idle_n2 + tp * n2f, spool * 1.0, spool * 3.0, dt);
    e->n1 = seek(e->n1, idle_n1 + tp * n1f, spool * 1.0, spool * 2.4, dt);
  }
  double n2norm = (e->n2 - idle_n2) / n2f;
  double thrust = idle + mil * n2norm * n2norm;
  if (e->aug == 0.0) thrust *= (1.0 - bleed);
  if (aug_cmd > 0.0) {
    e->aug = 1.0;
    double tdiff = maxthrust * tab2(&T_AugThrust, mach, h_rho) - thrust;
    thrust += tdiff * aug_cmd;
  } else {
    e->aug = 0.0;
  }
  return thrust;
}

/* ------------------------------------------------------------------------------------------
 * one FGFDMExec::Run() frame
 *   Propagate -> Inertial -> Atmosphere -> Systems(FCS) -> MassBalance -> Auxiliary ->
 *   Propulsion -> Aerodynamics -> (Ground/External: none) -> Accelerations
 * ic != 0: evaluation without integration (RunIC).
 * ---------------------------------------------------------------------------------------- */
static void propagate_integrate(env_t* e, double dt) {
  /* rotational position: rect Euler with QExp (q <- q * exp(0.5 dt wI)) */
  double h[3] = {0.5 * dt * e->wI[0], 0.5 * dt * e->wI[1], 0.5 * dt * e->wI[2]};
  double ang = sqrt(h[0] * h[0] + h[1] * h[1] + h[2] * h[2]);
  double sa = ang > 0.0 ? sin(ang) / ang : 1.0, ca = cos(ang);
  double p[4] = {ca, h[0] * sa, h[1] * sa, h[2] * sa};
  const double* q = e->q;
  double n[4] = {q[0] * p[0] - q[1] * p[1] - q[2] * p[2] - q[3] * p[3],
                 q[0] * p[1] + q[1] * p[0] + q[2] * p[3] - q[3] * p[2],
                 q[0] * p[2] - q[1] * p[3] + q[2] * p[0] + q[3] * p[1],
                 q[0] * p[3] + q[1] * p[2] - q[2] * p[1] + q[3] * p[0]};
  /* rotational rate: rect Euler */
  for (int i = 0; i < 3; i++) e->wI[i] += dt * e->wId[i];
  /* translational position: AB3 over inertial velocity */
  for (int i = 0; i < 3; i++) {
    double v0 = e->vI[i];
    e->rI[i] += (1.0 / 12.0) * dt * (23.0 * v0 - 16.0 * e->vIh1[i] + 5.0 * e->vIh2[i]);
    e->vIh2[i] = e->vIh1[i];
    e->vIh1[i] = v0;
  }
  /* translational rate: AB2 over inertial acceleration */
  for (int i = 0; i < 3; i++) {
    e->vI[i] += dt * (1.5 * e->aI[i] - 0.5 * e->aIp[i]);
    e->aIp[i] = e->aI[i];
  }
  /* Earth position angle and quaternion normalisation */
  e->epa += OMEGA_E * dt;
  e->epa_c = cos(e->epa);
  e->epa_s = sin(e->epa);
  double nn = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2] + n[3] * n[3]);
  for (int i = 0; i < 4; i++) e->q[i] = n[i] / nn;
}

typedef struct { double thrust, F[3], M[3], qbar, vt; } frame_diag_t;

static void frame(env_t* e, double dt, int ic, frame_diag_t* diag) {
  derived_t d;
  if (!ic) propagate_integrate(e, dt);
  derive(e, &d);
  /* Inertial */
  double gE[3];
  gravity_j2(&d, gE);
  if (g_phys_mask & F16REF_PHYS_NO_GRAVITY) gE[0] = gE[1] = gE[2] = 0.0;
  /* Atmosphere (standard day: density altitude == geometric altitude) */
  double atm[4];
  f16ref_atmosphere(d.h_ft, atm);
  const double rho = atm[2], sos = atm[3], p_st = atm[1];
  const double sigma = rho / atm_rho_sl();
  /* Systems */
  fcs_out_t fc;
  fcs_run(e, &d, dt, ic, &fc);
  /* Auxiliary */
  double wb[3], wt[3] = {e->wind[0] + e->gust[0], e->wind[1] + e->gust[1], e->wind[2] + e->gust[2]};
  mv(d.Tl2b, wt, wb);
  double ua = d.uvw[0] - wb[0], va = d.uvw[1] - wb[1], wa = d.uvw[2] - wb[2];
  double vt = sqrt(ua * ua + va * va + wa * wa);
  double muw = ua * ua + wa * wa;
  double alpha = muw > 0.0 ? atan2(wa, ua) : 0.0;
  double beta = muw > 0.0 ? atan2(va, sqrt(muw)) : 0.0;
  double qbar = 0.5 * rho * vt * vt;
  double mach = vt / sos;
  double vc_kts = f16ref_vcas_kts(mach, p_st);
  double vg = sqrt(d.vned[0] * d.vned[0] + d.vned[1] * d.vned[1]);
  double paero = d.pqr[0], qaero = d.pqr[1], raero = d.pqr[2];
  double bi2vel = 0.0, ci2vel = 0.0;
  if (vt != 0.0) { bi2vel = B_W / (2.0 * vt); ci2vel = CBAR / (2.0 * vt); }
  /* pilot-station acceleration: vBodyAccel + PQRidot x eye + wI x (wI x eye) */
  double t1[3], t2[3], t3[3];
  cross(e->wId, K.eye, t1);
  cross(e->wI, K.eye, t2);
  cross(e->wI, t2, t3);
  double npy = (e->ba[1] + t1[1] + t3[1]) / K.gref;
  double npz = (e->ba[2] + t1[2] + t3[2]) / K.gref;
  /* h_b-mac-ft: (h_agl - (Tb2l * RPBody)_down) / b */
  double vmac[3];
  mv(d.Tb2l, K.rp, vmac);
  double hbmac = (d.h_ft - vmac[2]) / B_W;
  e->lx[F16L_ALPHA] = alpha; e->lx[F16L_BETA] = beta; e->lx[F16L_MACH] = mach;
  e->lx[F16L_VC_KTS] = vc_kts; e->lx[F16L_VG_FPS] = vg;
  e->lx[F16L_P_AERO] = paero; e->lx[F16L_Q_AERO] = qaero; e->lx[F16L_R_AERO] = raero;
  e->lx[F16L_NPY] = npy; e->lx[F16L_NPZ] = npz;
  /* Propulsion */
  double thrust = engine_run(e, fc.throttle, mach, d.h_ft, sigma, dt, ic);
  if (g_phys_mask & F16REF_PHYS_NO_THRUST) thrust = 0.0;
  /* Aerodynamics: data-driven products over the XML function list (f16.xml:986-1917) */
  double P[RP_COUNT];
  P[RP_aero_qbar_psf] = qbar; P[RP_metrics_Sw_sqft] = S_W; P[RP_metrics_bw_ft] = B_W;
  P[RP_metrics_cbarw_ft] = CBAR; P[RP_aero_alpha_rad] = alpha; P[RP_aero_beta_rad] = beta;
  P[RP_velocities_mach] = mach; P[RP_velocities_p_aero_rad_sec] = paero;
  P[RP_velocities_q_aero_rad_sec] = qaero; P[RP_velocities_r_aero_rad_sec] = raero;
  P[RP_aero_bi2vel] = bi2vel; P[RP_aero_ci2vel] = ci2vel;
  P[RP_aero_function_kCLge] = tab1(&T_kCLge, hbmac);
  P[RP_fcs_elevator_pos_rad] = fc.de; P[RP_fcs_aileron_pos_rad] = fc.da;
  P[RP_fcs_rudder_pos_rad] = fc.dr; P[RP_fcs_lef_pos_rad] = fc.dlef;
  P[RP_fcs_flaperon_mix_rad] = fc.flap_mix; P[RP_fcs_speedbrake_pos_rad] = fc.dsb;
  P[RP_gear_gear_pos_norm] = 0.0;
  double ax[6] = {0, 0, 0, 0, 0, 0};
  for (int k = 0; k < REF_N_AERO_FNS; k++) {
    const ref_aero_fn* f = &REF_AERO_FNS[k];
    double v = 1.0;
    for (int j = 0; j < f->nprops; j++) v *= P[f->props[j]];
    if (f->has_value) v *= f->value;
    else v *= tab2(f->table, P[f->tvar[0]], f->tvar[1] >= 0 ? P[f->tvar[1]] : 0.0);
    ax[f->axis] += v;
  }
  if (g_phys_mask & F16REF_PHYS_NO_AERO)
    for (int k = 0; k < 6; k++) ax[k] = 0.0;
  /* wind axes (D, Y, L) -> body: vFw = (-D, Y, -L), vForces = Tw2b * vFw */
  double ca = cos(alpha), sa = sin(alpha), cb = cos(beta), sb = sin(beta);
  double Fw[3] = {-ax[AX_DRAG], ax[AX_SIDE], -ax[AX_LIFT]};
  double F[3];
  F[0] = ca * cb * Fw[0] - ca * sb * Fw[1] - sa * Fw[2];
  F[1] = sb * Fw[0] + cb * Fw[1];
  F[2] = sa * cb * Fw[0] - sa * sb * Fw[1] + ca * Fw[2];
  double M[3] = {ax[AX_ROLL], ax[AX_PITCH], ax[AX_YAW]};
  double rxF[3];
  cross(K.rp, F, rxF);
  for (int i = 0; i < 3; i++) M[i] += rxF[i];
  /* thrust along body +x at the thruster (Engines/direct.xml, f16.xml:251-262) */
  double Ft[3] = {thrust, 0.0, 0.0}, Mt[3];
  cross(K.eng, Ft, Mt);
  for (int i = 0; i < 3; i++) { F[i] += Ft[i]; M[i] += Mt[i]; }
  /* Accelerations */
  for (int i = 0; i < 3; i++) e->ba[i] = F[i] / K.mass;
  double gb[3];
  mv(d.Tec2b, gE, gb);
  double acc_b[3] = {e->ba[0] + gb[0], e->ba[1] + gb[1], e->ba[2] + gb[2]};
  mv(d.Tb2i, acc_b, e->aI);
  double Jw[3], wxJw[3], rhs[3];
  mv(K.J, e->wI, Jw);
  cross(e->wI, Jw, wxJw);
  for (int i = 0; i < 3; i++) rhs[i] = M[i] - wxJw[i];
  mv(K.Jinv, rhs, e->wId);
  if (diag) {
    diag->thrust = thrust; diag->qbar = qbar; diag->vt = vt;
    for (int i = 0; i < 3; i++) { diag->F[i] = F[i]; diag->M[i] = M[i]; }
  }
}

/* ------------------------------------------------------------------------------------------
 * IC (FGFDMExec::RunIC + FGPropulsion::InitRunning(-1))
 * ---------------------------------------------------------------------------------------- */
static void apply_ic(env_t* e, const double* ic, double dt) {
  init_consts();
  double rE[3];
  f16ref_geodetic_to_ecef(ic[F16_IC_LAT_GEOD_RAD], ic[F16_IC_LON_RAD], ic[F16_IC_H_SL_FT], rE);
  e->epa = 0.0; e->epa_c = 1.0; e->epa_s = 0.0;
  for (int i = 0; i < 3; i++) e->rI[i] = rE[i];
  /* local frame at the IC location (geocentric lat, as FGLocation) */
  double rxy = sqrt(rE[0] * rE[0] + rE[1] * rE[1]), r = sqrt(rxy * rxy + rE[2] * rE[2]);
  double slat = rE[2] / r, clat = rxy / r;
  double slon = rxy == 0.0 ? 0.0 : rE[1] / rxy, clon = rxy == 0.0 ? 1.0 : rE[0] / rxy;
  double L[9] = {-clon * slat, -slon * slat, clat, -slon, clon, 0.0, -clon * clat, -slon * clat, -slat};
  double Tl2b[9], Ti2b[9];
  euler_T(ic[F16_IC_PHI_RAD], ic[F16_IC_THETA_RAD], ic[F16_IC_PSI_RAD], Tl2b);
  mm(Tl2b, L, Ti2b); /* Ti2ec == I at EPA 0 */
  mat_quat(Ti2b, e->q);
  double qn = sqrt(e->q[0] * e->q[0] + e->q[1] * e->q[1] + e->q[2] * e->q[2] + e->q[3] * e->q[3]);
  for (int i = 0; i < 4; i++) e->q[i] /= qn;
  quat_T(e->q, Ti2b);
  double uvw[3] = {ic[F16_IC_U_FPS], ic[F16_IC_V_FPS], ic[F16_IC_W_FPS]}, vb[3];
  mtv(Ti2b, uvw, vb);
  e->vI[0] = vb[0] - OMEGA_E * e->rI[1];
  e->vI[1] = vb[1] + OMEGA_E * e->rI[0];
  e->vI[2] = vb[2];
  double w[3] = {0, 0, OMEGA_E}, wb[3];
  mv(Ti2b, w, wb);
  e->wI[0] = ic[F16_IC_P_RPS] + wb[0];
  e->wI[1] = ic[F16_IC_Q_RPS] + wb[1];
  e->wI[2] = ic[F16_IC_R_RPS] + wb[2];
  for (int i = 0; i < 3; i++) { e->wId[i] = 0.0; e->ba[i] = 0.0; e->aI[i] = 0.0; e->aIp[i] = 0.0; }
  e->tef = e->ail = e->ele = e->rud = e->lef = e->sb = 0.0;
  e->pid_r_i = e->pid_r_p = e->pid_p_i = e->pid_p_p = e->pid_y_i = e->pid_y_p = 0.0;
  e->n1 = 30.0; e->n2 = 60.0; e->aug = 0.0;
  for (int i = 0; i < F16L_N; i++) e->lx[i] = 0.0;
  for (int i = 0; i < 4; i++) e->cmd[i] = ic[F16_IC_CMD_AIL + i];
  for (int i = 0; i < 3; i++) e->wind[i] = ic[F16_IC_WIND_N_FPS + i];
  /* three evaluation passes without integration (the FCS reads the previous pass's
   * auxiliary latch, whose n-pilot terms read the pass before's accelerations: three passes
   * make FCS -> forces -> accelerations -> n-pilot -> FCS consistent), then
   * InitializeDerivatives */
  frame(e, dt, 1, NULL);
  frame(e, dt, 1, NULL);
  frame(e, dt, 1, NULL);
  for (int i = 0; i < 3; i++) {
    e->vIh1[i] = e->vIh2[i] = e->vI[i];
    e->aIp[i] = e->aI[i];
  }
}

/* ------------------------------------------------------------------------------------------
 * env layer (jsbsim_gym.py)
 * ---------------------------------------------------------------------------------------- */
/* normalize_angle_mpi_pi (:60-78) applied to a float32 state element (numpy 1.26 scalar
 * semantics: the float32 value is promoted to float64 by `% (2*np.pi)`). */
static float norm_angle(float a) {
  if (isnan(a) || isinf(a)) return 0.0f;
  double x = fmod((double)a, 2.0 * PI);
  if (x < 0.0) x += 2.0 * PI; /* Python modulo has the sign of the divisor */
  if (x >= PI) x -= 2.0 * PI;
  if (x == 0.0) x = 0.0; /* Python's float % returns +0.0 */
  return (float)x;
}
/* _get_current_single_observation (:172-197) */
static void make_frame(const env_t* e, float* f) {
  derived_t d;
  derive(e, &d);
  float s[12];
  s[0] = (float)d.lat_gc; s[1] = (float)d.lon; s[2] = (float)(d.h_ft * FT2M);
  s[3] = (float)e->lx[F16L_MACH]; s[4] = (float)e->lx[F16L_ALPHA]; s[5] = (float)e->lx[F16L_BETA];
  s[6] = (float)d.pqr[0]; s[7] = (float)d.pqr[1]; s[8] = (float)d.pqr[2];
  s[9] = (float)d.eul[0]; s[10] = (float)d.eul[1]; s[11] = (float)d.eul[2];
  s[9] = norm_angle(s[9]); s[10] = norm_angle(s[10]); s[11] = norm_angle(s[11]);
  s[0] = (float)((double)s[0] * RADIUS_M);
  s[1] = (float)((double)s[1] * RADIUS_M);
  for (int i = 0; i < 12; i++) f[i] = s[i];
  f[12] = e->goal[0]; f[13] = e->goal[1]; f[14] = e->goal[2];
}
/* np.linalg.norm over a float32 3-vector, fixed sequential float32 order */
static float norm3f(float a, float b, float c) {
  volatile float s = a * a;
  s = s + b * b;
  s = s + c * c;
  return sqrtf(s);
}

/* Philox4x32-10 */
void f16ref_philox4x32(const uint32_t key[2], const uint32_t ctr[4], uint32_t out[4]) {
  uint32_t k0 = key[0], k1 = key[1];
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  for (int r = 0; r < 10; r++) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
static double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}
/* device goal RNG: jsbsim_gym.py:312-323 formula, Philox stream keyed by
 * (seed; global env id, episode count, purpose=0x474F414C 'GOAL') */
static void rng_goal(uint64_t seed, uint64_t gid, uint64_t ep, float* g) {
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t ctr[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)ep, 0x474F414Cu};
  uint32_t o[4], o2[4];
  f16ref_philox4x32(key, ctr, o);
  ctr[3] ^= 0x1u;
  f16ref_philox4x32(key, ctr, o2);
  double dist = 1000.0 + (10000.0 - 1000.0) * u53(o[0], o[1]);
  double bear = 0.0 + (2.0 * PI - 0.0) * u53(o[2], o[3]);
  double alt = 1000.0 + (4000.0 - 1000.0) * u53(o2[0], o2[1]);
  g[0] = (float)(dist * cos(bear));
  g[1] = (float)(dist * sin(bear));
  g[2] = (float)alt;
}

/* cfg5 random IC (include/f16env.h F16_FLAG_RANDOM_IC): component j uniform in
 * [lo_j, hi_j] from word j%4 of Philox (seed; gid, gid_hi, ep, 'RIC'+j/4) */
static void rng_ic(uint64_t seed, uint64_t gid, uint64_t ep, const double* lo, const double* hi, double* ic) {
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t o[4];
  for (int j = 0; j < F16_IC_N; j++) {
    if ((j & 3) == 0) {
      uint32_t ctr[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)ep, 0x52494300u + (uint32_t)(j >> 2)};
      f16ref_philox4x32(key, ctr, o);
    }
    double u = ((double)o[j & 3] + 0.5) * (1.0 / 4294967296.0);
    ic[j] = lo[j] + (hi[j] - lo[j]) * u;
  }
}
/* cfg5 gust noise: three Box-Muller normals from Philox (seed; gid, gid_hi ^ 'GUST', ep, s) */
static void rng_normals(uint64_t seed, uint64_t gid, uint64_t ep, uint32_t s, double* xi) {
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t ctr[4] = {(uint32_t)gid, (uint32_t)(gid >> 32) ^ 0x47555354u, (uint32_t)ep, s};
  uint32_t o[4];
  f16ref_philox4x32(key, ctr, o);
  const double s24 = 1.0 / 16777216.0;
  double u1 = ((double)(o[0] >> 8) + 0.5) * s24, u2 = (double)(o[1] >> 8) * s24;
  double u3 = ((double)(o[2] >> 8) + 0.5) * s24, u4 = (double)(o[3] >> 8) * s24;
  double r1 = sqrt(-2.0 * log(u1)), r2 = sqrt(-2.0 * log(u3));
  xi[0] = r1 * cos(2.0 * PI * u2);
  xi[1] = r1 * sin(2.0 * PI * u2);
  xi[2] = r2 * cos(2.0 * PI * u4);
}
static void gust_coeffs(const f16env_config* c, double* a, double* b) {
  *a = c->gust_tau_s > 0.0 ? exp(-(double)c->down_sample * c->dt / c->gust_tau_s) : 0.0;
  *b = c->gust_sigma_fps * sqrt(1.0 - *a * *a);
}

static void env_reset(f16ref* h, int i, const float* goal, const double* ic) {
  env_t* e = &h->env[i];
  const uint64_t gid = (uint64_t)(h->cfg.env_id_base + i);
  double ric[F16_IC_N];
  if (!ic && (h->cfg.flags & F16_FLAG_RANDOM_IC)) {
    rng_ic(h->cfg.seed, gid, e->ep_count, h->cfg.ic_lo, h->cfg.ic_hi, ric);
    ic = ric;
  }
  if (h->cfg.flags & F16_FLAG_GUSTS) { /* stationary start g_0 = sigma xi_0 */
    double xi[3];
    rng_normals(h->cfg.seed, gid, e->ep_count, 0u, xi);
    for (int k = 0; k < 3; k++) e->gust[k] = h->cfg.gust_sigma_fps * xi[k];
  } else {
    e->gust[0] = e->gust[1] = e->gust[2] = 0.0;
  }
  apply_ic(e, ic ? ic : h->cfg.ic, h->cfg.dt);
  if (goal) { e->goal[0] = goal[0]; e->goal[1] = goal[1]; e->goal[2] = goal[2]; }
  else rng_goal(h->cfg.seed, gid, e->ep_count, e->goal);
  e->ep_count += 1;
  e->step = 0;
  e->ep_ret = 0.0;
  float f[F16_OBS_DIM];
  make_frame(e, f);
  const int K_ = h->cfg.stack_k;
  for (int k = 0; k < K_; k++) memcpy(e->stack + k * F16_OBS_DIM, f, sizeof f);
  e->head = 0;
  float dx = f[12] - f[0], dy = f[13] - f[1], dz = f[14] - f[2];
  e->last_d = norm3f(dx, dy, (g_phys_mask & F16REF_TEST_SHAPING_2D) ? 0.0f : dz);
}
static void write_stack(const f16ref* h, const env_t* e, float* out) {
  const int K_ = h->cfg.stack_k;
  for (int k = 0; k < K_; k++) {
    int slot = (e->head + k) % K_;
    memcpy(out + k * F16_OBS_DIM, e->stack + slot * F16_OBS_DIM, F16_OBS_DIM * sizeof(float));
  }
}

f16ref* f16ref_create(const f16env_config* cfg) {
  init_consts();
  { double o[4]; f16ref_atmosphere(0.0, o); (void)atm_rho_sl(); (void)atm_a_sl(); }
  f16ref* h = (f16ref*)calloc(1, sizeof(f16ref));
  h->cfg = *cfg;
  h->n = cfg->n_envs;
  h->env = (env_t*)calloc((size_t)h->n, sizeof(env_t));
  h->stacks = (float*)calloc((size_t)h->n * cfg->stack_k * F16_OBS_DIM, sizeof(float));
  for (int i = 0; i < h->n; i++) h->env[i].stack = h->stacks + (size_t)i * cfg->stack_k * F16_OBS_DIM;
  return h;
}
void f16ref_destroy(f16ref* h) {
  if (!h) return;
  free(h->env); free(h->stacks); free(h);
}
int f16ref_n_envs(const f16ref* h) { return h->n; }
uint64_t f16ref_obs_bounds_count(const f16ref* h) { return h->obs_oob; }
int f16ref_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
/* thread count of the following parallel loops (bench.py's CPU-baseline core scaling); n <= 0
 * restores the OMP_NUM_THREADS default */
int f16ref_set_threads(int n) {
#ifdef _OPENMP
  static int dflt = 0;
  if (!dflt) dflt = omp_get_max_threads();
  omp_set_num_threads(n > 0 ? n : dflt);
  return omp_get_max_threads();
#else
  (void)n;
  return 1;
#endif
}

int f16ref_reset(f16ref* h, const uint8_t* mask, const float* goals, const double* ic, float* obs) {
  const int KO = h->cfg.stack_k * F16_OBS_DIM;
#pragma omp parallel for schedule(static)
  for (int i = 0; i < h->n; i++) {
    if (mask && !mask[i]) continue;
    const float* g = goals ? goals + 3 * i : NULL;
    if (g && isnan(g[0])) g = NULL; /* NaN row: device-stream goal (include/f16env.h) */
    env_reset(h, i, g, ic ? ic + (size_t)F16_IC_N * i : NULL);
    if (obs) write_stack(h, &h->env[i], obs + (size_t)KO * i);
  }
  return 0;
}

int f16ref_step(f16ref* h, const float* act, float* obs, float* rew, uint8_t* term,
                uint8_t* trunc, float* terminal_obs, double* ep_ret, int32_t* ep_len) {
  const int KO = h->cfg.stack_k * F16_OBS_DIM, K_ = h->cfg.stack_k;
  const double dt = h->cfg.dt;
  const float dg = (float)h->cfg.dg_m, crash = (float)h->cfg.crash_alt_m;
#pragma omp parallel for schedule(dynamic, 64)
  for (int i = 0; i < h->n; i++) {
    env_t* e = &h->env[i];
    e->step += 1;                                                   /* :215 */
    for (int j = 0; j < 4; j++) e->cmd[j] = (double)act[4 * i + j]; /* :219-222 */
    if (h->cfg.flags & F16_FLAG_GUSTS) {                            /* cfg5 gust update */
      double xi[3], ga, gb;
      gust_coeffs(&h->cfg, &ga, &gb);
      rng_normals(h->cfg.seed, (uint64_t)(h->cfg.env_id_base + i), e->ep_count - 1, (uint32_t)e->step, xi);
      for (int k = 0; k < 3; k++) e->gust[k] = ga * e->gust[k] + gb * xi[k];
    }
    for (int s = 0; s < h->cfg.down_sample; s++) frame(e, dt, 0, NULL); /* :225-232 */
    float f[F16_OBS_DIM];
    make_frame(e, f);                                               /* :234 */
    memcpy(e->stack + e->head * F16_OBS_DIM, f, sizeof f);          /* :235 deque append */
    e->head = (e->head + 1) % K_;
    /* F16_FLAG_NAN_GUARD (build-defined, include/f16env.h): a non-finite position, Mach,
       alpha, beta or body rate ends the step terminated (term = 3) with reward 0 */
    int bad = 0;
    if (h->cfg.flags & F16_FLAG_NAN_GUARD)
      for (int j = 0; j < 9; j++) bad |= !isfinite(f[j]);
    if ((h->cfg.flags & F16_FLAG_OBS_CHECK) && obs_out_of_bounds(f)) {
#pragma omp atomic
      h->obs_oob++;
    }
    double r = 0.0;
    int te = 0, tr = 0;
    if (bad) {
      te = 3;
    } else {
      /* reward / termination (:237-261), float32 arithmetic on the frame */
      float alt = f[2];
      if (alt < crash) { r = -10.0; te = 1; }
      float dx = f[0] - f[12], dy = f[1] - f[13];
      volatile float d2 = dx * dx;
      d2 = d2 + dy * dy;
      float dalt = alt - f[14];
      if (!te && sqrtf(d2) < dg && fabsf(dalt) < dg) { r = 10.0; te = 1; }
      tr = e->step >= h->cfg.max_steps; /* env :260 OR gymnasium TimeLimit(1200) */
      /* PositionReward (:493-507) */
      float gx = f[12] - f[0], gy = f[13] - f[1], gz = f[14] - f[2];
      /* (F16REF_TEST_SHAPING_2D: the negative control of the reward parity tests) */
      float dcur = norm3f(gx, gy, (g_phys_mask & F16REF_TEST_SHAPING_2D) ? 0.0f : gz);
      float ddiff = e->last_d - dcur;
      r += h->cfg.goal_gain * (double)ddiff;
      e->last_d = dcur;
      e->ep_ret += r;                                               /* Monitor :96-99 */
    }
    rew[i] = (float)r;
    term[i] = (uint8_t)te;
    trunc[i] = (uint8_t)tr;
    float* o = obs + (size_t)KO * i;
    write_stack(h, e, o);                                           /* :263 */
    if (te || tr) {
      if (ep_ret) ep_ret[i] = e->ep_ret;
      if (ep_len) ep_len[i] = e->step;
      if (terminal_obs) memcpy(terminal_obs + (size_t)KO * i, o, KO * sizeof(float));
      if (!(h->cfg.flags & F16_FLAG_NO_AUTORESET)) {                /* dummy_vec_env.py:68-71 */
        env_reset(h, i, NULL, NULL);
        write_stack(h, e, o);
      }
    }
  }
  return 0;
}

int f16ref_get_state(const f16ref* h, double* c) {
  for (int i = 0; i < h->n; i++) {
    const env_t* e = &h->env[i];
    double* s = c + (size_t)F16C_N * i;
    for (int k = 0; k < 3; k++) {
      s[F16C_RI + k] = e->rI[k]; s[F16C_VI + k] = e->vI[k]; s[F16C_VIH1 + k] = e->vIh1[k];
      s[F16C_VIH2 + k] = e->vIh2[k]; s[F16C_AI + k] = e->aI[k]; s[F16C_AIP + k] = e->aIp[k];
      s[F16C_WI + k] = e->wI[k]; s[F16C_WID + k] = e->wId[k]; s[F16C_BA + k] = e->ba[k];
      s[F16C_GOAL + k] = e->goal[k]; s[F16C_WIND + k] = e->wind[k]; s[F16C_GUST + k] = e->gust[k];
    }
    for (int k = 0; k < 4; k++) { s[F16C_Q + k] = e->q[k]; s[F16C_CMD + k] = e->cmd[k]; }
    s[F16C_EPA_C] = e->epa_c; s[F16C_EPA_S] = e->epa_s;
    s[F16C_TEF] = e->tef; s[F16C_AIL] = e->ail; s[F16C_ELE] = e->ele; s[F16C_RUD] = e->rud;
    s[F16C_LEF] = e->lef; s[F16C_SB] = e->sb;
    s[F16C_PID_R_I] = e->pid_r_i; s[F16C_PID_R_P] = e->pid_r_p;
    s[F16C_PID_P_I] = e->pid_p_i; s[F16C_PID_P_P] = e->pid_p_p;
    s[F16C_PID_Y_I] = e->pid_y_i; s[F16C_PID_Y_P] = e->pid_y_p;
    s[F16C_N1] = e->n1; s[F16C_N2] = e->n2; s[F16C_AUG] = e->aug;
    for (int k = 0; k < F16L_N; k++) s[F16C_LX + k] = e->lx[k];
    s[F16C_LAST_D] = e->last_d; s[F16C_STEP] = e->step; s[F16C_EP_RET] = e->ep_ret;
    s[F16C_EP_COUNT] = (double)e->ep_count;
  }
  return 0;
}
int f16ref_set_state(f16ref* h, const double* c) {
  for (int i = 0; i < h->n; i++) {
    env_t* e = &h->env[i];
    const double* s = c + (size_t)F16C_N * i;
    for (int k = 0; k < 3; k++) {
      e->rI[k] = s[F16C_RI + k]; e->vI[k] = s[F16C_VI + k]; e->vIh1[k] = s[F16C_VIH1 + k];
      e->vIh2[k] = s[F16C_VIH2 + k]; e->aI[k] = s[F16C_AI + k]; e->aIp[k] = s[F16C_AIP + k];
      e->wI[k] = s[F16C_WI + k]; e->wId[k] = s[F16C_WID + k]; e->ba[k] = s[F16C_BA + k];
      e->goal[k] = (float)s[F16C_GOAL + k]; e->wind[k] = s[F16C_WIND + k]; e->gust[k] = s[F16C_GUST + k];
    }
    for (int k = 0; k < 4; k++) { e->q[k] = s[F16C_Q + k]; e->cmd[k] = s[F16C_CMD + k]; }
    e->epa_c = s[F16C_EPA_C]; e->epa_s = s[F16C_EPA_S];
    e->epa = atan2(e->epa_s, e->epa_c);
    e->tef = s[F16C_TEF]; e->ail = s[F16C_AIL]; e->ele = s[F16C_ELE]; e->rud = s[F16C_RUD];
    e->lef = s[F16C_LEF]; e->sb = s[F16C_SB];
    e->pid_r_i = s[F16C_PID_R_I]; e->pid_r_p = s[F16C_PID_R_P];
    e->pid_p_i = s[F16C_PID_P_I]; e->pid_p_p = s[F16C_PID_P_P];
    e->pid_y_i = s[F16C_PID_Y_I]; e->pid_y_p = s[F16C_PID_Y_P];
    e->n1 = s[F16C_N1]; e->n2 = s[F16C_N2]; e->aug = s[F16C_AUG];
    for (int k = 0; k < F16L_N; k++) e->lx[k] = s[F16C_LX + k];
    e->last_d = (float)s[F16C_LAST_D]; e->step = (int32_t)s[F16C_STEP]; e->ep_ret = s[F16C_EP_RET];
    e->ep_count = (uint64_t)s[F16C_EP_COUNT];
  }
  return 0;
}

/* ------------------------------------------------------------------------------------------
 * Trim (BASELINE cfg 2; the reference never trims -- jsbsim_gym.py:166-170,305-306).
 * Steady wings-level flight at (h, Vt): unknowns x = (alpha, elevator cmd, throttle cmd),
 * residuals = (udot, wdot) of the body-axis velocity wrt the local frame and qdot, from the
 * RunIC evaluation. Newton with forward-difference Jacobian, fixed 12 iterations.
 * ---------------------------------------------------------------------------------------- */
static void trim_residual(const double* icb, const double* x, double dt, double* res) {
  env_t e;
  memset(&e, 0, sizeof e);
  double ic[F16_IC_N];
  memcpy(ic, icb, sizeof ic);
  double vt = icb[F16_IC_U_FPS];
  ic[F16_IC_U_FPS] = vt * cos(x[0]);
  ic[F16_IC_V_FPS] = 0.0;
  ic[F16_IC_W_FPS] = vt * sin(x[0]);
  ic[F16_IC_THETA_RAD] = x[0];
  ic[F16_IC_PHI_RAD] = 0.0;
  ic[F16_IC_P_RPS] = ic[F16_IC_Q_RPS] = ic[F16_IC_R_RPS] = 0.0;
  ic[F16_IC_CMD_AIL] = 0.0; ic[F16_IC_CMD_RUD] = 0.0;
  ic[F16_IC_CMD_ELE] = x[1];
  ic[F16_IC_CMD_THR] = x[2];
  apply_ic(&e, ic, dt);
  /* FGAccelerations::CalculateUVWdot (body velocity wrt ECEF): specific force + gravity
   * - (pqr + 2 w_b) x uvw - Ti2b (w x (w x rI)) */
  derived_t d;
  derive(&e, &d);
  double gE[3], gb[3];
  gravity_j2(&d, gE);
  mv(d.Tec2b, gE, gb);
  double w[3] = {0, 0, OMEGA_E}, wb[3], c1[3], t[3], wxr[3], wxwxr[3], cent[3];
  mv(d.Ti2b, w, wb);
  for (int i = 0; i < 3; i++) t[i] = d.pqr[i] + 2.0 * wb[i];
  cross(t, d.uvw, c1);
  cross(w, e.rI, wxr);
  cross(w, wxr, wxwxr);
  mv(d.Ti2b, wxwxr, cent);
  res[0] = e.ba[0] + gb[0] - c1[0] - cent[0];
  res[1] = e.ba[2] + gb[2] - c1[2] - cent[2];
  res[2] = e.wId[1];
}
static void trim_one(const double* icb, double dt, double* ic_out, double* resid) {
  double x[3] = {0.05, 0.0, 0.5};
  const double hstep[3] = {1e-5, 1e-5, 1e-5};
  double r[3];
  for (int it = 0; it < 12; it++) {
    trim_residual(icb, x, dt, r);
    double Jm[9], Ji[9];
    for (int j = 0; j < 3; j++) {
      double xp[3] = {x[0], x[1], x[2]}, rp[3];
      xp[j] += hstep[j];
      trim_residual(icb, xp, dt, rp);
      for (int i = 0; i < 3; i++) Jm[3 * i + j] = (rp[i] - r[i]) / hstep[j];
    }
    if (inv3(Jm, Ji) != 0) break;
    double dx[3];
    mv(Ji, r, dx);
    for (int i = 0; i < 3; i++) x[i] -= dx[i];
    x[0] = clip(x[0], -0.3, 0.6);
    x[1] = clip(x[1], -1.0, 0.44);
    x[2] = clip(x[2], 0.0, 1.0);
  }
  trim_residual(icb, x, dt, r);
  memcpy(ic_out, icb, F16_IC_N * sizeof(double));
  double vt = icb[F16_IC_U_FPS];
  ic_out[F16_IC_U_FPS] = vt * cos(x[0]);
  ic_out[F16_IC_V_FPS] = 0.0;
  ic_out[F16_IC_W_FPS] = vt * sin(x[0]);
  ic_out[F16_IC_THETA_RAD] = x[0];
  ic_out[F16_IC_PHI_RAD] = 0.0;
  ic_out[F16_IC_P_RPS] = ic_out[F16_IC_Q_RPS] = ic_out[F16_IC_R_RPS] = 0.0;
  ic_out[F16_IC_CMD_AIL] = 0.0; ic_out[F16_IC_CMD_RUD] = 0.0;
  ic_out[F16_IC_CMD_ELE] = x[1];
  ic_out[F16_IC_CMD_THR] = x[2];
  if (resid) for (int i = 0; i < 3; i++) resid[i] = fabs(r[i]);
}
int f16ref_trim(f16ref* h, const double* ic_in, double* ic_out, double* residual_out) {
#pragma omp parallel for schedule(dynamic, 16)
  for (int i = 0; i < h->n; i++)
    trim_one(ic_in + (size_t)F16_IC_N * i, h->cfg.dt, ic_out + (size_t)F16_IC_N * i,
             residual_out ? residual_out + 3 * i : NULL);
  return 0;
}

int f16ref_sample_actions(const f16ref* h, uint64_t seed, uint64_t step, float* act) {
  static const float lo[4] = {-1.f, -1.f, -1.f, 0.f}, hi[4] = {1.f, 1.f, 1.f, 1.f};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  for (int i = 0; i < h->n; i++) {
    uint64_t gid = (uint64_t)(h->cfg.env_id_base + i);
    uint32_t ctr[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)step, (uint32_t)(step >> 32)};
    uint32_t o[4];
    f16ref_philox4x32(key, ctr, o);
    for (int j = 0; j < 4; j++) {
      float u = (float)(o[j] >> 8) * (1.0f / 16777216.0f);
      act[4 * i + j] = lo[j] + (hi[j] - lo[j]) * u;
    }
  }
  return 0;
}

double f16ref_aero_table(int k, double x, double y) {
  const ref_aero_fn* f = &REF_AERO_FNS[k];
  if (f->has_value) return f->value;
  return tab2(f->table, x, y);
}
int f16ref_n_aero_fns(void) { return REF_N_AERO_FNS; }
