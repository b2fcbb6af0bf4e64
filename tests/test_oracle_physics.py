"""The oracle's equations of motion and FCS components against analytic invariants that do not
depend on JSBSim (VERDICT r01 missing #4). JSBSim itself is absent, so these bound the
oracle's own error instead of pinning it to JSBSim:

  * torque-free rigid body (aero, thrust and gravity off through the oracle's test-only physics
    mask): inertial velocity constant and position linear exactly; inertial angular momentum and
    rotational energy conserved to the order of JSBSim's default rotational integrator
    (rectangular Euler: the drift halves when dt halves);
  * gravity-only vacuum flight (central gravity): 40 s against the closed-form Kepler solution
    (universal variables), second-order convergence of the AB2/AB3 translational integrators;
    with J2, against an RK4 reference integration of the same field;
  * FCS / engine components against their documented behaviour: FGKinematic traverse and
    detent clamping, FGPID trigger semantics, zero-centred aerosurface_scale, FGTurbine Seek.
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from f16_jsb_amd.abi import F16C_Q, F16C_RI, F16C_VI, F16C_WI, F16_FLAG_NO_AUTORESET
from oracle_ref import OracleEnvs, default_ic, lib

NO_AERO, NO_THRUST, NO_GRAVITY, NO_J2 = 0x1, 0x2, 0x4, 0x8
GM = 14.0764417572e15          # ft^3/s^2 (FGInertial)
WGS_A, J2 = 20925646.32546, 1.08262982e-03


@pytest.fixture
def physics_mask(oracle_lib):
    def set_mask(m):
        oracle_lib.f16ref_set_physics_mask(int(m))
    yield set_mask
    oracle_lib.f16ref_set_physics_mask(0)


def _quat_T(q):
    q0, q1, q2, q3 = q
    return np.array([
        [q0 * q0 + q1 * q1 - q2 * q2 - q3 * q3, 2 * (q1 * q2 + q0 * q3), 2 * (q1 * q3 - q0 * q2)],
        [2 * (q1 * q2 - q0 * q3), q0 * q0 - q1 * q1 + q2 * q2 - q3 * q3, 2 * (q2 * q3 + q0 * q1)],
        [2 * (q1 * q3 + q0 * q2), 2 * (q2 * q3 - q0 * q1), q0 * q0 - q1 * q1 - q2 * q2 + q3 * q3]])


def _run(ic, dt, seconds, down_sample=4, record=None):
    """One env on the oracle, zero actions, crash / truncation disabled; returns states."""
    steps = int(round(seconds / (dt * down_sample)))
    e = OracleEnvs(1, stack_k=1, dt=dt, down_sample=down_sample, max_steps=10**9, crash_alt_m=-1e12,
                   flags=F16_FLAG_NO_AUTORESET)
    e.reset(goals=np.zeros((1, 3), np.float32), ic=ic[None])
    out = [e.get_state()[0].copy()]
    a = np.zeros((1, 4), np.float32)
    for t in range(steps):
        e.step(a)
        if record is None or (t + 1) % record == 0:
            out.append(e.get_state()[0].copy())
    e.close()
    return np.array(out)


def _torque_free(dt, seconds=10.0):
    ic = default_ic()
    ic[6], ic[7], ic[8] = 0.3, -0.2, 1.0        # phi theta psi
    ic[9], ic[10], ic[11] = 0.6, -0.4, 0.3      # p q r (rad/s): tumbling, ixz couples roll / yaw
    ds = int(round(4 * (1 / 120) / dt))
    return _run(ic, dt, seconds, down_sample=ds)


def _rot_invariants(S, J):
    H = []
    E = []
    for s in S:
        w = s[F16C_WI:F16C_WI + 3]
        Ti2b = _quat_T(s[F16C_Q:F16C_Q + 4])
        H.append(Ti2b.T @ (J @ w))
        E.append(0.5 * w @ J @ w)
    return np.array(H), np.array(E)


def test_torque_free_rigid_body(physics_mask, oracle_lib):
    physics_mask(NO_AERO | NO_THRUST | NO_GRAVITY)
    J = np.zeros(9)
    m = ctypes.c_double()
    oracle_lib.f16ref_mass_props(J.ctypes.data_as(ctypes.c_void_p), ctypes.byref(m))
    J = J.reshape(3, 3)
    drift = {}
    for dt in (1 / 120, 1 / 240):
        S = _torque_free(dt)
        # no force: the inertial velocity is constant and the position linear, exactly
        v = S[:, F16C_VI:F16C_VI + 3]
        assert np.abs(v - v[0]).max() == 0.0
        t = np.arange(len(S)) * 4 / 120
        r_lin = S[0, F16C_RI:F16C_RI + 3] + t[:, None] * v[0]
        assert np.abs(S[:, F16C_RI:F16C_RI + 3] - r_lin).max() < 1e-6 * np.abs(r_lin).max()
        H, E = _rot_invariants(S, J)
        dh = np.abs(np.linalg.norm(H - H[0], axis=1)).max() / np.linalg.norm(H[0])
        de = np.abs(E - E[0]).max() / E[0]
        drift[dt] = (dh, de)
        # the body rates really move (a tumbling, not a steady, rotation)
        w = S[:, F16C_WI:F16C_WI + 3]
        assert np.abs(w - w[0]).max() > 0.05
    (h1, e1), (h2, e2) = drift[1 / 120], drift[1 / 240]
    # first-order (rectangular Euler) drift: small, and halved with the step
    assert h1 < 2e-2 and e1 < 2e-2, drift
    assert 1.6 < h1 / h2 < 2.5 and 1.6 < e1 / e2 < 2.5, drift


def _stumpff(z):
    if z > 1e-8:
        s = np.sqrt(z)
        return (1 - np.cos(s)) / z, (s - np.sin(s)) / s ** 3
    if z < -1e-8:
        s = np.sqrt(-z)
        return (np.cosh(s) - 1) / -z, (np.sinh(s) - s) / s ** 3
    return 0.5 - z / 24 + z * z / 720, 1 / 6 - z / 120 + z * z / 5040


def kepler(r0, v0, t, mu=GM):
    """Closed-form two-body propagation (universal variables, Newton on chi)."""
    r0n = np.linalg.norm(r0)
    vr0 = r0 @ v0 / r0n
    alpha = 2 / r0n - v0 @ v0 / mu
    smu = np.sqrt(mu)
    chi = smu * abs(alpha) * t
    for _ in range(50):
        z = alpha * chi * chi
        C, S = _stumpff(z)
        F = r0n * vr0 / smu * chi * chi * C + (1 - alpha * r0n) * chi ** 3 * S + r0n * chi - smu * t
        dF = r0n * vr0 / smu * chi * (1 - z * S) + (1 - alpha * r0n) * chi * chi * C + r0n
        d = F / dF
        chi -= d
        if abs(d) < 1e-12:
            break
    z = alpha * chi * chi
    C, S = _stumpff(z)
    f = 1 - chi * chi / r0n * C
    g = t - chi ** 3 * S / smu
    return f * r0 + g * v0


def _vacuum_ic(lat=0.0):
    ic = default_ic()
    ic[0] = lat
    ic[2] = 40000.0   # ft: 40 s of free fall stays above the ellipsoid
    ic[3] = 900.0
    ic[7] = 0.1       # climbing a little
    return ic


def test_gravity_only_vacuum_matches_kepler(physics_mask):
    physics_mask(NO_AERO | NO_THRUST | NO_J2)
    err = {}
    for dt in (1 / 120, 1 / 240):
        ds = int(round(4 * (1 / 120) / dt))
        S = _run(_vacuum_ic(), dt, 40.0, down_sample=ds)
        r0, v0 = S[0, F16C_RI:F16C_RI + 3], S[0, F16C_VI:F16C_VI + 3]
        r40 = S[-1, F16C_RI:F16C_RI + 3]
        err[dt] = np.linalg.norm(r40 - kepler(r0, v0, 40.0))
        fall = np.linalg.norm(r0) - np.linalg.norm(r40)
        assert fall > 15000.0  # it really fell (~0.5 g t^2 against the climb)
    # second order (AB2 velocity / AB3 position with the constant-history start)
    assert err[1 / 120] < 1e-3, err  # measured 1.9e-4 ft after 40 s
    assert 3.0 < err[1 / 120] / err[1 / 240] < 5.0, err


def _rk4_j2(r, v, t, h):
    def acc(x):
        rn = np.linalg.norm(x)
        sl = x[2] / rn
        pre = 1.5 * J2 * (WGS_A / rn) ** 2
        gm = GM / rn ** 2
        return -gm * np.array([(1 + pre * (1 - 5 * sl * sl)) * x[0] / rn, (1 + pre * (1 - 5 * sl * sl)) * x[1] / rn,
                               (1 + pre * (3 - 5 * sl * sl)) * x[2] / rn])
    for _ in range(int(round(t / h))):
        k1r, k1v = v, acc(r)
        k2r, k2v = v + 0.5 * h * k1v, acc(r + 0.5 * h * k1r)
        k3r, k3v = v + 0.5 * h * k2v, acc(r + 0.5 * h * k2r)
        k4r, k4v = v + h * k3v, acc(r + h * k3r)
        r = r + h / 6 * (k1r + 2 * k2r + 2 * k3r + k4r)
        v = v + h / 6 * (k1v + 2 * k2v + 2 * k3v + k4v)
    return r


def test_gravity_j2_vacuum_matches_rk4(physics_mask):
    physics_mask(NO_AERO | NO_THRUST)
    S = _run(_vacuum_ic(lat=0.6), 1 / 120, 40.0, record=300)
    r0, v0 = S[0, F16C_RI:F16C_RI + 3], S[0, F16C_VI:F16C_VI + 3]
    ref = _rk4_j2(r0, v0, 40.0, 1 / 480)
    assert np.linalg.norm(S[-1, F16C_RI:F16C_RI + 3] - ref) < 1e-3  # measured 1.9e-4 ft
    # and J2 matters at this latitude: the central-field answer is far off
    assert np.linalg.norm(kepler(r0, v0, 40.0) - ref) > 1.0


def _kin(oracle_lib, out, inp, det, tim, dt, ic=0):
    d = np.asarray(det, np.float64)
    t = np.asarray(tim, np.float64)
    return oracle_lib.f16ref_kinematic(out, inp, d.ctypes.data_as(ctypes.c_void_p), t.ctypes.data_as(ctypes.c_void_p),
                                       len(d), dt, ic)


def test_fgkinematic_traverse(oracle_lib):
    """FGKinematic (f16.xml elevator actuator :630-643: detents -1 / 1, 0.3 s full travel):
    output moves toward the clamped input at (d1 - d0) / t per second, never overshoots, lands
    on it exactly; trim mode (RunIC) jumps; inputs beyond the detents clamp."""
    det, tim, dt = [-1.0, 1.0], [0.0, 0.3], 1 / 120
    rate = 2.0 / 0.3
    out = 0.0
    seq = []
    for _ in range(40):
        out = _kin(oracle_lib, out, 5.0, det, tim, dt)
        seq.append(out)
    seq = np.array(seq)
    n_full = int(np.floor(1.0 / (rate * dt)))
    np.testing.assert_allclose(seq[:n_full], rate * dt * np.arange(1, n_full + 1), rtol=1e-12)
    assert seq.max() == 1.0 and np.all(np.diff(seq) >= 0) and seq[-1] == 1.0
    assert _kin(oracle_lib, 0.2, -3.0, det, tim, dt, ic=1) == -1.0
    # TEF (f16.xml:334-350): detents -1 / 0 / 1, times 3 / 0 / 3 -- the segment into 0 from -1
    # is instantaneous, 0 -> 1 takes 3 s
    det3, tim3 = [-1.0, 0.0, 1.0], [3.0, 0.0, 3.0]
    assert _kin(oracle_lib, -1.0, 0.0, det3, tim3, dt) == 0.0
    o = 0.0
    for _ in range(180):  # 1.5 s of a 3 s traverse
        o = _kin(oracle_lib, o, 1.0, det3, tim3, dt)
    assert abs(o - 0.5) < 1e-9


def test_fgpid_trigger_semantics(oracle_lib):
    """FGPID (f16.xml:383-389 roll-rate PID): out = kp in + I + kd (in - prev)/dt; with the
    trigger 0 the integral accumulates ki dt in, a non-zero trigger holds it, a negative one
    resets it to zero; RunIC (ic) neither integrates nor differentiates."""
    kp, ki, kd, dt = 3.0, 5e-4, -1.25e-3, 1 / 120
    I, prev = ctypes.c_double(0.0), ctypes.c_double(0.0)
    f = lambda x, trig, ic=0: oracle_lib.f16ref_pid(x, ctypes.byref(I), ctypes.byref(prev), trig, kp, ki, kd, dt, ic)  # noqa: E731
    out = f(0.5, 0.0)
    assert I.value == pytest.approx(ki * dt * 0.5) and out == pytest.approx(kp * 0.5 + I.value + kd * 0.5 / dt)
    i1 = I.value
    out = f(0.7, 1.0)                       # held
    assert I.value == i1 and out == pytest.approx(kp * 0.7 + i1 + kd * 0.2 / dt)
    f(0.7, 0.0)
    assert I.value == pytest.approx(i1 + ki * dt * 0.7)
    f(0.1, -1.0)                            # reset
    assert I.value == 0.0
    out = f(0.4, 0.0, ic=1)                 # trim mode
    assert I.value == 0.0 and out == pytest.approx(kp * 0.4) and prev.value == 0.4


def test_aerosurface_scale_and_seek(oracle_lib):
    """aerosurface_scale, zero-centred (f16.xml rudder :746-751): 0 -> 0, each side scaled by its
    own end; FGTurbine Seek (F100-PW-229 spool): approach at the accel rate when below the
    target and the decel rate above, never overshooting."""
    s = oracle_lib.f16ref_aero_scale
    assert s(0.0, -1, 1, -0.524, 0.524) == 0.0
    assert s(0.5, -1, 1, -0.524, 0.524) == pytest.approx(0.262)
    assert s(-0.25, -1, 1, -0.4, 0.6) == pytest.approx(-0.1)
    sk = oracle_lib.f16ref_seek
    v = 60.0
    for _ in range(10):
        v2 = sk(v, 100.0, 20.0, 60.0, 0.1)
        assert v2 == pytest.approx(min(v + 2.0, 100.0))
        v = v2
    assert v == 80.0
    assert sk(90.0, 80.0, 20.0, 60.0, 0.1) == pytest.approx(84.0)
    assert sk(81.0, 80.0, 20.0, 60.0, 0.1) == 80.0
