"""Pin the CPU oracle against every known answer available without running reference code
(SURVEY.md 8c): the reference's own XML data (tables, constants), published standards
(US-1976 atmosphere, WGS84, Random123 Philox KATs), the numpy goal stream of
jsbsim_gym.py:312-323, and the env semantics of jsbsim_gym.py / dummy_vec_env.py."""
from __future__ import annotations

import json
import math
import os
import re
import xml.etree.ElementTree as ET

import numpy as np
import pytest

from oracle_ref import OracleEnvs, atmosphere, default_ic, lib, philox

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
REF_XML = "/root/reference/aircraft/f16/f16.xml"


def model():
    with open(os.path.join(GOLD, "f16_model.json")) as f:
        return json.load(f)


# ------------------------------------------------------------------------------------------
# tables: fixture vs XML (when the reference is present) and oracle lookups vs fixture
# ------------------------------------------------------------------------------------------
@pytest.mark.skipif(not os.path.exists(REF_XML), reason="reference XML not present")
def test_fixture_matches_reference_xml():
    m = model()
    root = ET.parse(REF_XML).getroot()
    aero = root.find("aerodynamics")
    by_name = {}
    for axis in aero.findall("axis"):
        for f in axis.findall("function"):
            by_name[f.get("name").split("/")[-1]] = f
    assert len(by_name) == len(m["aero_functions"]) == 40
    for fn in m["aero_functions"]:
        x = by_name[fn["name"]]
        props = [p.text.strip() for p in x.find("product").findall("property")]
        assert props == fn["props"], fn["name"]
        tab = x.find("product").find("table")
        if tab is None:
            assert float(x.find("product").find("value").text) == fn["value"]
            continue
        toks = [ln.split() for ln in tab.find("tableData").text.strip().splitlines() if ln.strip()]
        if fn["table"]["cols"] is None:
            assert [float(t[0]) for t in toks] == fn["table"]["rows"]
            assert [float(t[1]) for t in toks] == fn["table"]["data"]
        else:
            assert [float(v) for v in toks[0]] == fn["table"]["cols"]
            assert [float(t[0]) for t in toks[1:]] == fn["table"]["rows"]
            assert [[float(v) for v in t[1:]] for t in toks[1:]] == fn["table"]["data"]
        with open(REF_XML) as fh:
            line = fh.read().splitlines()[fn["xml_line"] - 1]
        assert fn["name"] in line


def _kind_grid(t):
    rows = t["rows"]
    cols = t["cols"]
    return rows, cols


def test_oracle_tables_known_answers():
    """At every breakpoint the oracle returns the table entry; beyond the range it clamps
    (no extrapolation, f16.xml:536-537); between breakpoints it interpolates linearly."""
    m = model()
    L = lib()
    assert L.f16ref_n_aero_fns() == len(m["aero_functions"])
    for k, fn in enumerate(m["aero_functions"]):
        if "table" not in fn:
            assert L.f16ref_aero_table(k, 0.0, 0.0) == fn["value"]
            continue
        t = fn["table"]
        rows, cols, data = t["rows"], t["cols"], t["data"]
        if cols is None:
            for x, v in zip(rows, data):
                assert L.f16ref_aero_table(k, x, 0.0) == pytest.approx(v, rel=1e-14, abs=1e-15)
            assert L.f16ref_aero_table(k, rows[0] - 1.0, 0.0) == data[0]
            assert L.f16ref_aero_table(k, rows[-1] + 1.0, 0.0) == data[-1]
            mid = 0.5 * (rows[0] + rows[1])
            assert L.f16ref_aero_table(k, mid, 0.0) == pytest.approx(0.5 * (data[0] + data[1]), abs=1e-12)
        else:
            for i, x in enumerate(rows):
                for j, y in enumerate(cols):
                    assert L.f16ref_aero_table(k, x, y) == pytest.approx(data[i][j], rel=1e-14, abs=1e-15)
            assert L.f16ref_aero_table(k, rows[0] - 1, cols[0] - 1) == pytest.approx(data[0][0], abs=1e-15)
            assert L.f16ref_aero_table(k, rows[-1] + 1, cols[-1] + 1) == pytest.approx(data[-1][-1], abs=1e-15)
            xm, ym = 0.5 * (rows[0] + rows[1]), 0.5 * (cols[0] + cols[1])
            want = 0.25 * (data[0][0] + data[1][0] + data[0][1] + data[1][1])
            assert L.f16ref_aero_table(k, xm, ym) == pytest.approx(want, abs=1e-12)


def _slopes(v):
    """slope[i] = f32(v[i+1]) - f32(v[i]) along axis 0 in fp32, 0 on the last row"""
    v = np.asarray(v, np.float64).astype(np.float32)
    d = np.zeros_like(v)
    d[:-1] = v[1:] - v[:-1]
    return v, d


def _pair_slot(j, g):
    """(value, slope) float offsets of table j within a g-table entry: g values then g slopes for
    even g (tools/gen_tables.py put_rows), pairwise -- (2 values | 2 slopes) per table pair, an odd
    last table as (value | slope) -- for odd g"""
    if g % 2 == 0:
        return j, g + j
    c = j - j % 2
    w = min(2, g - c)
    return 2 * c + j % 2, 2 * c + w + j % 2


def test_kernel_blob_matches_fixture():
    """The fp32 LDS blob in f16_tables.h holds exactly the fixture's tables (rounded to fp32),
    each beside its fp32 slope along the first interpolation axis (value, slope layout)."""
    m = model()
    src = open(os.path.join(ROOT, "f16_jsb_amd", "csrc", "f16_tables.h")).read()
    offs = {k: int(v) for k, v in re.findall(r"#define OFF_(\w+) (\d+)", src)}
    body = src.split("F16_BLOB_INIT[F16_BLOB_FLOATS] = {")[1].split("};")[0]
    blob = np.array([float(x.rstrip("f")) for x in body.replace("\n", " ").split(",") if x.strip()], np.float32)
    fns = {f["name"]: f for f in m["aero_functions"]}
    a1d = ["CDDlef", "CDDsb", "CDq", "CDq_Dlef", "CYp", "CYr", "CLDlef", "CLDsb", "CLq", "CLq_Dsb",
           "Clp", "Clr", "CmDsb", "Cmq", "Cnp", "Cnr"]
    for j, n in enumerate(a1d):  # [12][16 values | 16 slopes]
        v, d = _slopes(fns[n]["table"]["data"])
        np.testing.assert_array_equal(blob[offs["alpha1d"] + np.arange(12) * 32 + j], v)
        np.testing.assert_array_equal(blob[offs["alpha1d"] + np.arange(12) * 32 + 16 + j], d)
    for key, names, ncol in (("ade", ["CDDh", "CLDh", "CmDh"], 5), ("ab13", ["Clb", "Cnb"], 13),
                             ("ab7", ["Clda", "Cldr", "Cnda", "Cndr"], 7)):
        g = len(names)
        for j, n in enumerate(names):  # [12][ncol][g values | g alpha-slopes]; odd g pairwise
            v, d = _slopes(fns[n]["table"]["data"])
            base = offs[key] + (np.arange(12)[:, None] * ncol + np.arange(ncol)[None, :]) * 2 * g
            vo, so = _pair_slot(j, g)
            np.testing.assert_array_equal(blob[base + vo], v)
            np.testing.assert_array_equal(blob[base + so], d)
    # engine: (mach x density-alt) union grid [14][8][3 values | 3 mach-slopes], Idle/Mil rows
    # clamped at their last mach row
    eng = m["engine"]["tables"]
    rows = eng["AugThrust"]["rows"]
    for j, n in enumerate(("IdleThrust", "MilThrust", "AugThrust")):
        t = np.asarray(eng[n]["data"], np.float64)
        full = t[np.minimum(np.arange(len(rows)), len(t) - 1)]
        v, d = _slopes(full)
        base = offs["engu_v"] + (np.arange(len(rows))[:, None] * 8 + np.arange(8)[None, :]) * 6
        vo, so = _pair_slot(j, 3)
        np.testing.assert_array_equal(blob[base + vo], v)
        np.testing.assert_array_equal(blob[base + so], d)
    # the nine Mach tables on their union grid, [13][pairwise 9 values / mach-slopes]: checked as
    # a pure re-layout of the blob order the kernel's blends read (value, slope per table)
    nt, nu = 9, 13
    for j in range(nt):
        vo, so = _pair_slot(j, nt)
        v = blob[offs["machu_v"] + np.arange(nu) * 2 * nt + vo]
        d = blob[offs["machu_v"] + np.arange(nu) * 2 * nt + so]
        np.testing.assert_array_equal(d[:-1], (v[1:] - v[:-1]).astype(np.float32))
        assert d[-1] == 0.0
    # ... and against the fixture: table j's values at the union breakpoints are
    # the fixture table MACH_1D[j] interpolated there (end-clamped), so a pair / table mix-up that
    # stays internally consistent (two tables swapped) fails here. The union grid is the header's.
    mach_1d = ["CDmach", "CYb_M", "Clb_M", "Clda_M", "Cldr_M", "Cma_M", "Cnb_M", "Cnda_M", "Cndr_M"]
    union = sorted({b for n in mach_1d for b in fns[n]["table"]["rows"]})
    hdr = re.search(r"BP_machu\[(\d+)\] = \{([^}]*)\}", src)
    assert int(hdr.group(1)) == nu == len(union)
    np.testing.assert_array_equal(np.array([float(x.strip().rstrip("f")) for x in hdr.group(2).split(",")], np.float32),
                                  np.array(union, np.float32))
    for j, n in enumerate(mach_1d):
        rows, data = fns[n]["table"]["rows"], fns[n]["table"]["data"]
        want = np.array([np.interp(x, rows, data) for x in union], np.float64).astype(np.float32)
        vo, so = _pair_slot(j, nt)
        got = blob[offs["machu_v"] + np.arange(nu) * 2 * nt + vo]
        # np.interp clamps at the ends like FGTable; the generator's own fp64 lerp may round the
        # last bit differently inside a segment, the breakpoints themselves are exact
        np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-7, err_msg=n)
        on_bp = np.isin(np.array(union), np.array(rows))
        np.testing.assert_array_equal(got[on_bp], np.asarray(data, np.float64).astype(np.float32)[
            np.searchsorted(rows, np.array(union)[on_bp])], err_msg=n)
    v, d = _slopes(m["kCLge"]["data"])
    np.testing.assert_array_equal(blob[offs["kclge_vd"] + 2 * np.arange(len(v))], v)
    np.testing.assert_array_equal(blob[offs["kclge_vd"] + 2 * np.arange(len(v)) + 1], d)
    # (lo, 1/span) bracket pairs are 8-byte aligned for ds_read_b64
    assert all(v % 2 == 0 for k, v in offs.items() if k.startswith("pair_") or k.endswith("_vd") or "_vd_" in k)


# ------------------------------------------------------------------------------------------
# published standards
# ------------------------------------------------------------------------------------------
# US Standard Atmosphere 1976 table values (geometric altitude m: T K, P Pa, rho kg/m^3)
US76 = [
    (0.0, 288.150, 101325.0, 1.2250),
    (1000.0, 281.651, 89876.0, 1.1117),
    (5000.0, 255.676, 54048.0, 0.73643),
    (11000.0, 216.774, 22700.0, 0.36480),
    (20000.0, 216.650, 5529.3, 0.088910),
    (32000.0, 228.490, 889.06, 0.013555),
]


@pytest.mark.parametrize("z,T,P,rho", US76)
def test_us76_atmosphere(z, T, P, rho):
    out = atmosphere(z / 0.3048)
    assert out[0] / 1.8 == pytest.approx(T, abs=2e-3)
    assert out[1] * 47.88025898033584 == pytest.approx(P, rel=2e-4)
    assert out[2] * 515.3788183931961 == pytest.approx(rho, rel=2e-4)
    assert out[3] * 0.3048 == pytest.approx(math.sqrt(1.4 * 287.05287 * out[0] / 1.8), rel=1e-6)


def test_wgs84_round_trip():
    import ctypes
    L = lib()
    rng = np.random.default_rng(1)
    for _ in range(200):
        lat = rng.uniform(-1.5, 1.5)
        lon = rng.uniform(-3.1, 3.1)
        h = rng.uniform(-1000, 200000)
        e = np.zeros(3)
        L.f16ref_geodetic_to_ecef(lat, lon, h, e.ctypes.data_as(ctypes.c_void_p))
        h2 = L.f16ref_geodetic_altitude(e.ctypes.data_as(ctypes.c_void_p))
        assert h2 == pytest.approx(h, abs=1e-5)


def test_philox_random123_kat():
    assert philox([0, 0], [0, 0, 0, 0]).tolist() == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert philox([0xFFFFFFFF] * 2, [0xFFFFFFFF] * 4).tolist() == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert philox([0xA4093822, 0x299F31D0], [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344]).tolist() == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_vcas_sea_level_identity():
    """At sea level the calibrated airspeed equals the true airspeed (subsonic)."""
    L = lib()
    a0 = atmosphere(0.0)
    for mach in (0.1, 0.5, 0.9):
        vc = L.f16ref_vcas_kts(mach, a0[1])
        assert vc * 1852.0 / (3600 * 0.3048) == pytest.approx(mach * a0[3], rel=1e-9)


# ------------------------------------------------------------------------------------------
# env layer semantics (jsbsim_gym.py)
# ------------------------------------------------------------------------------------------
def test_reference_goal_vectors():
    """SURVEY.md 8c goal vectors (numpy default_rng, jsbsim_gym.py:312-323)."""
    from f16_jsb_amd.env import reference_goal
    with open(os.path.join(GOLD, "goal_rng.json")) as f:
        g = json.load(f)
    for seed, want in g["goals"].items():
        np.testing.assert_array_equal(reference_goal(int(seed)), np.float32(want))


def test_ic_frame_matches_reference_ic():
    """Initial frame from the reference IC (u=900 fps, h=5000 ft, lat=lon=0, attitude 0)."""
    e = OracleEnvs(1, stack_k=10)
    goal = np.array([[100.0, -200.0, 3000.0]], np.float32)
    obs = e.reset(goals=goal)
    assert obs.shape == (1, 10, 15)
    assert np.all(obs[0] == obs[0, 0])                       # K copies (jsbsim_gym.py:325-329)
    f = obs[0, 0]
    assert f[0] == 0.0 and f[1] == 0.0
    assert f[2] == np.float32(5000.0 * 0.3048)               # h-sl-meters
    a = atmosphere(5000.0)[3]
    assert f[3] == pytest.approx(900.0 / a, rel=1e-6)        # mach
    assert np.all(np.abs(f[4:12]) < 1e-6)
    np.testing.assert_array_equal(f[12:], goal[0])


def _py_norm_angle(a):
    """jsbsim_gym.py:60-78 on a float32 state element (numpy 1.26 semantics)."""
    a = np.float32(a)
    if np.isnan(a) or np.isinf(a):
        return np.float32(0.0)
    x = float(a) % (2 * np.pi)
    if x >= np.pi:
        x -= 2 * np.pi
    return np.float32(x)


def test_crash_goal_truncation_semantics():
    """down_sample=0 freezes the physics so the env logic is isolated: crash (-10, :245-247),
    goal (+10, :252-257), truncation (TimeLimit 1200 / max_steps), auto-reset with
    terminal observation (dummy_vec_env.py:68-71), Monitor return/length."""
    ic = default_ic()
    # lane 0: below the crash altitude; lane 1: goal at the aircraft; lane 2: plain
    ics = np.tile(ic, (3, 1))
    ics[0, 2] = 20.0  # 6.1 m
    e = OracleEnvs(3, stack_k=4, down_sample=0, max_steps=3)
    goals = np.array([[5000, 5000, 3000], [0.0, 0.0, 1524.0], [5000, 5000, 3000]], np.float32)
    obs0 = e.reset(goals=goals, ic=ics)
    act = np.zeros((3, 4), np.float32)
    obs, rew, term, trunc, tobs, eret, elen = e.step(act)
    assert term.tolist() == [True, True, False] and trunc.tolist() == [False, False, False]
    assert rew[0] == np.float32(-10.0) and rew[1] == np.float32(10.0) and rew[2] == np.float32(0.0)
    assert eret[0] == -10.0 and elen[0] == 1 and eret[1] == 10.0
    # terminal obs = stack after the step; returned obs = reset stack
    np.testing.assert_array_equal(tobs[0, :3], obs0[0, 1:])
    assert np.all(obs[0] == obs[0, 0])
    obs, rew, term, trunc, *_ = e.step(act)
    obs, rew, term, trunc, tobs, eret, elen = e.step(act)
    assert trunc[2] and not term[2] and elen[2] == 3


def test_normalize_angle_matches_reference_formula():
    """make_frame's angle normalisation == jsbsim_gym.normalize_angle_mpi_pi on float32."""
    e = OracleEnvs(1, stack_k=1, down_sample=0)
    ic = default_ic()
    for psi in (0.0, 0.5, np.pi - 1e-7, np.pi, np.pi + 1e-6, 2 * np.pi - 1e-7, 3.0, 5.5):
        ic2 = ic.copy()
        ic2[8] = psi
        obs = e.reset(goals=np.zeros((1, 3), np.float32), ic=ic2[None])
        st = e.get_state()
        # psi as JSBSim reports it, in [0, 2pi)
        want = _py_norm_angle(np.float32(psi % (2 * np.pi)))
        assert obs[0, 0, 11] == pytest.approx(float(want), abs=2e-6)


def test_trimmed_flight_is_level():
    """Trim (BASELINE cfg 2): after trimming at 5000 ft / 900 fps and holding the trim
    command, altitude and speed stay near their initial values for 1200 steps (40 s)."""
    ic = default_ic()
    e = OracleEnvs(1, stack_k=1)
    tic, res = e.trim(ic[None])
    assert np.all(res < 1e-3), res
    obs = e.reset(goals=np.zeros((1, 3), np.float32), ic=tic)
    act = np.array([[0.0, tic[0, 13], 0.0, tic[0, 15]]], np.float32)
    h0, m0 = obs[0, 0, 2], obs[0, 0, 3]
    for t in range(1200):
        obs, *_ = e.step(act)
    assert abs(obs[0, -1, 2] - h0) < 30.0
    assert abs(obs[0, -1, 3] - m0) < 0.01


def test_cfg1_single_env_1000_random_steps():
    """BASELINE cfg1: 1 env, reference IC, 1000 steps of Box-uniform random actions
    from numpy.random.default_rng(0) (jsbsim_gym.py:143-148 bounds), first reset seed 0
    (jsbsim_gym.py:312-323 goal), through the CPU oracle: finite observations inside the
    float32 frame format, the step counter / Monitor length bookkeeping across auto-resets,
    and returns equal to the sum of the step rewards."""
    from f16_jsb_amd.env import reference_goal
    e = OracleEnvs(1, stack_k=10)
    obs = e.reset(goals=reference_goal(0)[None, :])
    np.testing.assert_array_equal(obs[0, -1, 12:], reference_goal(0))
    rng = np.random.default_rng(0)
    low, high = np.array([-1, -1, -1, 0], np.float32), np.array([1, 1, 1, 1], np.float32)
    ep_len, ep_ret, episodes = 0, 0.0, 0
    for t in range(1000):
        a = rng.uniform(low, high).astype(np.float32)[None, :]
        obs, rew, term, trunc, tobs, eret, elen = e.step(a)
        assert obs.shape == (1, 10, 15) and obs.dtype == np.float32 and np.all(np.isfinite(obs))
        ep_len += 1
        ep_ret += float(rew[0])
        assert not (term[0] and trunc[0])
        if term[0] or trunc[0]:
            episodes += 1
            assert elen[0] == ep_len and trunc[0] == (ep_len >= 1200)
            assert eret[0] == pytest.approx(ep_ret, abs=1e-3)
            assert np.all(obs[0] == obs[0, 0])  # K copies of the reset frame
            ep_len, ep_ret = 0, 0.0
        else:
            # attitude angles normalised to [-pi, pi) (jsbsim_gym.py:186-188)
            assert np.all(np.abs(obs[0, -1, 9:12]) <= np.float32(np.pi))
    assert episodes + (ep_len > 0) >= 1
