#!/usr/bin/env python3
"""F-16 model compiler: reads the reference's JSBSim aircraft XML and emits

  * ``tests/golden/f16_model.json``   -- every table / function / constant with
                                          its source line (the golden fixture);
  * ``oracle/f16ref_tables.h``        -- fp64 C data for the CPU oracle (data only,
                                          natural XML layout);
  * ``f16_jsb_amd/csrc/f16_tables.h`` -- fp32 LDS blob for the HIP kernel, grouped
                                          by shared breakpoint vectors.

Sources (read as DATA, never executed):
  /root/reference/aircraft/f16/f16.xml                 (metrics 37-60, mass 62-83,
        propulsion 245-300, FCS tables 434-443/539-551/676-686/897-907,
        aerodynamics 986-1917)
  /root/reference/aircraft/f16/Engines/F100-PW-229.xml (engine 1-84)

Run here (the reference is not on the GPU box); outputs are committed.
"""
from __future__ import annotations

import json
import os
import re
import sys
import xml.etree.ElementTree as ET

import numpy as np

REF = os.environ.get("F16_REFERENCE", "/root/reference")
XML = os.path.join(REF, "aircraft/f16/f16.xml")
ENG = os.path.join(REF, "aircraft/f16/Engines/F100-PW-229.xml")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# Property vocabulary used by the aero function products (f16.xml:986-1917).
PROPS = [
    "aero/qbar-psf", "metrics/Sw-sqft", "metrics/bw-ft", "metrics/cbarw-ft",
    "aero/alpha-rad", "aero/beta-rad", "velocities/mach",
    "velocities/p-aero-rad_sec", "velocities/q-aero-rad_sec", "velocities/r-aero-rad_sec",
    "aero/bi2vel", "aero/ci2vel", "aero/function/kCLge",
    "fcs/elevator-pos-rad", "fcs/aileron-pos-rad", "fcs/rudder-pos-rad",
    "fcs/lef-pos-rad", "fcs/flaperon-mix-rad", "fcs/speedbrake-pos-rad",
    "gear/gear-pos-norm",
]
AXES = ["DRAG", "SIDE", "LIFT", "ROLL", "PITCH", "YAW"]


def _line_of(lines, pattern, start=0):
    rx = re.compile(pattern)
    for i in range(start, len(lines)):
        if rx.search(lines[i]):
            return i + 1
    raise KeyError(pattern)


def _parse_table(tab):
    """Return dict(indep=[...], rows=[...], cols=[...]|None, data=[[...]])."""
    ivs = tab.findall("independentVar")
    txt = tab.find("tableData").text
    toks = [ln.split() for ln in txt.strip().splitlines() if ln.strip()]
    if len(ivs) == 1:
        rows = [float(t[0]) for t in toks]
        data = [float(t[1]) for t in toks]
        return {"indep": [ivs[0].text.strip()], "rows": rows, "cols": None, "data": data}
    assert len(ivs) == 2
    order = {iv.get("lookup", "row"): iv.text.strip() for iv in ivs}
    cols = [float(x) for x in toks[0]]
    rows, data = [], []
    for t in toks[1:]:
        assert len(t) == len(cols) + 1, t
        rows.append(float(t[0]))
        data.append([float(x) for x in t[1:]])
    return {"indep": [order["row"], order["column"]], "rows": rows, "cols": cols, "data": data}


def parse():
    with open(XML) as f:
        xml_lines = f.read().splitlines()
    with open(ENG) as f:
        eng_lines = f.read().splitlines()
    root = ET.parse(XML).getroot()
    eng = ET.parse(ENG).getroot()

    model = {"source": {"f16.xml": XML, "engine": ENG}}

    # ---- metrics / mass balance (f16.xml:37-83) --------------------------------
    met = root.find("metrics")
    model["metrics"] = {
        "wingarea_ft2": float(met.find("wingarea").text),
        "wingspan_ft": float(met.find("wingspan").text),
        "chord_ft": float(met.find("chord").text),
        "xml_line": _line_of(xml_lines, r"<metrics>"),
    }
    locs = {}
    for loc in met.findall("location"):
        locs[loc.get("name")] = [float(loc.find(a).text) for a in "xyz"]
    model["metrics"]["aerorp_in"] = locs["AERORP"]
    model["metrics"]["eyepoint_in"] = locs["EYEPOINT"]
    model["metrics"]["vrp_in"] = locs["VRP"]
    mb = root.find("mass_balance")
    model["mass"] = {
        "negated_crossproduct_inertia": mb.get("negated_crossproduct_inertia") == "true",
        "ixx": float(mb.find("ixx").text), "iyy": float(mb.find("iyy").text),
        "izz": float(mb.find("izz").text), "ixy": float(mb.find("ixy").text),
        "ixz": float(mb.find("ixz").text), "iyz": float(mb.find("iyz").text),
        "emptywt_lbs": float(mb.find("emptywt").text),
        "cg_in": [float(mb.find("location").find(a).text) for a in "xyz"],
        "pointmasses": [
            {"name": pm.get("name"), "weight_lbs": float(pm.find("weight").text),
             "loc_in": [float(pm.find("location").find(a).text) for a in "xyz"]}
            for pm in mb.findall("pointmass")
        ],
        "xml_line": _line_of(xml_lines, r"<mass_balance"),
    }
    prop = root.find("propulsion")
    thr = prop.find("engine").find("thruster")
    model["propulsion"] = {
        "thruster_loc_in": [float(thr.find("location").find(a).text) for a in "xyz"],
        "thruster_orient_deg": [float(thr.find("orient").find(a).text) for a in ("roll", "pitch", "yaw")],
        "tanks": [
            {"loc_in": [float(t.find("location").find(a).text) for a in "xyz"],
             "capacity_lbs": float(t.find("capacity").text),
             "contents_lbs": float(t.find("contents").text)}
            for t in prop.findall("tank")
        ],
        "xml_line": _line_of(xml_lines, r"<propulsion>"),
    }

    # ---- FCS tables (scheduled_gain) -----------------------------------------
    fcs_tables = {}
    for sg in root.iter("scheduled_gain"):
        name = sg.get("name")
        t = _parse_table(sg.find("table"))
        t["xml_line"] = _line_of(xml_lines, r'scheduled_gain name="%s"' % re.escape(name))
        fcs_tables[name] = t
    model["fcs_tables"] = fcs_tables

    # ---- aerodynamics (f16.xml:986-1917) -------------------------------------
    aero = root.find("aerodynamics")
    fn = aero.find("function")
    assert fn.get("name") == "aero/function/kCLge"
    kclge = _parse_table(fn.find("table"))
    kclge["xml_line"] = _line_of(xml_lines, r'function name="aero/function/kCLge"')
    model["kCLge"] = kclge
    funcs = []
    for axis in aero.findall("axis"):
        an = axis.get("name")
        for f in axis.findall("function"):
            name = f.get("name")
            prod = f.find("product")
            props = [p.text.strip() for p in prod.findall("property")]
            for p in props:
                assert p in PROPS, (name, p)
            vals = [float(v.text) for v in prod.findall("value")]
            tabs = prod.findall("table")
            assert len(vals) + len(tabs) == 1, name
            ent = {"name": name.split("/")[-1], "axis": an, "props": props,
                   "xml_line": _line_of(xml_lines, r'function name="%s"' % re.escape(name))}
            if vals:
                ent["value"] = vals[0]
            else:
                ent["table"] = _parse_table(tabs[0])
                if tabs[0].get("name"):
                    ent["table_name"] = tabs[0].get("name")
            funcs.append(ent)
    model["aero_functions"] = funcs

    # ---- engine (F100-PW-229.xml) ----------------------------------------------
    e = {k: float(eng.find(k).text) for k in (
        "milthrust", "maxthrust", "bypassratio", "tsfc", "atsfc", "bleed",
        "idlen1", "idlen2", "maxn1", "maxn2", "augmented", "augmethod", "injected")}
    e["tables"] = {}
    for f in eng.findall("function"):
        t = _parse_table(f.find("table"))
        t["xml_line"] = _line_of(eng_lines, r'function name="%s"' % f.get("name"))
        e["tables"][f.get("name")] = t
    model["engine"] = e
    return model


# ------------------------------------------------------------------------------
# emitters
# ------------------------------------------------------------------------------
def _cname(s):
    return re.sub(r"[^A-Za-z0-9]", "_", s)


def _lit(v, fmt):
    s = fmt % v
    if s.endswith("f"):
        core = s[:-1]
        if not any(ch in core for ch in ".eEn"):
            core += ".0"
        return core + "f"
    if not any(ch in s for ch in ".eEn"):
        s += ".0"
    return s


def _fmt(vals, per=8, fmt="%.17g"):
    out = []
    for i in range(0, len(vals), per):
        out.append("    " + ", ".join(_lit(v, fmt) for v in vals[i:i + per]) + ",")
    return "\n".join(out)


def emit_oracle(model, path):
    """Plain fp64 tables + a data-driven aero function list for oracle/f16ref.c."""
    L = ["/* GENERATED by tools/gen_tables.py from the reference's f16.xml / F100-PW-229.xml.",
         " * DATA ONLY (test infrastructure for the oracle). Do not edit by hand. */",
         "#ifndef F16REF_TABLES_H", "#define F16REF_TABLES_H", "",
         "typedef struct { int nrows, ncols; const double *rows, *cols, *data; int xml_line; } ref_table;",
         "/* ncols == 0 => 1-D table (data[nrows]); else data[nrows*ncols] row-major */", ""]

    def table(cn, t):
        L.append("static const double %s_rows[%d] = {\n%s\n};" % (cn, len(t["rows"]), _fmt(t["rows"])))
        if t["cols"] is None:
            L.append("static const double %s_data[%d] = {\n%s\n};" % (cn, len(t["data"]), _fmt(t["data"])))
            L.append("static const ref_table %s = { %d, 0, %s_rows, 0, %s_data, %d };" % (
                cn, len(t["rows"]), cn, cn, t["xml_line"]))
        else:
            flat = [v for r in t["data"] for v in r]
            L.append("static const double %s_cols[%d] = {\n%s\n};" % (cn, len(t["cols"]), _fmt(t["cols"])))
            L.append("static const double %s_data[%d] = {\n%s\n};" % (cn, len(flat), _fmt(flat)))
            L.append("static const ref_table %s = { %d, %d, %s_rows, %s_cols, %s_data, %d };" % (
                cn, len(t["rows"]), len(t["cols"]), cn, cn, cn, t["xml_line"]))
        L.append("")

    table("T_kCLge", model["kCLge"])
    for name, t in model["fcs_tables"].items():
        table("T_" + _cname(name.split("/")[-1]), t)
    for name, t in model["engine"]["tables"].items():
        table("T_" + name, t)
    for f in model["aero_functions"]:
        if "table" in f:
            for p in f["props"]:
                pass
            t = dict(f["table"])
            t["xml_line"] = f["xml_line"]
            table("T_" + f["name"], t)

    L.append("enum ref_prop {")
    for p in PROPS:
        L.append("  RP_%s," % _cname(p))
    L.append("  RP_COUNT };")
    L.append("enum ref_axis { " + ", ".join("AX_%s" % a for a in AXES) + " };")
    L.append("")
    L.append("typedef struct { const char* name; int axis; int nprops; int props[6]; int has_value; double value;")
    L.append("                 const ref_table* table; int tvar[2]; int xml_line; } ref_aero_fn;")
    L.append("static const ref_aero_fn REF_AERO_FNS[] = {")
    for f in model["aero_functions"]:
        props = [PROPS.index(p) for p in f["props"]]
        props += [0] * (6 - len(props))
        if "table" in f:
            tv = [PROPS.index(v) for v in f["table"]["indep"]] + [-1]
            L.append('  { "%s", AX_%s, %d, {%s}, 0, 0.0, &T_%s, {%d, %d}, %d },' % (
                f["name"], f["axis"], len(f["props"]), ", ".join(map(str, props)), f["name"],
                tv[0], tv[1], f["xml_line"]))
        else:
            L.append('  { "%s", AX_%s, %d, {%s}, 1, %.17g, 0, {-1, -1}, %d },' % (
                f["name"], f["axis"], len(f["props"]), ", ".join(map(str, props)), f["value"],
                f["xml_line"]))
    L.append("};")
    L.append("#define REF_N_AERO_FNS %d" % len(model["aero_functions"]))
    L.append("")
    L.append("#endif")
    with open(path, "w") as fh:
        fh.write("\n".join(L) + "\n")


# The HIP kernel's blob: shared breakpoint vectors + tables grouped by them so one
# (index, factor) pair per breakpoint vector serves every table that uses it.
ALPHA_1D = ["CDDlef", "CDDsb", "CDq", "CDq_Dlef", "CYp", "CYr", "CLDlef", "CLDsb", "CLq", "CLq_Dsb",
            "Clp", "Clr", "CmDsb", "Cmq", "Cnp", "Cnr"]
ALPHA_DE_2D = ["CDDh", "CLDh", "CmDh"]          # 12 x 5 over (alpha, elevator-pos-rad)
ALPHA_BETA13 = ["Clb", "Cnb"]                   # 12 x 13 over (alpha, beta)
ALPHA_BETA7 = ["Clda", "Cldr", "Cnda", "Cndr"]  # 12 x 7  over (alpha, beta)
MACH_1D = ["CDmach", "CYb_M", "Clb_M", "Clda_M", "Cldr_M", "Cma_M", "Cnb_M", "Cnda_M", "Cndr_M"]


def emit_kernel(model, path):
    fns = {f["name"]: f for f in model["aero_functions"]}
    blob = []
    offs = {}

    def put(key, vals):
        # every table starts at an even float offset: the kernels read (value, value) /
        # (slope, slope) and (lo, 1/span) pairs as one 8-byte element (ld2, ds_read_b64), which an
        # odd-length table before them would silently misalign; the header below
        # static_asserts it for every OFF_*
        if len(blob) % 2:
            blob.append(0.0)
        assert len(blob) % 2 == 0
        offs[key] = len(blob)
        blob.extend(vals)

    alpha_bp = fns["CDDlef"]["table"]["rows"]
    for n in ALPHA_1D + ALPHA_DE_2D + ALPHA_BETA13 + ALPHA_BETA7:
        assert fns[n]["table"]["rows"] == alpha_bp, n
        assert fns[n]["table"]["indep"][0] == "aero/alpha-rad", n
    de_bp = fns["CDDh"]["table"]["cols"]
    for n in ALPHA_DE_2D:
        assert fns[n]["table"]["cols"] == de_bp and fns[n]["table"]["indep"][1] == "fcs/elevator-pos-rad"
    b13 = fns["Clb"]["table"]["cols"]
    b7 = fns["Clda"]["table"]["cols"]
    for n in ALPHA_BETA13:
        assert fns[n]["table"]["cols"] == b13 and fns[n]["table"]["indep"][1] == "aero/beta-rad"
    for n in ALPHA_BETA7:
        assert fns[n]["table"]["cols"] == b7 and fns[n]["table"]["indep"][1] == "aero/beta-rad"
    for n in MACH_1D:
        assert fns[n]["table"]["indep"] == ["velocities/mach"], n
    listed = set(ALPHA_1D + ALPHA_DE_2D + ALPHA_BETA13 + ALPHA_BETA7 + MACH_1D)
    assert listed == {f["name"] for f in model["aero_functions"] if "table" in f}

    # Every table is stored as (value, slope) along the interpolation axis the kernel blends
    # first: slope[i] = f32(v[i+1]) - f32(v[i]) (fp32 arithmetic, 0 on the last row), so a
    # lerp is one FMA v + f * slope -- bit-identical to f * (v1 - v0) + v0 computed in-kernel.
    def put_rows(key, rows_vals, group, pairwise=False):
        """rows over the interpolation axis, each a list of entries of `group` values; emitted
        per (row, entry) as the group's values then its slopes -- or, pairwise (odd groups),
        per pair of tables as their two values then their two slopes (an odd last table as its
        value, slope), so that every (value, value) and (slope, slope) pair a packed blend reads
        sits at an even float offset: an aligned register pair straight from the LDS read"""
        v = [np.array(r, np.float64).astype(np.float32) for r in rows_vals]
        vals = []
        for i in range(len(v)):
            d = (v[i + 1] - v[i]) if i + 1 < len(v) else np.zeros_like(v[i])
            for e in range(len(v[i]) // group):
                step = 2 if pairwise else group
                for c in range(e * group, (e + 1) * group, step):
                    hi = min(c + step, (e + 1) * group)
                    vals += [float(x) for x in v[i][c:hi]]
                    vals += [float(x) for x in d[c:hi]]
        put(key, vals)

    # alpha-1D tables: [12 alpha][16 values | 16 slopes]
    put_rows("alpha1d", [[fns[n]["table"]["data"][i] for n in ALPHA_1D] for i in range(12)], len(ALPHA_1D))
    # 2-D over (alpha, X): [12 alpha][X][group values | group alpha-slopes]; the 3-table group
    # (alpha, elevator) pairwise: [2 values | 2 alpha-slopes | value | alpha-slope]
    put_rows("ade", [[fns[n]["table"]["data"][i][j] for j in range(len(de_bp)) for n in ALPHA_DE_2D]
                     for i in range(12)], len(ALPHA_DE_2D), pairwise=True)
    put_rows("ab13", [[fns[n]["table"]["data"][i][j] for j in range(len(b13)) for n in ALPHA_BETA13]
                      for i in range(12)], len(ALPHA_BETA13))
    put_rows("ab7", [[fns[n]["table"]["data"][i][j] for j in range(len(b7)) for n in ALPHA_BETA7]
                     for i in range(12)], len(ALPHA_BETA7))

    # ---- union grids (exact re-gridding: every original breakpoint is a union breakpoint,
    # so the piecewise-linear, end-clamped functions are unchanged up to fp rounding) -------
    def interp_clamped(rows, data, x):
        if x <= rows[0]:
            return data[0]
        if x >= rows[-1]:
            return data[-1]
        i = 1
        while i < len(rows) - 1 and rows[i] < x:
            i += 1
        f = (x - rows[i - 1]) / (rows[i] - rows[i - 1])
        return data[i - 1] + f * (data[i] - data[i - 1])

    mach_u = sorted({b for n in MACH_1D for b in fns[n]["table"]["rows"]})
    # [13 mach][(2 values | 2 slopes) x 4, value | slope]
    put_rows("machu_v", [[interp_clamped(fns[n]["table"]["rows"], fns[n]["table"]["data"], x) for n in MACH_1D]
                         for x in mach_u], len(MACH_1D), pairwise=True)
    eng_rows = model["engine"]["tables"]["AugThrust"]["rows"]
    eng_cols = model["engine"]["tables"]["AugThrust"]["cols"]
    eng_names = ("IdleThrust", "MilThrust", "AugThrust")
    for n in eng_names:
        t = model["engine"]["tables"][n]
        assert t["cols"] == eng_cols
        assert t["rows"] == eng_rows[:len(t["rows"])]
    eng_u = []
    for i in range(len(eng_rows)):
        row = []
        for j in range(len(eng_cols)):
            for n in eng_names:
                t = model["engine"]["tables"][n]
                ii = min(i, len(t["rows"]) - 1)  # FGTable clamps the row factor at the last row
                row.append(t["data"][ii][j])
        eng_u.append(row)
    # [14 mach][8 density-alt][2 values | 2 mach-slopes | value | mach-slope]
    put_rows("engu_v", eng_u, len(eng_names), pairwise=True)
    # small 1-D tables: (value, slope) pairs
    put_rows("kclge_vd", [[v] for v in model["kCLge"]["data"]], 1)
    for n, t in model["fcs_tables"].items():
        put_rows("fcs_vd_" + n.split("/")[-1], [[v] for v in t["data"]], 1)
    # (lo, 1/span) pairs for LDS brackets (8-byte aligned for ds_read_b64)
    while len(blob) % 4:  # whole 16-byte pieces: the kernels stage the blob by LDS-DMA
        blob.append(0.0)

    def pairs(bp):
        out = []
        for i in range(len(bp) - 1):
            out += [bp[i], 1.0 / (bp[i + 1] - bp[i])]
        return out
    for key, bp in (("alpha", alpha_bp), ("de", de_bp), ("beta13", b13), ("beta7", b7),
                    ("machu", mach_u), ("kclge", model["kCLge"]["rows"])):
        put("pair_" + key, pairs(bp))
    for n, t in model["fcs_tables"].items():
        put("pair_fcs_" + n.split("/")[-1], pairs(t["rows"]))
    while len(blob) % 4:  # whole 16-byte pieces: the kernels stage the blob by LDS-DMA
        blob.append(0.0)
    mach_meta = [(n, len(fns[n]["table"]["rows"])) for n in MACH_1D]
    eng_meta = [(n, len(model["engine"]["tables"][n]["rows"]), len(model["engine"]["tables"][n]["cols"]))
                for n in eng_names]

    L = ["/* GENERATED by tools/gen_tables.py from the reference's f16.xml / F100-PW-229.xml.",
         " * fp32 table blob staged into LDS by the step kernel. Do not edit by hand. */",
         "#pragma once", ""]
    L.append("#define F16_BLOB_FLOATS %d" % len(blob))
    L.append("#define F16_N_ALPHA %d" % len(alpha_bp))
    L.append("#define F16_N_DE %d" % len(de_bp))
    L.append("#define F16_N_B13 %d" % len(b13))
    L.append("#define F16_N_B7 %d" % len(b7))
    L.append("#define F16_N_A1D %d" % len(ALPHA_1D))
    for i, n in enumerate(ALPHA_1D):
        L.append("#define A1D_%s %d" % (n, i))
    for i, n in enumerate(ALPHA_DE_2D):
        L.append("#define ADE_%s %d" % (n, i))
    for i, n in enumerate(ALPHA_BETA13):
        L.append("#define AB13_%s %d" % (n, i))
    for i, n in enumerate(ALPHA_BETA7):
        L.append("#define AB7_%s %d" % (n, i))
    for n, nr in mach_meta:
        L.append("#define MACH_N_%s %d" % (n, nr))
    L.append("#define KCLGE_N %d" % len(model["kCLge"]["rows"]))
    L.append("#define MACHU_N %d" % len(mach_u))
    L.append("#define MACHU_NT %d" % len(MACH_1D))
    for i, n in enumerate(MACH_1D):
        L.append("#define MU_%s %d" % (n, i))
    L.append("#define ENGU_NR %d" % len(eng_rows))
    L.append("#define ENGU_NC %d" % len(eng_cols))
    L.append("static constexpr float BP_machu[%d] = {%s};" % (len(mach_u), ", ".join(_lit(v, "%.9gf") for v in mach_u)))
    for n, t in model["fcs_tables"].items():
        L.append("#define FCS_N_%s %d" % (_cname(n.split("/")[-1]), len(t["rows"])))
    for n, nr, nc in eng_meta:
        L.append("#define ENG_NR_%s %d" % (n, nr))
        L.append("#define ENG_NC_%s %d" % (n, nc))
    for k, v in offs.items():
        L.append("#define OFF_%s %d" % (_cname(k), v))
    for k in offs:
        L.append('static_assert(OFF_%s %% 2 == 0, "8-byte pair reads need an even float offset");' % _cname(k))
    L.append("")
    L.append("/* breakpoint vectors are also emitted as constexpr arrays so unrolled searches fold")
    L.append(" * them into instruction literals (no LDS reads for breakpoints). */")
    for key, bp in (("alpha_bp", alpha_bp), ("de_bp", de_bp), ("beta13_bp", b13), ("beta7_bp", b7)):
        L.append("static constexpr float BP_%s[%d] = {%s};" % (key, len(bp), ", ".join(_lit(v, "%.9gf") for v in bp)))
    for n, nr in mach_meta:
        L.append("static constexpr float BP_mach_%s[%d] = {%s};" % (n, nr, ", ".join(_lit(v, "%.9gf") for v in fns[n]["table"]["rows"])))
    L.append("static constexpr float BP_kclge[%d] = {%s};" % (len(model["kCLge"]["rows"]), ", ".join(_lit(v, "%.9gf") for v in model["kCLge"]["rows"])))
    for n, t in model["fcs_tables"].items():
        L.append("static constexpr float BP_fcs_%s[%d] = {%s};" % (_cname(n.split("/")[-1]), len(t["rows"]), ", ".join(_lit(v, "%.9gf") for v in t["rows"])))
    for n, nr, nc in eng_meta:
        t = model["engine"]["tables"][n]
        L.append("static constexpr float BP_engr_%s[%d] = {%s};" % (n, nr, ", ".join(_lit(v, "%.9gf") for v in t["rows"])))
        L.append("static constexpr float BP_engc_%s[%d] = {%s};" % (n, nc, ", ".join(_lit(v, "%.9gf") for v in t["cols"])))
    L.append("")
    L.append("__device__ __attribute__((aligned(16))) const float F16_BLOB_INIT[F16_BLOB_FLOATS] = {")
    L.append(_fmt(blob, per=8, fmt="%.9gf"))
    L.append("};")
    with open(path, "w") as fh:
        fh.write("\n".join(L) + "\n")


def main():
    if not os.path.exists(XML):
        sys.exit("reference XML not found at %s (generator runs only in the build container)" % XML)
    model = parse()
    os.makedirs(os.path.join(ROOT, "tests/golden"), exist_ok=True)
    with open(os.path.join(ROOT, "tests/golden/f16_model.json"), "w") as fh:
        model_out = dict(model)
        model_out["source"] = {"f16.xml": "aircraft/f16/f16.xml",
                               "engine": "aircraft/f16/Engines/F100-PW-229.xml"}
        json.dump(model_out, fh, indent=1)
    emit_oracle(model, os.path.join(ROOT, "oracle/f16ref_tables.h"))
    emit_kernel(model, os.path.join(ROOT, "f16_jsb_amd/csrc/f16_tables.h"))
    print("aero functions:", len(model["aero_functions"]),
          "fcs tables:", len(model["fcs_tables"]), "engine tables:", len(model["engine"]["tables"]))


if __name__ == "__main__":
    main()
