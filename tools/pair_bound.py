#!/usr/bin/env python3
"""Issue bound of a lane-pair step kernel, from static VALU counts of the
frame sections a pair of lanes could divide SIMT-uniformly plus the SQ counters measured on the
box (profiles/r04_half_wave_ab.json). CPU only: compiles tools/probes/pair_sections.hip to
gfx950 assembly and counts instructions per kernel.

    python tools/pair_bound.py [--json profiles/r04_lane_pair_bound.json]

A lane pair puts one env on two lanes of a wave: 32 envs per wave, 2 048 waves = two per SIMD at
65 536 envs. Both lanes of a pair execute the same instruction stream (SIMT), so a role branch
("lane 0 does the FCS, lane 1 the engine") runs both sides on the whole wave under an exec
mask and saves nothing; what divides is only work that is the SAME code on different data --
here the 34 aerodynamic table blends (role-dependent LDS addresses) and the alpha / beta
atan2 pair. Everything else (the fp64 propagation, derive, atmosphere, FCS, engine, the force
and moment sums, accelerations, the env layer) runs on both lanes.
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "probes", "pair_sections.hip")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=on", "-fno-slp-vectorize",
         "-I", os.path.join(ROOT, "include"), "-Wno-unused-value", "-Wno-unused-result", "--cuda-device-only", "-S"]
KERNELS = ("k_base", "k_brackets", "k_blends", "k_aero", "k_io2", "k_fatan2", "k_frame", "k_frame_io")


def counts(asm: str):
    lines = asm.splitlines()
    out = {}
    for name in KERNELS:
        start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\d+%s\w*:" % name, l))
        end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith("s_endpgm"))
        c = collections.Counter()
        for l in lines[start:end]:
            s = l.strip()
            if not s or s.startswith((".", ";")) or s.endswith(":"):
                continue
            op = s.split()[0]
            c["valu" if op.startswith("v_") and not op.startswith("v_accvgpr") else
              "lds" if op.startswith("ds_") else "other"] += 1
        out[name] = dict(c)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        s = os.path.join(td, "p.s")
        subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, SRC, "-o", s], check=True, stderr=subprocess.DEVNULL)
        c = counts(open(s).read())
    v = {k: c[k]["valu"] for k in KERNELS}
    # the 34 coefficient blends + their LDS address math; an UPPER bound: the probe's ~34 adds that
    # keep every value live are counted with them
    blends = v["k_blends"] - v["k_brackets"]
    sums = v["k_aero"] - v["k_blends"]                 # force / moment sums (not divisible: different terms)
    atan = v["k_fatan2"] - v["k_io2"] + 1              # k_io2's one add
    frame = v["k_frame"] - v["k_frame_io"]             # static, rare branches included
    divisible = blends + atan                          # per frame, SIMT-uniform: half saved per lane
    exchange = 17 + 1                                  # DPP moves: the other lane's 17 coefficients, one angle
    saved_per_frame = divisible / 2 - exchange
    meas = json.load(open(os.path.join(ROOT, "profiles", "r04_half_wave_ab.json")))["sq_counters_per_wave"]
    prod = next(x for k, x in meas.items() if k.startswith("production"))
    half = next(x for k, x in meas.items() if k.startswith("half"))
    frames = 4
    pair_active = half["SQ_ACTIVE_INST_ANY_per_wave"] - frames * saved_per_frame  # quad-cycles per pair wave-step
    simd_issue = 2 * pair_active
    res = {
        "what": "Issue bound of a lane-pair split of the windowed step at 65 536 envs (VERDICT r03 item 3)",
        "tool": "tools/pair_bound.py (static gfx950 VALU counts of tools/probes/pair_sections.hip) + SQ counters "
                "of profiles/r04_half_wave_ab.json",
        "static_valu": v,
        "per_frame": {"aero_blends_divisible": blends, "aero_force_moment_sums": sums, "fatan2_one": atan,
                      "frame_static_total": frame, "divisible": divisible, "dpp_exchange": exchange,
                      "saved_per_lane": saved_per_frame,
                      "divisible_frac_of_frame": round(divisible / frame, 4)},
        "measured": {"production_active_quads_per_wave_step": prod["SQ_ACTIVE_INST_ANY_per_wave"],
                     "production_wave_life_quads": prod["SQ_WAVE_CYCLES_per_wave"],
                     "half_wave_active_quads_per_wave_step": half["SQ_ACTIVE_INST_ANY_per_wave"],
                     "half_wave_kernel_us": 20.8, "production_kernel_us": 15.8},
        "pair_estimate": {"active_quads_per_pair_wave_step": round(pair_active, 1),
                          "simd_issue_quads_two_waves": round(simd_issue, 1),
                          "vs_production_wave_life": round(simd_issue / prod["SQ_WAVE_CYCLES_per_wave"], 3),
                          "projected_kernel_us_from_half_wave": round(20.8 * pair_active / half["SQ_ACTIVE_INST_ANY_per_wave"], 2)},
        "reading": None,
    }
    res["reading"] = (
        "A pair wave carries the half-populated wave's stream minus what the two lanes can divide: per frame %d VALU "
        "(the 34 table blends %d, an upper bound, + one atan2 %d) of ~%d, i.e. %.1f%%, of which each lane saves half "
        "less %d DPP moves = %.1f VALU, %.1f%% of the half-populated wave's %.0f issue quad-cycles per step. The "
        "half-populated wave (two waves per SIMD, each with a whole env's stream) measured 20.8 us against 15.8 us; "
        "scaled by the pair wave's shorter stream: %.1f us. Two pair waves per SIMD would issue %.0f quad-cycles per "
        "step if their issue does not overlap (the half-populated waves' counters: 2 x 5 023 against a 10 064 "
        "quad-cycle wave life), %.2fx the production wave's whole life (%.0f). Not built." % (
            divisible, blends, atan, frame, 100.0 * divisible / frame, exchange, saved_per_frame,
            100.0 * frames * saved_per_frame / half["SQ_ACTIVE_INST_ANY_per_wave"], half["SQ_ACTIVE_INST_ANY_per_wave"],
            res["pair_estimate"]["projected_kernel_us_from_half_wave"], simd_issue,
            simd_issue / prod["SQ_WAVE_CYCLES_per_wave"], prod["SQ_WAVE_CYCLES_per_wave"]))
    print(json.dumps(res, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
