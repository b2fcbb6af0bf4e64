#!/usr/bin/env python3
"""VALU utilisation of f16_step_kernel from the SQ counter passes of tools/gpu_session.sh `sq`
(three rocprofv3 --pmc runs of bench.py, 8 SQ counters each), per wave and per env step.

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles
(/opt/skills/guides/MI355X_MICROARCH.md, per-instruction constants table); instruction
counts are instructions. The kernel runs one wave per SIMD (1 024 waves on 1 024 SIMDs at
65 536 envs), so a wave's VALU-active fraction is its SIMD's VALU-busy fraction over the
wave's lifetime.

    python tools/pmc_valu.py DIR_OR_CSV [DIR_OR_CSV ...] --envs 65536 --stack 4 [--out profiles/pmc_valu.json]
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import statistics


def rows(path):
    if os.path.isdir(path):
        path = os.path.join(path, "run_counter_collection.csv")
    return csv.DictReader(open(path))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("inputs", nargs="+")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--stack", type=int, default=4)
    ap.add_argument("--kernel", default="f16_step_win_kernel")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    vals = collections.defaultdict(list)
    for p in args.inputs:
        for r in rows(p):
            if r["Kernel_Name"].removeprefix("void ").startswith(args.kernel) and int(r["Grid_Size"]) == args.envs:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    med = {k: statistics.median(v) for k, v in vals.items()}
    waves = med["SQ_WAVES"]
    per_wave = {k: round(v / waves, 1) for k, v in sorted(med.items()) if k != "SQ_WAVES"}
    cyc = med["SQ_WAVE_CYCLES"]
    out = {
        "kernel": args.kernel,
        "envs": args.envs,
        "stack_k": args.stack,
        "waves": int(waves),
        "launches": min(len(v) for v in vals.values()),
        "per_wave_step": per_wave,
        "wave_cycles": round(4 * cyc / waves),
        "valu_insts_per_wave_step": per_wave["SQ_INSTS_VALU"],
        "valu_busy_frac": round(med["SQ_ACTIVE_INST_VALU"] / cyc, 3),
        "wait_any_frac": round(med["SQ_WAIT_ANY"] / cyc, 3),
        "wait_inst_any_frac": round(med["SQ_WAIT_INST_ANY"] / cyc, 3),
        "units": "SQ_WAVE_CYCLES/SQ_WAIT_*/SQ_ACTIVE_INST_* in quad-cycles (wave_cycles is x4); "
                 "SQ_INSTS_* are instruction counts; medians over launches, / SQ_WAVES",
    }
    s = json.dumps(out, indent=1)
    print(s)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
