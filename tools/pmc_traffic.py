#!/usr/bin/env python3
"""Per-launch HBM traffic of f16_step_kernel from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE; separate runs, the TCC block cannot hold both), corrected as
/opt/skills/guides/MI355X_MICROARCH.md (HBM section) prescribes: counters are in KiB and on
gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so it is doubled.

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR --envs 65536 --stack 4 [--out profiles/pmc_traffic.json]
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_launch(d, counter, kernel, grid):
    p = d if d.endswith(".csv") else os.path.join(d, "run_counter_collection.csv")
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(p))
            if r["Kernel_Name"].removeprefix("void ").startswith(kernel) and r["Counter_Name"] == counter and int(r["Grid_Size"]) == grid]
    if not vals:
        raise SystemExit("no %s rows for %s (grid %d) in %s" % (counter, kernel, grid, p))
    return statistics.median(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--stack", type=int, default=4)
    ap.add_argument("--kernel", default="f16_step_win_kernel")
    ap.add_argument("--layout", default="window", choices=("window", "contiguous"))
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--extra-bytes", type=int, default=0,
                    help="per env step on top of the layout's bytes (cfg5: 24, the gust state's read + write, as bench.py)")
    a = ap.parse_args()
    from f16_jsb_amd._lib import lib
    from f16_jsb_amd.abi import algorithmic_bytes_per_env_step
    fetch_kib, nf = per_launch(a.fetch_dir, "FETCH_SIZE", a.kernel, a.envs)
    write_kib, nw = per_launch(a.write_dir, "WRITE_SIZE", a.kernel, a.envs)
    rd = 2.0 * fetch_kib * 1024.0
    wr = write_kib * 1024.0
    state_bytes = int(lib().f16env_state_bytes_per_env())
    alg = (algorithmic_bytes_per_env_step(a.stack, state_bytes) + a.extra_bytes) * a.envs
    lay = (algorithmic_bytes_per_env_step(a.stack, state_bytes, a.layout) + a.extra_bytes) * a.envs  # this layout's
    d = {
        "kernel": a.kernel, "layout": a.layout, "envs": a.envs, "stack_k": a.stack, "state_bytes": state_bytes,
        "extra_bytes_per_env_step": a.extra_bytes,
        "fetch_size_kib_median": fetch_kib, "write_size_kib_median": write_kib, "launches": [nf, nw],
        "hbm_read_bytes_per_launch": int(rd), "hbm_write_bytes_per_launch": int(wr),
        "hbm_bytes_per_launch": int(rd + wr),
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": round((rd + wr) / alg, 4),
        "layout_bytes_per_launch": lay,
        "traffic_over_layout_bytes": round((rd + wr) / lay, 4),
        "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB -> bytes; WRITE_SIZE as read",
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
