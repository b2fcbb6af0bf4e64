#!/usr/bin/env python3
"""Register / scratch / LDS use of every kernel in a built library (CPU, no GPU needed).

    python tools/kernel_resources.py [lib.so] [--filter SUBSTR]

Reads the gfx950 code object's AMDGPU metadata note (llvm-readelf --notes): per kernel the
VGPR / AGPR / SGPR counts, private (scratch) bytes per lane and static LDS bytes -- spills show
up as scratch > 0.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def code_object(so_path: str, d: str) -> str:
    lib = os.path.join(d, "lib.so")
    shutil.copy(so_path, lib)
    subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", lib], cwd=d, check=True, capture_output=True)
    co = [f for f in os.listdir(d) if "gfx950" in f]
    if not co:
        raise SystemExit("no gfx950 code object in %s" % so_path)
    return os.path.join(d, co[0])


def resources(so_path: str):
    d = tempfile.mkdtemp(prefix="f16res_")
    try:
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", code_object(so_path, d)],
                               check=True, capture_output=True, text=True).stdout
    finally:
        shutil.rmtree(d, ignore_errors=True)
    out, cur = [], None
    for line in notes.splitlines():
        s = line.strip()
        m = re.match(r"- \.agpr_count:\s+(\d+)", s)
        if m:
            cur = {"agpr": int(m.group(1))}
            out.append(cur)
            continue
        if cur is None:
            continue
        for key, name in ((".vgpr_count", "vgpr"), (".sgpr_count", "sgpr"), (".private_segment_fixed_size", "scratch"),
                          (".group_segment_fixed_size", "lds"), (".vgpr_spill_count", "vgpr_spill"),
                          (".sgpr_spill_count", "sgpr_spill")):
            m = re.match(re.escape(key) + r":\s+(\d+)", s)
            if m:
                cur[name] = int(m.group(1))
        m = re.match(r"\.name:\s+(\S+)", s)
        if m and "name" not in cur:
            cur["name"] = m.group(1)
    return out


def demangle(names):
    p = subprocess.run([shutil.which("c++filt") or "c++filt"], input="\n".join(names), capture_output=True, text=True)
    return p.stdout.splitlines() if p.returncode == 0 else names


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    flt = None
    if "--filter" in sys.argv:
        flt = sys.argv[sys.argv.index("--filter") + 1]
        args = [a for a in args if a != flt]
    so = args[0] if args else os.path.join(ROOT, "f16_jsb_amd", "libf16env.so")
    rows = resources(so)
    names = demangle([r.get("name", "?") for r in rows])
    for r, n in sorted(zip(rows, names), key=lambda x: x[1]):
        if flt and flt not in n:
            continue
        print("%-70s vgpr %3d agpr %3d sgpr %3d scratch %4d lds %6d spill v%d s%d" % (
            n[:70], r.get("vgpr", -1), r.get("agpr", -1), r.get("sgpr", -1), r.get("scratch", -1), r.get("lds", -1),
            r.get("vgpr_spill", -1), r.get("sgpr_spill", -1)))


if __name__ == "__main__":
    main()
