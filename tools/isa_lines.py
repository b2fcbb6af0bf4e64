#!/usr/bin/env python3
"""Where the frame loop's VALU instructions come from (cross-compiled here, no GPU needed).

    python tools/isa_lines.py [-DFLAG ...] [--kernel MANGLED_NAME] [--top 40]

Compiles the device code with the product library's flags plus -gline-tables-only (line tables
do not change code generation), finds the kernel's FDM frame loop (the innermost loop with
800-1000 VALU instructions, as tools/isa_stats.py reports it) and attributes each VALU
instruction to the source line of its `.loc` directive (the innermost inlined location) and to
the device function that line belongs to. DESIGN.md section 9 quotes its output.
"""
from __future__ import annotations

import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "f16_jsb_amd", "csrc", "f16env.hip")
KERNEL = "_Z22f16_step_win_nt_kernelILi0ELi1ELb0EEvPK15HIP_vector_typeIfLj4EEPKfS3_l8StepArgs"
SOURCES = {"f16env.hip": "f16_jsb_amd/csrc/f16env.hip", "f16_device.h": "f16_jsb_amd/csrc/f16_device.h"}


def is_valu(line: str) -> bool:
    t = line.strip().split()
    return bool(t) and t[0].startswith("v_") and not t[0].startswith("v_accvgpr")


def frame_loop(body):
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    best = None
    for i, l in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", l)
        if not m:
            continue
        t = m.group(1) or m.group(2)
        if t in labels and labels[t] < i:
            a, b = labels[t], i
            n = sum(1 for x in body[a:b] if is_valu(x))
            if 800 <= n <= 1000 and (best is None or b - a < best[1] - best[0]):
                best = (a, b, n)
    return best


def func_of(cache, fname, line):
    path = SOURCES.get(fname)
    if not path:
        return fname
    if path not in cache:
        cache[path] = open(os.path.join(ROOT, path)).read().splitlines()
    src = cache[path]
    for j in range(min(line - 1, len(src) - 1), -1, -1):
        m = re.match(r"^(?:template.*)?__device__.*?(\w+)\s*\(", src[j])
        if m:
            return m.group(1)
    return "?"


def main():
    flags = [a for a in sys.argv[1:] if a.startswith("-D")]
    kernel = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else KERNEL
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize",
                        "-ffp-contract=on", "-mllvm", "-amdgpu-kernarg-preload-count=8", "-I", os.path.join(ROOT, "include"),
                        "-Wno-unused-value", "-Wno-unused-result", "--cuda-device-only", "-S", "-gline-tables-only",
                        SRC, "-o", out, *flags], check=True, stderr=subprocess.DEVNULL)
        lines = open(out).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(kernel + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    files = {}
    for l in lines[:start]:
        m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]*)"', l)
        if m:
            files[int(m.group(1))] = os.path.basename(m.group(2))
    body = lines[start:end]
    loop = frame_loop(body)
    if loop is None:
        sys.exit("no frame loop (800-1000 VALU) found in %s" % kernel)
    a, b, n = loop
    print("kernel %s %s\n  frame loop: %d VALU" % (kernel, " ".join(flags), n))
    cache, cur = {}, None
    per_func, per_line = collections.Counter(), collections.Counter()
    for l in body[a:b]:
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            cur = (files.get(int(m.group(1)), "?"), int(m.group(2)))
            continue
        if is_valu(l):
            per_func[func_of(cache, *cur) if cur else "?"] += 1
            per_line[cur] += 1
    print("  by function:")
    for f, c in per_func.most_common(top):
        print("  %5d  %s" % (c, f))
    print("  by source line:")
    for (f, ln), c in per_line.most_common(top):
        print("  %5d  %s:%d" % (c, f, ln))


if __name__ == "__main__":
    main()
