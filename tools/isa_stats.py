#!/usr/bin/env python3
"""Static ISA statistics of the step kernel (cross-compiled here, no GPU needed).

    python tools/isa_stats.py [-DFLAG ...] [--kernel MANGLED_NAME] [--dump out.s]

(default kernel: the bench headline's f16_step_win_nt_kernel<0, 1, false>)

Prints the kernel's VGPR/AGPR/SGPR-spill counts, the VALU / VMEM / LDS / SALU instruction
counts of the whole kernel and of each loop (the FDM frame loop dominates: it runs
down_sample times per env step), and the most frequent opcodes of the hottest loop.
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


def classify(op: str) -> str:
    if op.startswith("v_accvgpr"):
        return "agpr_mov"
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_waitcnt") or op.startswith("s_nop") or op.startswith("s_barrier"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    # -D/-f flags and -mllvm=OPTION (passed to hipcc as "-mllvm OPTION") go to the compiler
    flags = [a for a in sys.argv[1:] if a.startswith(("-D", "-f"))]
    for a in sys.argv[1:]:
        if a.startswith("-mllvm="):
            flags += ["-mllvm", a[len("-mllvm="):]]
    kernel = "_Z22f16_step_win_nt_kernelILi0ELi1ELb0EEvPK15HIP_vector_typeIfLj4EEPKfS3_l8StepArgs"
    dump = None
    src_asm = None
    args = [a for a in sys.argv[1:] if not a.startswith(("-D", "-f", "-mllvm="))]
    for i, a in enumerate(args):
        if a == "--kernel":
            kernel = args[i + 1]
        if a == "--dump":
            dump = args[i + 1]
        if a == "--from":  # an existing device-assembly dump (hipcc --cuda-device-only -S): no compile
            src_asm = args[i + 1]
    if src_asm:
        analyse(open(src_asm).read().splitlines(), kernel, flags)
        return
    with tempfile.TemporaryDirectory() as td:
        out = dump or os.path.join(td, "k.s")
        # the product library's flags (build.py): contraction per source expression, kernarg preload
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize",
                        "-ffp-contract=on", "-mllvm", "-amdgpu-kernarg-preload-count=8",
                        "-I", os.path.join(ROOT, "include"), "-Wno-unused-value", "-Wno-unused-result",
                        "--cuda-device-only", "-S", SRC, "-o", out, *flags], check=True,
                       stderr=subprocess.DEVNULL)
        lines = open(out).read().splitlines()
    analyse(lines, kernel, flags)


def analyse(lines, kernel, flags):
    start = next(i for i, l in enumerate(lines) if l.startswith(kernel + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    meta = {}
    for l in lines[end:]:
        m = re.match(r"\s+\.set %s\.(num_vgpr|num_agpr|numbered_sgpr|private_seg_size), (\d+)" % re.escape(kernel), l)
        if m:
            meta[m.group(1)] = int(m.group(2))
    # loops: a block label that a later branch targets (back edge)
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"(\.LBB\d+_\d+):", l)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, l in enumerate(body):
        m = re.search(r"s_(?:c)?branch\w*\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))

    def count(seg):
        c = collections.Counter()
        ops = collections.Counter()
        for l in seg:
            m = re.match(r"\s+([a-z_0-9]+)", l)
            if not m or l.strip().startswith(";"):
                continue
            op = m.group(1)
            c[classify(op)] += 1
            ops[op] += 1
        return c, ops

    tot, _ = count(body)
    print("kernel %s %s" % (kernel, " ".join(flags)))
    print("  vgpr %s agpr %s sgpr %s scratch %s" % (meta.get("num_vgpr"), meta.get("num_agpr"),
                                                   meta.get("numbered_sgpr"), meta.get("private_seg_size")))
    print("  whole kernel: " + ", ".join("%s %d" % kv for kv in sorted(tot.items())))
    best = None
    for a, b in loops:
        c, ops = count(body[a:b + 1])
        if c["valu"] < 100:
            continue
        print("  loop lines %d-%d: " % (a, b) + ", ".join("%s %d" % kv for kv in sorted(c.items())))
        if best is None or c["valu"] > best[0]["valu"]:
            best = (c, ops)
    if best:
        print("  hottest loop top opcodes: " + ", ".join("%s %d" % kv for kv in best[1].most_common(24)))


if __name__ == "__main__":
    main()
