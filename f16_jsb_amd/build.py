"""In-tree build of libf16env.so for gfx950 (hipcc cross-compiles without a GPU).

    python -m f16_jsb_amd.build [--verbose]
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "f16env.hip")
OUT = os.path.join(HERE, "libf16env.so")
# debug build: the same kernels with the F16_CHECK index / range invariants
# compiled in (f16_device.h), read back by f16env_debug_checks; tests load it by F16ENV_LIB
OUT_DEBUG = os.path.join(HERE, "libf16env_debug.so")
# miscompile guard (test only): the same source at -O1 -- other instruction selection, scheduling
# and register allocation, the same rounding (-ffp-contract=on fixes contraction per source
# expression) -- compared bit for bit against the product by tests/test_gpu_o1_differential.py
OUT_O1 = os.path.join(HERE, "libf16env_o1.so")
DEPS = [SRC, os.path.join(HERE, "csrc", "f16_device.h"), os.path.join(HERE, "csrc", "f16_tables.h"),
        os.path.join(ROOT, "include", "f16env.h")]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def build(verbose: bool = False, force: bool = False, extra=(), debug: bool = False, o1: bool = False,
          out: str | None = None) -> str:
    """out: another library path (A/B variants, tools/ab_builds.py); default the product's."""
    out = out or (OUT_DEBUG if debug else (OUT_O1 if o1 else OUT))
    if debug:
        extra = tuple(extra) + ("-DF16_DEBUG_CHECKS",)
    if o1:
        extra = tuple(extra) + ("-O1",)  # after the -O3 below: the last -O wins
    if not force and os.path.exists(out):
        t_out = os.path.getmtime(out)
        if all(os.path.getmtime(d) <= t_out for d in DEPS):
            return out
    # -fno-slp-vectorize: packed-f32 pairing costs more v_mov than it saves at one wave/SIMD.
    # kernarg preload (gfx950): the first 8 argument dwords arrive in SGPRs at wave start; the
    # windowed step kernels take their prologue's addresses there (StepPre): 65 536 envs kernel
    # 16.51 -> 16.19 us (two same-box A/Bs, profiles/r02_variants_preload.txt)
    # -ffp-contract=on: a*b+c is fused per source expression by the front end (llvm.fmuladd),
    # not by the backend's per-kernel pattern matching, so every template instance rounds the
    # same expression the same way: the contiguous and windowed layouts and the one- / two-
    # waves-per-SIMD builds are bit-identical (with =fast, HIP's default, a cfg5 lane in 65 536
    # diverged by step 4 between layouts; step kernel time unchanged, tools/diag/con_ab.sh)
    cmd = [hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=on", "-shared", "-fPIC",
           "-fno-slp-vectorize",
           "-mllvm", "-amdgpu-kernarg-preload-count=8",
           "-I", os.path.join(ROOT, "include"), "-Wno-unused-value", "-Wno-unused-result",
           SRC, "-o", out + ".tmp", *extra]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(verbose="--verbose" in sys.argv, force="--force" in sys.argv, debug="--debug" in sys.argv,
                o1="--o1" in sys.argv))
