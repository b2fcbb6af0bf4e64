"""Static checks of the built gfx950 code object (CPU; no GPU needed).

Round 2 recorded all-zero rewards from f16_step_win_nt_kernel<3, 1> whenever the step kernel
carried a run-time reset path. Round 3 found the cause in the ISA: the shaping term
r += 0.01 (last_d - d) of PositionReward (jsbsim_gym.py:493-507) compiled to
`v_sub_f32 v0, v207, v207` -- the register allocator wrote the new distance into the tuple
register that still held the previous one before reading it (a backend miscompile of ROCm 7.2's
LLVM; the source workaround is in env_reward, f16env.hip). No fp32 source expression of the
library subtracts a value from itself, so any `v_sub_f32 vX, vY, vY` (or `v_add_f32 vX, vY, -vY`)
in the code object is that bug again; the test disassembles every kernel and fails on one.

fp64 `v_add_f64 D, X, -X` does occur legitimately: derive() (f16_device.h) forms
(float)(xE - A.r0[0]) etc. for the altitude advance, and where derive runs at the AltRef's own
reference point (frame 0 of a step, every RunIC pass) both operands are the same value. The
compiler keeps x - x (it is NaN, not 0, for non-finite x), and each such difference is narrowed
by the (float) cast right after. The second test pins that shape: an fp64 self-difference whose
result is not narrowed to fp32 within a few instructions is not derive's and fails.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import tempfile

import pytest

LLVM_OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def _disassemble(so_path: str) -> str:
    d = tempfile.mkdtemp(prefix="f16isa_")
    try:
        lib = os.path.join(d, "lib.so")
        shutil.copy(so_path, lib)
        subprocess.run([LLVM_OBJDUMP, "--offloading", lib], cwd=d, check=True, capture_output=True)
        co = [f for f in os.listdir(d) if "gfx950" in f]
        assert co, "no gfx950 code object in %s" % so_path
        return subprocess.run([LLVM_OBJDUMP, "-d", "--no-show-raw-insn", os.path.join(d, co[0])],
                              check=True, capture_output=True, text=True).stdout
    finally:
        shutil.rmtree(d, ignore_errors=True)


# both shipped code objects: the product and the bounds-checked debug build (its F16_CHECK atomics
# change register allocation, and it is the library soak.py / debug_build_run.py exercise)
BUILDS = [False, True]


@pytest.mark.skipif(not os.path.exists(LLVM_OBJDUMP), reason="ROCm llvm-objdump not present")
@pytest.mark.parametrize("debug", BUILDS, ids=["product", "debug"])
def test_no_self_subtraction_in_step_kernels(debug):
    from f16_jsb_amd.build import build
    asm = _disassemble(build(debug=debug))
    kernel = None
    bad = []
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            kernel = m.group(1)
            continue
        if (re.search(r"\bv_sub(rev)?_f32(_e32|_e64)?\s+v\d+, (v\d+), \3(\s|$)", line)
                or re.search(r"\bv_add_f32(_e32|_e64)?\s+v\d+, (v\d+), -\2(\s|$)", line)
                or re.search(r"\bv_add_f32(_e32|_e64)?\s+v\d+, -(v\d+), \2(\s|$)", line)
                # the same shape in other operations that no source expression forms on one
                # value: integer x - x / x ^ x (the compiler materialises a 0 as a move), and
                # x < x / x > x compares (x != x is the NaN test, and stays allowed)
                or re.search(r"\bv_(sub|subrev)_(u32|i32|co_u32|nc_u32)(_e32|_e64)?\s+v\d+(, vcc|, s\[\d+:\d+\])?, (v\d+), \5(\s|,|$)", line)
                or re.search(r"\bv_xor_b32(_e32|_e64)?\s+v\d+, (v\d+), \2(\s|$)", line)
                or re.search(r"\bv_cmp_(lt|gt)_f32(_e32|_e64)?\s+(vcc|s\[\d+:\d+\]), (v\d+), \4(\s|$)", line)):
            bad.append((kernel, line.strip()))
    assert not bad, "x - x subtraction(s) in the code object (register-allocation miscompile): %s" % bad[:4]
    # the step kernels are in there at all (the scan saw the real code)
    assert "f16_step_win_nt_kernel" in asm and "f16_step_kernel" in asm


@pytest.mark.skipif(not os.path.exists(LLVM_OBJDUMP), reason="ROCm llvm-objdump not present")
@pytest.mark.parametrize("debug", BUILDS, ids=["product", "debug"])
def test_fp64_self_differences_are_derive_reference_point(debug):
    from f16_jsb_amd.build import build
    lines = _disassemble(build(debug=debug)).splitlines()
    pat = re.compile(r"\bv_add_f64(_e64)?\s+(v\[\d+:\d+\]), (-?)(v\[\d+:\d+\]), (-?)(v\[\d+:\d+\])")
    seen, bad = 0, []
    for i, line in enumerate(lines):
        m = pat.search(line)
        if not m or m.group(4) != m.group(6) or m.group(3) == m.group(5):
            continue
        seen += 1
        # the next instruction that reads the difference must be its narrowing, and it must
        # come before anything overwrites it (scheduling can put many instructions between)
        reg = re.escape(m.group(2))
        cvt = re.compile(r"\bv_cvt_f32_f64(_e32|_e64)?\s+v\d+, " + reg + r"(\s|$)")
        ok = False
        for nxt in lines[i + 1:i + 400]:
            if cvt.search(nxt):
                ok = True
                break
            if re.search(reg, nxt):  # any other read or a redefinition first
                break
        if not ok:
            bad.append(line.strip())
    assert not bad, "fp64 x - x not narrowed to fp32 (not derive's reference-point difference): %s" % bad[:4]
    assert seen > 0  # the pattern matches the disassembler's syntax (derive's are in there)


# ---------------------------------------------------------------------------------------------
# Round 6: the round-5 memory aperture violation. A build whose derive()
# formed the body velocity rows and ground speed with raw `asm("v_pk_fma_f32 ...")` (the PK_FMA /
# PK_MUL macros) faulted in test_persistent_rollout_two_wave_build_matches_fused_steps
# [contiguous-cfg5] -- f16_rollout_kernel<3, 2>, whose in-kernel RunIC ran that code inside a
# 256-register kernel with 468 B of spills. Its ISA (rebuilt from commit 81e0cf8 on the CPU, DESIGN.md
# 8 round 6) passes the three ISA checks below and -verify-machineinstrs, so the faulting access
# was not located; the mechanism is removed instead: no VALU inline asm in the device sources.
CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "f16_jsb_amd", "csrc")
# asm templates the device code may hold: empty (register pinning / compiler barriers) and the
# scalar waits / timers it issues explicitly; anything else -- a VALU, VMEM or LDS instruction
# the compiler cannot see into -- fails
ASM_ALLOWED = re.compile(r'^(|s_waitcnt [a-z0-9() ]+|s_memtime %0\\n\\ts_waitcnt lgkmcnt\(0\))$')


def test_no_valu_inline_asm_in_device_sources():
    bad, seen = [], 0
    for fn in sorted(os.listdir(CSRC)):
        if not fn.endswith((".hip", ".h")):
            continue
        src = open(os.path.join(CSRC, fn)).read()
        for m in re.finditer(r'\basm\s*(?:volatile\s*)?\(\s*"((?:[^"\\]|\\.)*)"', src):
            seen += 1
            if not ASM_ALLOWED.match(m.group(1)):
                line = src.count("\n", 0, m.start()) + 1
                bad.append("%s:%d: %r" % (fn, line, m.group(1)[:60]))
        # a macro that pastes an instruction string into asm (round 5's PK_FMA) is the same thing
        for m in re.finditer(r'#define\s+\w+\([^)]*\)\s+asm\s*\(\s*"([^"]*)"', src):
            if not ASM_ALLOWED.match(m.group(1)):
                bad.append("%s: macro asm %r" % (fn, m.group(1)[:60]))
    assert not bad, "inline asm emitting instructions the compiler cannot schedule or hazard-check: %s" % bad
    assert seen > 0  # the scan sees the register-pinning asm that is there


def _kernels(asm):
    kernel, body = None, []
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            if kernel:
                yield kernel, body
            kernel, body = m.group(1), []
        elif kernel:
            body.append(line.strip())
    if kernel:
        yield kernel, body


def _regs(text):
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", text):
        out.update([int(m.group(3))] if m.group(3) else range(int(m.group(1)), int(m.group(2)) + 1))
    return out


@pytest.mark.skipif(not os.path.exists(LLVM_OBJDUMP), reason="ROCm llvm-objdump not present")
@pytest.mark.parametrize("debug", BUILDS, ids=["product", "debug"])
def test_packed_pairs_and_sgpr_spill_lanes(debug):
    """Two of the round-6 checks of the faulting build, kept on the shipped code objects:
    (1) every packed fp32 instruction's 64-bit operands are even-aligned register pairs and its
    destination does not partially overlap a source; (2) a VGPR that holds spilled SGPRs in its
    lanes (v_writelane / v_readlane) is written by nothing but v_writelane in that kernel."""
    asm = _disassemble(build_lib(debug))
    bad, pk = [], 0
    for kernel, body in _kernels(asm):
        lanes = set()
        for ln in body:
            m = re.match(r"v_(?:writelane|readlane)_b32 (\S+), (\S+),", ln)
            if m:
                lanes |= _regs(m.group(1) if ln.startswith("v_writelane") else m.group(2))
        for ln in body:
            if ln.startswith("v_pk_") and "f32" in ln:
                pk += 1
                ops = [o.strip() for o in ln.split(None, 1)[1].split(",")]
                pairs = [re.match(r"-?\|?v\[(\d+):(\d+)\]", o) for o in ops]
                if any(p and int(p.group(1)) % 2 for p in pairs):
                    bad.append((kernel, "odd pair", ln))
                d = pairs[0]
                if d:
                    dl, dh = int(d.group(1)), int(d.group(2))
                    for p in pairs[1:]:
                        if p and (int(p.group(1)), int(p.group(2))) != (dl, dh) and not (
                                int(p.group(2)) < dl or int(p.group(1)) > dh):
                            bad.append((kernel, "partial overlap", ln))
            if lanes and not ln.startswith(("v_writelane", "v_readlane")) and ln.startswith("v_"):
                first = ln.split(None, 1)[1].split(",")[0] if " " in ln else ""
                if _regs(first) & lanes:
                    bad.append((kernel, "spill-lane VGPR written", ln))
    assert not bad, bad[:6]
    assert pk > 0  # the packed table blends are in there


def build_lib(debug):
    from f16_jsb_amd.build import build
    return build(debug=debug)


@pytest.mark.skipif(not os.path.exists(LLVM_OBJDUMP), reason="ROCm llvm-objdump not present")
def test_step_prologue_issues_its_loads_before_any_wait():
    """Round 6 ("The step's prologue"): past the argument-preload entry, the headline
    step kernels issue the table LDS-DMA and all 16 state-column loads before their first
    s_waitcnt. The kernel-argument round trip (~1 us per launch) then overlaps the state's instead
    of preceding it; round 5's code waited for the whole argument block first (the table staging
    strode by blockDim.x, an implicit-argument load), 0.65 us per step at 65 536 envs."""
    asm = _disassemble(build_lib(False))
    # (the headline kernel only: cfg5's 256-register <3, 2> build and the rollout-slot build still
    # wait once before their state loads -- two EnvArgs fields they load up front are spilled to
    # VGPR lanes at once, and the spill needs the value; measured neutral to remove for the
    # rollout slot's action-flag read, profiles/r06_ab_action_pointer.json)
    want = {"_Z22f16_step_win_nt_kernelILi0ELi1ELb0EEvPK15HIP_vector_typeIfLj4EEPKfS3_l8StepArgs": "cfg3 headline"}
    seen = set()
    for kernel, body in _kernels(asm):
        if kernel not in want:
            continue
        seen.add(kernel)
        # the compatibility prologue (argument loads for firmware without preload) ends in the
        # first s_branch; the preloaded entry follows it
        i = next(j for j, ln in enumerate(body) if ln.startswith("s_branch"))
        dma = state = 0
        for ln in body[i + 1:]:
            if ln.startswith("global_load_lds_dwordx4"):
                dma += 1
            elif ln.startswith("global_load_dwordx4"):
                state += 1
                if state == 16:
                    break
            elif ln.startswith("s_waitcnt") or ln.startswith("s_barrier"):
                pytest.fail("%s: %r before the 16 state loads (%d issued, %d table DMAs)"
                            % (want[kernel], ln, state, dma))
        assert state == 16 and dma >= 1, (want[kernel], state, dma)
    assert seen == set(want), sorted(set(want) - seen)
