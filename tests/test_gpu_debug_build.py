"""SURVEY.md S5 "a debug build with bounds checks": the bounds-checked build of the kernels
(libf16env_debug.so, F16_DEBUG_CHECKS: index / range invariants recorded as bits of a device
word, never a trap) runs every kernel family over edge cases in a child process
(tests/debug_build_run.py, F16ENV_LIB pointing at it) and must record no violation. The
product library answers that it carries no checks."""
from __future__ import annotations

import ctypes
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_debug_build_records_no_violation(gpu):
    from f16_jsb_amd.build import OUT_DEBUG
    assert os.path.exists(OUT_DEBUG), "build it: python -m f16_jsb_amd.build --debug (or __graft_entry__.build())"
    env = dict(os.environ, F16ENV_LIB=OUT_DEBUG)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "debug_build_run.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print(res)
    assert res["is_debug"] == 1
    assert res["violations"] == 0, "debug build recorded invariant violations: bits %#x" % res["violations"]
    assert len(res["ran"]) >= 9


def test_product_build_carries_no_checks(gpu):
    from f16_jsb_amd._lib import lib
    v = ctypes.c_uint32(7)
    from f16_jsb_amd.env import F16Envs
    e = F16Envs(64, stack_k=4)
    assert lib().f16env_debug_checks(e._h, None, ctypes.byref(v)) == 0 and v.value == 0
    e.close()
