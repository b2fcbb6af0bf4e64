"""Miscompile guard, differential.

Round 3's all-zero rewards were a register-allocation miscompile of ROCm 7.2's AMDGPU backend
in a few kernel instances (f16env.hip env_reward), found in the ISA; tests/test_isa_lint.py
catches that bug's shape (an fp32 x - x). A recurrence of another shape would pass the lint and
could pass the oracle tolerances if every instance miscompiled alike. Here the same source is
built a second way -- libf16env_o1.so at -O1: other instruction selection, scheduling and
register allocation; the same rounding, which the source fixes (-ffp-contract=on, explicit
FMAs) -- and the bounds-checked debug build a third (its check atomics change allocation
again). tests/o1_diff_run.py runs every kernel family on identical inputs under each library in
a child process; the outputs must agree bit for bit."""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(lib_path, out):
    # AMD_SERIALIZE_KERNEL=3: every launch waits for its kernel, so a device fault is reported at
    # the call that launched the faulting kernel (and the child's last "phase" line names its
    # section) instead of at a later synchronisation
    env = dict(os.environ, F16ENV_LIB=lib_path, AMD_SERIALIZE_KERNEL="3")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "o1_diff_run.py"), out], env=env,
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, "%s\n--- stdout tail:\n%s\n--- stderr tail:\n%s" % (
        os.path.basename(lib_path), r.stdout[-600:], r.stderr[-3000:])
    return dict(np.load(out))


def test_o1_and_debug_builds_bit_identical_to_product(gpu):
    from f16_jsb_amd.build import OUT, OUT_DEBUG, OUT_O1
    for p in (OUT_O1, OUT_DEBUG):
        assert os.path.exists(p), "build it: python -m f16_jsb_amd.build --o1 / --debug (or __graft_entry__.build())"
    with tempfile.TemporaryDirectory() as d:
        prod = _run(OUT, os.path.join(d, "prod.npz"))
        for name, path in (("-O1", OUT_O1), ("debug", OUT_DEBUG)):
            other = _run(path, os.path.join(d, "other.npz"))
            assert sorted(other) == sorted(prod)
            diff = [k for k in prod if not np.array_equal(prod[k], other[k], equal_nan=True)]
            assert not diff, "%s build differs from the product in %s" % (name, diff[:8])
    # the workload exercised what it should: resets, rewards, clipping policy, cfg5 resets
    assert prod["ref_window_occ1_flags"].any() and prod["cfg5_window_occ2_flags"].any()
    assert np.abs(prod["roll_window_actions"]).max() > 1.0
    assert np.isfinite(prod["roll_window_cfg5_advantages"]).all()
