"""The C ABI from a C++ host program alone (tests/c_abi/abi_parity.cpp): no Python and no
torch between the caller and libf16env.so. The harness creates a handle with the reference's
configuration (K = 10), owns its device buffers through the HIP runtime, and steps it beside
the CPU oracle for 30 random-action steps with every lane truncating and auto-resetting:
done flags and episode bookkeeping bit-exact, frames within the 30-step random-action
tolerance, rewards within 2e-3, the NULL-handle error path, canonical state export.
(Built by __graft_entry__.build(); a missing binary fails the test rather than skipping it.)"""
from __future__ import annotations

import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "c_abi", "abi_parity")


@pytest.mark.parametrize("n,steps", [(2048, 30), (65537, 13)])
def test_c_abi_parity_from_cpp(gpu, n, steps):
    assert os.path.exists(BIN), "build the harness first: make -C tests/c_abi (part of __graft_entry__.build())"
    r = subprocess.run([BIN, str(n), str(steps)], capture_output=True, text=True, timeout=240)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ABI PARITY OK" in r.stdout
