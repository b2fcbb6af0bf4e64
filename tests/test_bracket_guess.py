"""The guess-and-correct table bracket (f16_device.h bracket_guess, round 5) against FGTable's
segment search (the count of interior breakpoints below x, f16_device.h bracket / oracle
f16ref.c): a numpy float32 emulation of the device arithmetic over every float within 3000 ulps
of each breakpoint, a million uniform samples and the infinities, for the alpha, beta13 and union
Mach grids of the aerodynamic tables (f16.xml:1011-1036, 1421-1447, 1037-1767). CPU only."""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
f32 = np.float32


def _bp(name):
    src = open(os.path.join(ROOT, "f16_jsb_amd", "csrc", "f16_tables.h")).read()
    m = re.search(r"static constexpr float %s\[(\d+)\] = \{([^}]*)\};" % name, src)
    return np.array([float(v.strip().rstrip("f")) for v in m.group(2).split(",")], dtype=np.float32)


def _fma32(a, b, c):
    # float32 fma: the float64 product of two float32 values is exact; one rounding of the sum
    return (np.float64(a) * np.float64(b) + np.float64(c)).astype(np.float32)


def _count_segment(bp, x):
    n = len(bp)
    return (bp[1:n - 1][None, :] < x[:, None]).sum(axis=1)  # 0-based segment


def _guess_segment(bp, x, u):
    n = len(bp)
    g = np.clip(np.nan_to_num(u, nan=0.0, posinf=n - 3, neginf=0.0), 0, n - 3).astype(np.int64)
    up = x > bp[g + 1]
    return g + up


def _samples(bp):
    xs = [np.random.default_rng(1).uniform(-3, 5, 1_000_000).astype(np.float32)]
    for b in bp:
        k = np.arange(-3000, 3001)
        xs.append((np.float32(b).view(np.int32) + k).astype(np.int32).view(np.float32) if b > 0 else
                  np.float32(b) + (k * np.float32(1e-9)).astype(np.float32))
        xs.append(np.array([b, np.nextafter(b, f32(-9)), np.nextafter(b, f32(9))], dtype=np.float32))
    xs.append(np.array([np.inf, -np.inf, 3e38, -3e38, 0.0, -0.0], dtype=np.float32))
    return np.concatenate(xs).astype(np.float32)


@pytest.mark.parametrize("name", ["BP_alpha_bp", "BP_beta13_bp"])
def test_uniform_guess_matches_count(name):
    bp = _bp(name)
    n = len(bp)
    h = (float(bp[-1]) - float(bp[0])) / (n - 1)
    ginv, c0 = f32(1.0 / h), f32(-(float(bp[0]) + 0.5 * h) / h)
    x = _samples(bp)
    u = _fma32(x, ginv, c0)
    np.testing.assert_array_equal(_guess_segment(bp, x, u), _count_segment(bp, x))


def test_machu_guess_matches_count():
    bp = _bp("BP_machu")
    assert len(bp) == 13
    x = _samples(bp)
    xm = np.fmin(x, f32(4.0))  # fminf: the non-NaN operand
    u = _fma32(xm, f32(10.0), f32(-4.5))
    u = (u + np.where(xm > f32(0.805), f32(1.0), f32(0.0))).astype(np.float32)
    u = _fma32(f32(-5.0), np.maximum((xm - f32(1.2)).astype(np.float32), f32(0.0)), u)
    np.testing.assert_array_equal(_guess_segment(bp, x, u), _count_segment(bp, x))
