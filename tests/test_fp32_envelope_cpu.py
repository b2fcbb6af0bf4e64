"""The fp32 envelope machinery on the CPU (tests/fp32_envelope.py; the GPU comparison is
tests/test_gpu_fp32_envelope.py): the get_state / set_state control leaves the oracle's
trajectory bit-identical over the compared horizon, the perturbed variants are perturbed, and
their divergence grows with the horizon -- the yardstick the HIP path's divergence is held to."""
from __future__ import annotations

import numpy as np
import pytest

from fp32_envelope import F32_FIELDS, one_ulp, run, to_f32_storage


@pytest.mark.parametrize("cfg5", [False, True], ids=["reference_task", "cfg5"])
def test_envelope_control_is_exact_and_perturbations_grow(cfg5):
    out = run(n=64, steps=100, horizons=(1, 10, 30, 100), cfg5=cfg5)
    for t in (1, 10, 30, 100):
        d = out["control"][t]
        assert d["lanes"] == 64
        assert all(d[c][2] == 0.0 for c in d if c != "lanes"), (t, d)
    for v in ("ulp1", "round"):
        h10, h100 = out[v][10]["h_m"][1], out[v][100]["h_m"][1]
        a10, a100 = out[v][10]["alpha"][1], out[v][100]["alpha"][1]
        assert h100 > h10 and a100 > a10 > 0.0, (v, out[v])


def test_state_perturbations_touch_only_fp32_fields():
    from oracle_ref import OracleEnvs
    e = OracleEnvs(8, stack_k=4, seed=5)
    e.reset()
    for _ in range(3):
        e.step(e.sample_actions(99, 0))
    s = e.get_state()
    e.close()
    r = to_f32_storage(s)
    u = one_ulp(s, np.random.default_rng(0))
    others = np.setdiff1d(np.arange(s.shape[1]), F32_FIELDS)
    # fp32 storage: the fp64 fields (ECI position / velocity, Earth angle, episode return) are kept,
    # except the AB3 velocity history, which becomes fp32 deltas from the fp64 velocity
    keep = np.setdiff1d(others, np.r_[6:12])
    np.testing.assert_array_equal(r[:, keep], s[:, keep])
    np.testing.assert_array_equal(r[:, F32_FIELDS], s[:, F32_FIELDS].astype(np.float32).astype(np.float64))
    np.testing.assert_array_equal(u[:, others], s[:, others])
    f = s[:, F32_FIELDS].astype(np.float32)
    moved = u[:, F32_FIELDS].astype(np.float32)
    up, dn = np.nextafter(f, np.float32(np.inf)), np.nextafter(f, np.float32(-np.inf))
    assert np.all((moved == up) | (moved == dn))  # one fp32 ulp either way (through 0 too)
