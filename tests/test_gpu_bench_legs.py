"""bench.py's side legs: the cfg4 rollout leg runs green at a small size with
the MLP policy in the loop and the deferred bootstrap, and a failing leg keeps the headline line
but is named in `legs_failed` and makes bench.py exit non-zero."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--envs", "4096", "--rollout-envs", "2048", "--rollout-steps", "32", "--policy-steps", "16",
         "--burn-in", "8", "--no-cpu-baseline"]


@pytest.mark.gpu
def test_rollout_leg_small(gpu, monkeypatch):
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py", *SMALL])
    args = bench.parse()
    r = bench.rollout_bench(args, gpu, 0, 1)
    assert "error" not in r
    assert r["rollout_env_steps_per_s"] > 0 and r["rollout_fused_steps_env_steps_per_s"] > 0
    pol = r["policy_in_the_loop"]
    assert pol["steps"] == 16 and np.isfinite(pol["env_steps_per_s"]) and pol["env_steps_per_s"] > 0
    assert "deferred" in pol["policy"]
    assert np.isfinite(pol["bootstrap_per_step"]["env_steps_per_s"])
    assert 0 < r["gae_kernel_ms"] and r["gather_s"] is None


def _bench(extra, timeout=900):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "2", *SMALL, *extra],
                       capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    return p, (json.loads(lines[-1]) if lines else None)


@pytest.mark.gpu
def test_forced_leg_failure_exits_nonzero(gpu):
    p, d = _bench(["--fail-leg", "rollout"])
    assert p.returncode == 1, p.stderr[-3000:]
    assert d is not None, "the headline line must still be printed"
    assert d["legs_failed"] == ["rollout"]
    assert "forced failure" in d["rollout"]["error"]
    assert d["value"] > 0 and d["n_gpus"] == 1
