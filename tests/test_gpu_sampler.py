"""ABI 6 (round 6) on the GPU: the multi-step action sampler and the deferred-reset query.

* f16env_sample_actions_steps: T batches in one launch are bit-identical to T single
  f16env_sample_actions launches and to the oracle's Philox stream (action_space.sample() per
  env, jsbsim_gym.py:143-148), at a ragged env count with a nonzero env_id_base;
* f16env_window_resets_deferred: a cfg5 handle on the deferred-reset step (F16ENV_ICC_PERIOD=0)
  reads 1 and refuses fused_poses / fused_features at construction; the default
  handles read 0."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle_ref import OracleEnvs  # noqa: E402


@pytest.mark.parametrize("n,T", [(1000, 7), (65536, 3), (1, 5)])
def test_sample_actions_steps_matches_single_launches(gpu, n, T):
    import torch
    from f16_jsb_amd.env import F16Envs
    e = F16Envs(n, stack_k=4, seed=2, env_id_base=4321)
    many = e.sample_actions(99, 2**33 + 17, steps=T)
    single = torch.stack([e.sample_actions(99, 2**33 + 17 + t) for t in range(T)])
    torch.cuda.synchronize()
    assert torch.equal(many, single)
    ref = OracleEnvs(n, stack_k=1, env_id_base=4321)
    for t in (0, T - 1):
        np.testing.assert_array_equal(many[t].cpu().numpy(), ref.sample_actions(99, 2**33 + 17 + t))
    # a preallocated output and the shape check
    out = torch.empty((T, n, 4), dtype=torch.float32, device=gpu)
    assert e.sample_actions(99, 2**33 + 17, out=out, steps=T) is out
    assert torch.equal(out, many)
    with pytest.raises(ValueError):
        e.sample_actions(99, 0, out=torch.empty((T + 1, n, 4), dtype=torch.float32, device=gpu), steps=T)
    e.close()
    ref.close()


def test_resets_deferred_query_and_fused_refusal(gpu, monkeypatch):
    from f16_jsb_amd._lib import lib
    from f16_jsb_amd.env import F16Envs
    for kw in (dict(), dict(cfg5=True), dict(cfg5=True, autoreset=False)):
        e = F16Envs(256, stack_k=4, seed=1, obs_layout="window", **kw)
        assert lib().f16env_window_resets_deferred(e._h) == 0, kw
        e.close()
    monkeypatch.setenv("F16ENV_ICC_PERIOD", "0")
    e = F16Envs(256, stack_k=4, seed=1, obs_layout="window", cfg5=True)
    assert lib().f16env_window_resets_deferred(e._h) == 1
    e.close()
    for fused in ("fused_poses", "fused_features"):
        with pytest.raises(ValueError, match="deferred-reset"):
            F16Envs(256, stack_k=4, seed=1, obs_layout="window", cfg5=True, **{fused: True})
    # the reference task never defers: the fused handles construct and step
    e = F16Envs(256, stack_k=4, seed=1, obs_layout="window", fused_poses=True, fused_features=True)
    e.reset()
    e.step(None, seed=3, step=0)
    e.close()
