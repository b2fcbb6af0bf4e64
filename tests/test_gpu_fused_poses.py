"""Pose export in the plain step's epilogue (F16Envs(fused_poses=True), f16env_window_step_ex with
F16_STEP_POSES, ABI 5): after every step the bound (N, 10) buffer must equal, bit for bit, the
separate pose kernel over the returned observation's newest frame (telemetry.poses, f16env_poses:
JSBSimEnv.render, jsbsim_gym.py:381-415, itself checked against the numpy restatement in
tests/test_telemetry.py) -- with caller actions and in-kernel actions, with the fused feature
window on or off, through in-kernel auto-resets (short TimeLimits, cfg5 cache resets), window
restarts (short histories), both window orders and a partial last wave."""
from __future__ import annotations

import pytest

pytestmark = pytest.mark.gpu

CASES = [
    dict(n=1000, k=4, T=9, order="position", max_steps=5, cfg5=False, feat=False),
    dict(n=1000, k=4, T=9, order="position", max_steps=5, cfg5=False, feat=True),
    dict(n=257, k=10, T=21, order="env", max_steps=7, cfg5=False, feat=False),
    dict(n=513, k=3, T=7, order="position", max_steps=4, cfg5=True, feat=True),
    dict(n=4096, k=4, T=64, order="position", max_steps=1200, cfg5=False, feat=False),
]


@pytest.mark.parametrize("c", CASES, ids=["n%d_k%d_%s%s%s" % (c["n"], c["k"], c["order"], "_cfg5" if c["cfg5"] else "",
                                                            "_feat" if c["feat"] else "") for c in CASES])
def test_fused_poses_equal_pose_kernel(gpu, c):
    import torch
    from f16_jsb_amd import telemetry
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.features import features
    n, k = c["n"], c["k"]
    e = F16Envs(n, stack_k=k, seed=5, max_steps=c["max_steps"], cfg5=c["cfg5"], obs_layout="window",
                history=c["T"], window_order=c["order"], fused_poses=True, fused_features=c["feat"])
    e.reset()
    resets = 0
    for t in range(40):
        if t % 3 == 2:
            out = e.step(None, seed=9, step=t)  # in-kernel actions
        else:
            out = e.step(e.sample_actions(seed=9, step=t))
        resets += int((out.terminated | out.truncated).sum().item())
        assert e._poses_op == e._op, "the step should have written the pose export"
        fused = e.poses()
        assert fused.data_ptr() == e._poses.data_ptr()
        ref = telemetry.poses(e.obs)
        torch.cuda.synchronize()
        assert torch.equal(fused, ref), "step %d" % t
        if c["feat"] and t % 5 == 4:
            assert torch.equal(e.obs_features(), features(e.obs))
    if c["max_steps"] < 40:
        assert resets > 0, "expected in-kernel auto-resets"
    e.close()


def test_fused_poses_kernel_name_and_refusals(gpu):
    import torch
    from f16_jsb_amd._lib import F16EnvError, lib
    from f16_jsb_amd.abi import F16_STEP_POSES
    from f16_jsb_amd.env import F16Envs
    e = F16Envs(128, stack_k=4, seed=1, obs_layout="window", fused_poses=True)
    e.reset()
    name = lib().f16env_window_step_ex_kernel_name(e._h, F16_STEP_POSES).decode()
    assert name.startswith("f16_step_winx_kernel<") and name.endswith(", 1>"), name
    # unbound: the flag is refused before any launch
    assert lib().f16env_window_poses_bind(e._h, None) == 0
    with pytest.raises(F16EnvError):
        e.step(e.sample_actions(seed=1, step=0))
    e.close()
    with pytest.raises(ValueError):
        F16Envs(16, stack_k=4, obs_layout="contiguous", fused_poses=True)
