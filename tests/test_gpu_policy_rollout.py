"""Device rollouts with the policy in the loop and on the windowed layout.

The reference's collector is on_policy_algorithm.py:194-262:
  actions, values, log_probs = policy(obs)            (:202)
  env.step(np.clip(actions, low, high))               (:216-218)
  rewards[i] += gamma * V(terminal_obs[i]) for lanes that ended by truncation only (:236-245)
  rollout_buffer.add(obs, actions (UNCLIPPED), rewards, episode_starts, values, log_probs) (:247-254)
  last values V(new_obs) -> compute_returns_and_advantage (:258-262, buffers.py:403-438)

collect_rollout(policy_fn=...) does that with one windowed rollout-step launch per step
(f16env_window_step_rollout: the clip in-kernel, the slot's unclipped actions / rewards / next
starts / next frame written by the step kernel) and f16env_bootstrap_timeouts. Checked here:
  * at cfg4's per-GPU share (32 768 envs, K = 4), with a deterministic torch policy whose
    actions leave the Box, 30 steps against the oracle stepping np.clip of the same actions:
    stored actions / values / log-probs equal the policy's outputs bit for bit, done flags and
    episode starts bit-exact, raw rewards 2e-3, slot frames TOL_RAND30, the bootstrapped
    rewards bit-exact against a numpy restatement of :236-245 on the step's raw rewards and
    terminal values, and the GAE bit-exact against buffers.py:403-438 restated in numpy;
  * the windowed fused rollout is bit-identical to the contiguous one, and the persistent
    rollout (one launch, f16env_rollout_random / f16env_window_rollout_random) to the fused
    steps, at K = 4 and the reference's K = 10, in the reference task and cfg5 (random ICs +
    gusts);
  * the persistent windowed rollout against the oracle at K = 10 and in cfg5.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle_ref import OracleEnvs, default_ic  # noqa: E402
from reward_bound import reward_atol  # noqa: E402
from test_gpu_parity import TOL_RAND30, TOL_STEP, _assert_frames, _random_ics  # noqa: E402
from test_gpu_production import _assert_frames_stat, _stagger  # noqa: E402
from test_gpu_rollout import numpy_gae  # noqa: E402

LOW = np.array([-1, -1, -1, 0], np.float32)
HIGH = np.array([1, 1, 1, 1], np.float32)


def _policy(dev, env=None):
    """A deterministic policy(obs) -> (actions, values, log_probs) on the newest frame; about a
    third of its actions leave the Box. value(obs) is its value head alone. Records its outputs
    and, for the value calls, the env's raw step outputs at that moment."""
    import torch
    rng = np.random.default_rng(17)
    W = torch.as_tensor(rng.normal(size=(9, 4)).astype(np.float32) * 0.7, device=dev)
    b = torch.tensor([0.0, 0.1, 0.0, 0.5], device=dev)
    Wv = torch.as_tensor(rng.normal(size=(9, 1)).astype(np.float32), device=dev)
    rec, vrec = [], []

    def feats(obs):
        x = obs[:, -1, :]
        return torch.stack([x[:, 4] * 8, x[:, 5] * 8, x[:, 6], x[:, 7], x[:, 8], x[:, 9], x[:, 10],
                            (x[:, 2] - 1500.0) / 3000.0, x[:, 3] - 0.8], 1)

    def policy(obs):
        z = feats(obs)
        a = (z @ W + b).contiguous()
        v = (z @ Wv).reshape(-1)
        lp = -(a * a).sum(1)
        rec.append((a.clone(), v.clone(), lp.clone()))
        return a, v, lp

    def value(obs):
        v = (feats(obs) @ Wv).reshape(-1)
        if env is not None:
            vrec.append((v.clone(), env.rew.clone(), env.term.clone(), env.trunc.clone(), obs[:, -1].clone()))
        return v

    return policy, value, rec, vrec


def test_policy_rollout_cfg4_share_vs_oracle(gpu):
    import torch
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout
    N, K, T, SEED, GAMMA = 32768, 4, 30, 91, 0.99
    rng = np.random.default_rng(4)
    ic = _random_ics(N, rng)
    goals = rng.uniform(-5000, 5000, (N, 3)).astype(np.float32)
    goals[:, 2] = np.abs(goals[:, 2])
    ref = OracleEnvs(N, stack_k=K, seed=SEED)
    g = F16Envs(N, stack_k=K, seed=SEED, obs_layout="window")
    o = ref.reset(goals=goals, ic=ic)
    g.reset(goals=goals, ic=ic)
    _stagger(ref, g, o, span=25)  # a third of the lanes truncate inside the 30 steps
    policy, value, rec, vrec = _policy(gpu, g)
    buf = DeviceRolloutBuffer(T, N, K, gpu, gamma=GAMMA)
    last_v, last_d = collect_rollout(g, buf, seed=SEED, policy_fn=policy, value_fn=value, bootstrap="per_step")
    torch.cuda.synchronize()
    assert len(rec) == T and len(vrec) == T + 1
    fr, ac, rw = buf.frames.cpu().numpy(), buf.actions.cpu().numpy(), buf.rewards.cpu().numpy()
    st, vals, lps = buf.episode_starts.cpu().numpy(), buf.values.cpu().numpy(), buf.log_probs.cpu().numpy()
    o_prev = o
    clipped_any = boot = 0
    for t in range(T):
        a, v, lp = (x.cpu().numpy() for x in rec[t])
        np.testing.assert_array_equal(ac[t], a, err_msg="stored actions are the unclipped policy output @%d" % t)
        np.testing.assert_array_equal(vals[t], v)
        np.testing.assert_array_equal(lps[t], lp)
        clipped = np.clip(a, LOW, HIGH)
        clipped_any += int((clipped != a).any(axis=1).sum())
        if t == 0:
            np.testing.assert_array_equal(fr[0], o_prev[:, -1])
        else:
            _assert_frames(fr[t], o_prev[:, -1], TOL_RAND30, "slot frame @%d" % t)
        o_r, r_r, te_r, tr_r, tobs_r, *_ = ref.step(clipped)
        tv, r_raw, te_g, tr_g, tnew = (x.cpu().numpy() for x in vrec[t])
        np.testing.assert_array_equal(te_g.astype(bool), te_r, err_msg="terminated @%d" % t)
        np.testing.assert_array_equal(tr_g.astype(bool), tr_r, err_msg="truncated @%d" % t)
        np.testing.assert_allclose(r_raw, r_r, atol=reward_atol(TOL_RAND30), err_msg="raw reward @%d" % t)
        # on_policy_algorithm.py:236-245 restated: float32 rewards, gamma * terminal value
        want = r_raw.copy()
        m = tr_r & ~te_r
        want[m] = want[m] + np.float32(GAMMA) * tv[m]
        np.testing.assert_array_equal(rw[t], want, err_msg="bootstrapped rewards @%d" % t)
        boot += int(m.sum())
        if m.any():  # the bootstrap evaluated V on the right observation: the lane's final frame
            _assert_frames(tnew[m], tobs_r[m, -1], TOL_RAND30, "terminal obs @%d" % t)
        d = (te_r | tr_r).astype(np.float32)
        nxt = st[t + 1] if t + 1 < T else last_d.cpu().numpy()
        np.testing.assert_array_equal(nxt, d, err_msg="episode starts @%d" % (t + 1))
        o_prev = o_r
    assert boot >= N // 4, boot
    assert clipped_any > N, "the policy's actions should leave the Box often (the clip must matter)"
    _assert_frames(g.obs.cpu().numpy()[:, -1], o_prev[:, -1], TOL_RAND30, "env obs after 30 steps")
    # last values from the final observation, then GAE bit-exact with buffers.py:403-438
    np.testing.assert_array_equal(last_v.cpu().numpy(), vrec[T][0].cpu().numpy())
    buf.compute_returns_and_advantage(last_v, last_d)
    adv, ret = numpy_gae(rw, vals, st, last_v.cpu().numpy(), last_d.cpu().numpy().astype(bool), GAMMA, 0.95)
    np.testing.assert_array_equal(buf.advantages.cpu().numpy(), adv)
    np.testing.assert_array_equal(buf.returns.cpu().numpy(), ret)
    ref.close()
    g.close()


def _elementwise_policy(dev, k):
    """policy(obs) and value(obs) whose value for a row does not depend on the batch it is
    evaluated in (a fixed-order elementwise sum, no GEMM): the deferred bootstrap evaluates V over
    the stashed terminal observations, the per-step one over the whole batch every step."""
    import torch
    rng = np.random.default_rng(23)
    W = torch.as_tensor(rng.normal(size=(9, 4)).astype(np.float32) * 0.7, device=dev)
    wv = [float(x) for x in rng.normal(size=9).astype(np.float32)]

    def feats(obs):
        x = obs[:, -1, :]
        return [x[:, 4] * 8, x[:, 5] * 8, x[:, 6], x[:, 7], x[:, 8], x[:, 9], x[:, 10], (x[:, 2] - 1500.0) / 3000.0,
                x[:, 3] - 0.8]

    def value(obs):
        f = feats(obs)
        v = f[0] * wv[0]
        for j in range(1, 9):
            v = v + f[j] * wv[j]
        return v

    def policy(obs):
        z = torch.stack(feats(obs), 1)
        a = (z @ W + torch.tensor([0.0, 0.1, 0.0, 0.5], device=dev)).contiguous()
        return a, value(obs), -(a * a).sum(1)

    return policy, value


@pytest.mark.parametrize("layout,k", [("window", 4), ("contiguous", 4), ("window", 10)])
def test_deferred_bootstrap_equals_per_step(gpu, layout, k):
    """The deferred timeout bootstrap (terminal observations of truncated lanes stashed on device
    per step, one V evaluation after the rollout, f16env_bootstrap_stash / _apply) against the
    per-step one (V over the whole batch every step, f16env_bootstrap_timeouts): with a value head
    whose rows do not depend on the batch, every buffer -- rewards included -- and the last values
    are bit-identical, over two consecutive rollouts at cfg4's share with staggered truncations
    (and every lane truncating several times with a 9-step TimeLimit in the K = 10 case)."""
    import torch
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout
    N, T = 32768, 40
    ms = 9 if k == 10 else 1200
    runs = {}
    for mode in ("per_step", "deferred"):
        ref = OracleEnvs(N, stack_k=k, seed=61, max_steps=ms)
        g = F16Envs(N, stack_k=k, seed=61, max_steps=ms, obs_layout=layout)
        o = ref.reset()
        g.reset()
        _stagger(ref, g, o, span=min(25, ms))
        ref.close()
        policy, value = _elementwise_policy(gpu, k)
        out = {}
        for r in range(2):
            buf = DeviceRolloutBuffer(T, N, k, gpu)
            lv, ld = collect_rollout(g, buf, seed=61 + r, policy_fn=policy, value_fn=value, bootstrap=mode)
            for f in ("frames", "actions", "rewards", "episode_starts", "values", "log_probs"):
                out["%s%d" % (f, r)] = getattr(buf, f).clone()
            out["last_v%d" % r], out["last_d%d" % r] = lv.clone(), ld.clone()
        runs[mode] = out
        g.close()
    a, b = runs["per_step"], runs["deferred"]
    for f in a:
        assert torch.equal(a[f], b[f]), f
    trunc_boot = int((a["episode_starts0"][1:] > 0).sum())
    assert trunc_boot > N // 4, trunc_boot


def test_bootstrap_modes_vs_batch_of_one(gpu):
    """SB3 bootstraps each truncated lane with V evaluated on ITS terminal observation
    alone (a batch of one, on_policy_algorithm.py:236-245); both device modes evaluate a batch.
    With an MLP value head (GEMMs: a row may round differently at another batch size) the rewards
    of both modes agree with a batch-of-one reference to float32 rounding of V (|dr| <= 1e-5,
    gamma V ~ O(1)), every other reward and buffer is bit-identical, and the same lanes
    bootstrap."""
    import torch
    from bench import MlpActorCritic
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout
    N, T, k, ms = 256, 24, 4, 7
    net = MlpActorCritic(k * 15, gpu, seed=3)

    def v_batch_of_one(obs):
        return torch.cat([net.value(obs[i:i + 1]) for i in range(obs.shape[0])])

    runs = {}
    with torch.no_grad():
        for name, mode, vf in (("one", "per_step", v_batch_of_one), ("per_step", "per_step", net.value),
                               ("deferred", "deferred", net.value)):
            torch.manual_seed(5)  # the policy's Gaussian draws: the same stream in every run
            g = F16Envs(N, stack_k=k, seed=12, max_steps=ms, obs_layout="window")
            g.reset()
            buf = DeviceRolloutBuffer(T, N, k, gpu)
            lv, ld = collect_rollout(g, buf, seed=5, policy_fn=net, value_fn=vf, bootstrap=mode)
            runs[name] = {f: getattr(buf, f).clone() for f in ("frames", "actions", "rewards", "episode_starts")}
            runs[name]["trunc"] = g.trunc.clone()
            g.close()
    ref = runs["one"]
    boot = ref["episode_starts"][1:] > 0  # lanes whose episode ended (crash or truncation) at step t
    assert int(boot.sum()) > N // 2
    for name in ("per_step", "deferred"):
        r = runs[name]
        for f in ("frames", "actions", "episode_starts"):
            assert torch.equal(r[f], ref[f]), (name, f)
        d = (r["rewards"] - ref["rewards"]).abs()
        assert float(d.max()) <= 1e-5, (name, float(d.max()))
        # only bootstrapped (truncated-only) lanes can differ
        changed = d[:-1] > 0
        assert not bool((changed & ~boot).any()), name


def _crash_ics(n):
    ic = np.tile(default_ic(), (n, 1))
    ic[:, 2] = np.linspace(150.0, 9000.0, n)  # low lanes crash and auto-reset during the rollout
    ic[:, 7] = -0.35
    return ic


def _rollout(gpu, layout, k, cfg5, persistent, n=4096, T=48):
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout
    e = F16Envs(n, stack_k=k, seed=4, max_steps=40, cfg5=cfg5, obs_layout=layout)
    if cfg5:
        e.reset()
    else:
        e.reset(ic=_crash_ics(n))
    collect_rollout(e, DeviceRolloutBuffer(3, n, k, gpu), 17, persistent=persistent)  # carry-over starts
    b = DeviceRolloutBuffer(T, n, k, gpu)
    _, last_d = collect_rollout(e, b, 21, step0=100, persistent=persistent)
    out = {f: getattr(b, f).clone() for f in ("frames", "actions", "rewards", "episode_starts", "obs0")}
    out["last_d"] = last_d.clone()
    out["obs"] = e.obs.clone()
    out["state"] = e.get_state()
    e.close()
    return out


CASES = [(4, False), (10, False), (4, True), (10, True)]


@pytest.mark.parametrize("k,cfg5", CASES, ids=["k%d%s" % (k, "_cfg5" if c else "") for k, c in CASES])
def test_window_rollouts_bit_identical(gpu, k, cfg5):
    """Fused windowed rollout == fused contiguous rollout, persistent == fused in both layouts:
    actions (Philox), episode structure (crashes, truncation at 40 steps, auto-resets), frames,
    rewards, the final observation and state, bit for bit."""
    import torch
    runs = {(lay, p): _rollout(gpu, lay, k, cfg5, p) for lay in ("contiguous", "window") for p in (False, True)}
    base = runs[("contiguous", False)]
    assert int(base["episode_starts"][1:].sum().item()) > 0, "expected auto-resets in the rollout"
    for key, r in runs.items():
        for f in base:
            assert torch.equal(r[f], base[f]), (key, f)


@pytest.mark.parametrize("k,cfg5", [(10, False), (4, True)], ids=["k10", "cfg5"])
def test_persistent_window_rollout_vs_oracle(gpu, k, cfg5):
    """The one-launch windowed rollout (f16env_window_rollout_random) against the oracle stepping
    the same Philox actions: the reference's K = 10, and cfg5 (random-IC resets: a lane's first
    from the reset cache, later ones by its own RunIC in the kernel; gusts). 30 slots with a
    third of the lanes truncating: actions and episode starts bit-exact, rewards 2e-3, slot
    frames at TOL_RAND30 (cfg5: 99.9 % of the lanes, every lane within 10x, as the cfg5
    production test), the final observation continuing the rebuilt stack."""
    import torch
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout, rebuild_observations
    n, T, seed = 4096, 30, 33
    ms = 20 if cfg5 else 1200  # cfg5: lanes truncate twice in the 30 steps (cached, then in-kernel RunIC)
    ref = OracleEnvs(n, stack_k=k, seed=seed, cfg5=cfg5, max_steps=ms)
    g = F16Envs(n, stack_k=k, seed=seed, cfg5=cfg5, max_steps=ms, obs_layout="window")
    o = ref.reset()
    g.reset()
    _stagger(ref, g, o, span=min(25, ms))
    buf = DeviceRolloutBuffer(T, n, k, gpu)
    collect_rollout(g, buf, seed, step0=0)
    torch.cuda.synchronize()
    fr, ac, rw, st = (getattr(buf, f).cpu().numpy() for f in ("frames", "actions", "rewards", "episode_starts"))
    last = g._last_episode_starts.cpu().numpy()
    tol_max = TOL_RAND30 * 10 if cfg5 else TOL_RAND30
    o_prev = o
    resets = 0
    for t in range(T):
        a = ref.sample_actions(seed, t)
        np.testing.assert_array_equal(ac[t], a, err_msg="actions @%d" % t)
        if t == 0:
            np.testing.assert_array_equal(fr[0], o_prev[:, -1])
        else:
            _assert_frames_stat(fr[t], o_prev[:, -1], TOL_RAND30, tol_max, "slot frame @%d" % t)
        o_r, r_r, te_r, tr_r, *_ = ref.step(a)
        np.testing.assert_allclose(rw[t], r_r, atol=reward_atol(tol_max), err_msg="reward @%d" % t)
        d = (te_r | tr_r).astype(np.float32)
        nxt = st[t + 1] if t + 1 < T else last
        np.testing.assert_array_equal(nxt, d, err_msg="episode starts @%d" % (t + 1))
        if d.any():  # reset frames (the next slot's frame): Philox goal bit-exact, IC at TOL_STEP
            nf = fr[t + 1] if t + 1 < T else g.obs.cpu().numpy()[:, -1]
            dd = d.astype(bool)
            np.testing.assert_array_equal(nf[dd, 12:], o_r[dd, -1, 12:])
            _assert_frames(nf[dd], o_r[dd, -1], TOL_STEP, "reset frame @%d" % t)
        resets += int(d.sum())
        o_prev = o_r
    assert resets >= n // 3, resets
    fin = g.obs
    _assert_frames_stat(fin.cpu().numpy()[:, -1], o_prev[:, -1], TOL_RAND30, tol_max, "env obs after 30 slots")
    # the final window: K x the reset frame where the last slot ended an episode, else the
    # rebuilt stack of slot T-1 shifted by the newest frame
    last_obs = rebuild_observations(buf.frames, buf.obs0, buf.episode_starts, k, steps=[T - 1])[0]
    cont = ~torch.as_tensor(last, device=gpu).bool()
    assert torch.equal(fin[cont, :-1], last_obs[cont, 1:])
    assert torch.equal(fin[~cont], fin[~cont, :1].expand(-1, k, -1))
    # the next windowed step continues from there (both histories hold the window)
    o2 = g.step(g.sample_actions(seed, T)).obs
    o2_r = ref.step(ref.sample_actions(seed, T))[0]
    _assert_frames_stat(o2.cpu().numpy()[:, -1], o2_r[:, -1], TOL_RAND30, tol_max * 2, "step after the rollout")
    ref.close()
    g.close()


def test_window_rollout_features_and_ragged_n(gpu):
    """The windowed rollout step's features (f16env_features_strided on the returned window) equal
    the features kernel on a contiguous copy; a ragged N (n % 4 != 0: frame-log rows not 16-B
    aligned) writes the log with dword stores and matches the contiguous layout."""
    import torch
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.features import features
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout
    n, k = 1001, 5
    e = F16Envs(n, stack_k=k, seed=3, obs_layout="window")
    e.reset(ic=_crash_ics(n))
    feat = torch.empty((n, k, 17), dtype=torch.float32, device=gpu)
    for t in range(6):
        out = e.step_rollout(5, t, features=feat)
        want = features(out.obs.contiguous())
        assert torch.equal(feat, want), t
    e.close()
    bufs = []
    for lay in ("contiguous", "window"):
        e = F16Envs(n, stack_k=k, seed=3, obs_layout=lay)
        e.reset(ic=_crash_ics(n))
        b = DeviceRolloutBuffer(40, n, k, gpu)
        collect_rollout(e, b, 9, persistent=False)
        bufs.append((b, e.obs.clone()))
        e.close()
    (b0, o0), (b1, o1) = bufs
    for f in ("frames", "actions", "rewards", "episode_starts"):
        assert torch.equal(getattr(b0, f), getattr(b1, f)), f
    assert torch.equal(o0, o1)
