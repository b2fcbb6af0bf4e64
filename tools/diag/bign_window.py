"""Diagnostic: 2^21 + 77 envs, windowed layout, tail vs its 333-env shard (test_gpu_production
two_million case). Prints the kernel instances and, per step, where the tails differ."""
import sys
import torch
sys.path.insert(0, ".")
from f16_jsb_amd.env import F16Envs
from f16_jsb_amd.abi import F16C_EP_COUNT

n, tail = (1 << 21) + 77, 333
for hist in (16,):
    kw = dict(stack_k=4, seed=93, cfg5=len(sys.argv) > 1 and sys.argv[1] == "cfg5", max_steps=40, obs_layout="window", history=hist)
    big = F16Envs(n, env_id_base=0, **kw)
    small = F16Envs(tail, env_id_base=n - tail, **kw)
    print("history", hist, "kernels", big.step_kernel_name, big.waves_per_simd, "|", small.step_kernel_name, small.waves_per_simd, flush=True)
    ob, os_ = big.reset(), small.reset()
    print("reset equal", torch.equal(ob[n - tail:], os_), flush=True)
    for t in range(int(sys.argv[2]) if len(sys.argv) > 2 else 6):
        a = big.sample_actions(5, t)
        a_s = small.sample_actions(5, t)
        ep_before = small.get_state()[:, F16C_EP_COUNT].clone()
        o_b, o_s = big.step(a), small.step(a_s)
        d = (o_b.obs[n - tail:] - o_s.obs).abs()
        bad = (d.amax(dim=(1, 2)) > 0).nonzero().flatten()
        if bad.numel():
            dn = (o_s.terminated | o_s.truncated).bool()
            print("   differing lanes", bad.tolist()[:10], "done now", dn[bad].tolist()[:10],
                  "ep_count before", ep_before[bad].tolist()[:10], "slot/comp diffs",
                  [(int(i), (d[i] > 0).nonzero().tolist()[:6]) for i in bad[:3]], flush=True)
        sb = big.get_state()[n - tail:]
        ss = small.get_state()
        sd = (sb - ss).abs().amax(dim=0)
        if t == 0:
            print("rel state col diff", ((sb - ss).abs() / (ss.abs() + 1e-30)).amax(dim=0).tolist(), flush=True)
        print("t", t, "obs lanes differing", bad.numel(), "first", bad[:5].tolist(),
              "max", float(d.max()), "per-slot max", d.amax(dim=(0, 2)).tolist(),
              "per-component max", ["%.1e" % v for v in d.amax(dim=(0, 1)).tolist()],
              "state cols differing", (sd > 0).nonzero().flatten().tolist(), "rew eq", torch.equal(o_b.rew[n - tail:], o_s.rew),
              flush=True)
    big.close()
    small.close()
