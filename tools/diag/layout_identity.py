"""Diagnostic: are the contiguous and windowed layouts bit-identical (state, obs, rewards)?
Usage: python tools/diag/layout_identity.py [cfg5] [n] [steps]"""
import sys
import torch
sys.path.insert(0, ".")
from f16_jsb_amd.env import F16Envs
from f16_jsb_amd.abi import F16C_EP_COUNT, F16C_STEP

cfg5 = len(sys.argv) > 1 and sys.argv[1] == "cfg5"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 100
kw = dict(stack_k=4, seed=11, cfg5=cfg5, max_steps=60)
a = F16Envs(n, **kw)
b = F16Envs(n, obs_layout="window", history=16, **kw)
print("kernels", a.step_kernel_name, "|", b.step_kernel_name, flush=True)
print("reset obs equal", torch.equal(a.reset(), b.reset()))
for t in range(steps):
    act = a.sample_actions(3, t)
    oa, ob = a.step(act), b.step(act)
    sa, sb = a.get_state(), b.get_state()
    so = (sa != sb).any(dim=0).nonzero().flatten().tolist()
    sl = (sa != sb).any(dim=1).nonzero().flatten()
    if sl.numel():
        print("   state lanes", sl.tolist()[:8], "ep_count", sa[sl[:8], F16C_EP_COUNT].tolist(), "step", sa[sl[:8], F16C_STEP].tolist(),
              "done now", (oa.terminated | oa.truncated)[sl[:8]].tolist(), flush=True)
    do = (oa.obs != ob.obs)
    lanes = do.any(dim=2).any(dim=1).nonzero().flatten()
    comps = do.any(dim=0).any(dim=0).nonzero().flatten().tolist()
    if so or lanes.numel() or not torch.equal(oa.rew, ob.rew):
        print("t", t, "state cols", so, "obs lanes", lanes.numel(), "comps", comps, "rew eq", torch.equal(oa.rew, ob.rew),
              "max obs diff", float((oa.obs - ob.obs).abs().max()), flush=True)
print("done", flush=True)
