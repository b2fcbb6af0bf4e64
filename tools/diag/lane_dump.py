"""Diagnostic: one lane's observation frames and latch (lx) values in both layouts, per step.
Usage: python tools/diag/lane_dump.py LANE [cfg5] [n] [steps]"""
import sys
import torch
sys.path.insert(0, ".")
from f16_jsb_amd.env import F16Envs
from f16_jsb_amd.abi import F16C_LX, F16C_WIND, F16C_GUST

lane = int(sys.argv[1])
cfg5 = len(sys.argv) > 2 and sys.argv[2] == "cfg5"
n = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
kw = dict(stack_k=4, seed=11, cfg5=cfg5, max_steps=60)
a = F16Envs(n, **kw)
b = F16Envs(n, obs_layout="window", history=16, **kw)
a.reset(); b.reset()
torch.set_printoptions(precision=9, linewidth=250)
for t in range(steps):
    act = a.sample_actions(3, t)
    oa, ob = a.step(act), b.step(act)
    sa, sb = a.get_state()[lane], b.get_state()[lane]
    print("t", t, "act", act[lane].tolist())
    print("  obs A", oa.obs[lane, -1].tolist())
    print("  obs B", ob.obs[lane, -1].tolist())
    print("  lx A", sa[F16C_LX:F16C_LX + 10].tolist())
    print("  lx B", sb[F16C_LX:F16C_LX + 10].tolist())
    print("  wind/gust", sa[F16C_WIND:F16C_GUST + 3].tolist(), flush=True)
