"""Child process of tests/test_gpu_rccl.py: the rollout gather (f16_jsb_amd/rollout.py
gather_to_rank0) through torch.distributed's "nccl" backend -- RCCL on ROCm --
on this box's one GPU (world size 1: RCCL's own communicator and gather kernels run, the
transfer is rank 0 to itself). Prints one JSON line; exit status 0 only if the gathered
tensors equal the local shard bit for bit.

    MASTER_ADDR=127.0.0.1 MASTER_PORT=... python tests/rccl_gather_run.py
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout, env_major, gather_to_rank0

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    N, K, T = 4096, 4, 24
    envs = F16Envs(N, stack_k=K, seed=9, obs_layout="window")
    envs.reset()
    buf = DeviceRolloutBuffer(T, N, K, dev)
    collect_rollout(envs, buf, 9, step0=0)
    torch.cuda.synchronize()
    out = gather_to_rank0(buf, chunk_steps=5)  # 5 + 5 + 5 + 5 + 4: a short last chunk
    torch.cuda.synchronize()
    ok, bad = True, []
    for f, v in out.items():
        local = getattr(buf, f)
        if v.shape != (1,) + tuple(local.shape) or not torch.equal(v[0], local):
            ok, bad = False, bad + [f]
        if f != "obs0" and not torch.equal(env_major(v), local):
            ok, bad = False, bad + [f + " (env_major)"]
    nbytes = sum(v.numel() * v.element_size() for v in out.values())
    backend = dist.get_backend()
    dist.destroy_process_group()
    print(json.dumps({"backend": backend, "nccl_version": ".".join(map(str, torch.cuda.nccl.version())),
                      "fields": sorted(out), "bytes": nbytes, "bit_identical": ok, "mismatch": bad}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
