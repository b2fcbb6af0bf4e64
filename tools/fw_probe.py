"""Feature-window probe for rocprofv3 --kernel-trace --stats: at 65 536 envs, windowed layout,
K = 4 and K = 10, `steps` steps each followed by F16Envs.obs_features() (the incremental
f16_feature_window_kernel), then `steps` steps each followed by the whole-window transform
(features(envs.obs), f16_features_strided_kernel), so the summary holds both kernels' average
durations side by side; then rollout-slot steps (step_rollout with policy actions) without and
with obs_features after each (the feature window kept in the step's epilogue). Prints one JSON line with the host-driven ms per step of each form.

    rocprofv3 --kernel-trace --stats -d gpurun_out/fw -o run --output-format csv -- python3 tools/fw_probe.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(steps=300):
    import torch
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.features import features
    dev = torch.device("cuda", 0)
    out = {}
    for k in (4, 10):
        e = F16Envs(65536, stack_k=k, seed=3, obs_layout="window", device=dev)
        e.reset()
        acts = [e.sample_actions(5, i) for i in range(8)]
        buf = torch.empty((65536, k, 17), dtype=torch.float32, device=dev)
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        res = {}
        for name in ("plain", "window", "whole", "rollout_step", "rollout_step_fused"):
            roll = name.startswith("rollout")
            for i in range(20):
                if roll:
                    e.step_rollout(7, i, policy_actions=acts[i % 8])
                else:
                    e.step(acts[i % 8])
                if name in ("window", "rollout_step_fused"):
                    e.obs_features()  # (the first call allocates the feature histories)
            s.record()
            for i in range(steps):
                if roll:  # the rollout-slot step: with the feature window current, it keeps it
                    o = e.step_rollout(7, i, policy_actions=acts[i % 8]).obs
                else:
                    o = e.step(acts[i % 8]).obs
                if name in ("window", "rollout_step_fused"):
                    e.obs_features()
                elif name == "whole":
                    features(o, buf)
            t.record()
            torch.cuda.synchronize()
            res[name + "_ms_per_step"] = round(s.elapsed_time(t) / steps, 5)
        res["feature_window_calls"] = dict(e.feature_window_calls)
        # the incremental kernel alone, host out of the loop: 100 launches at the current position
        # captured as a HIP graph, replayed (kernel + dependent-launch boundary per launch)
        import ctypes
        from f16_jsb_amd._lib import check, lib
        e.obs_features()
        wrow, wenv = (16, e.T * 16) if e._env_major else (e.n * 16, 16)
        cur = e._cur

        def one():
            check(lib().f16env_features_window_step(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), e.n, k,
                                                    e._p, e._hist_ptr[cur], wrow, wenv, e._fh_ptr[cur],
                                                    e._fh_ptr[cur ^ 1], e.term.data_ptr(), e.trunc.data_ptr(), 1, 1),
                  "f16env_features_window_step")

        def graph_ms():
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                one()
            torch.cuda.current_stream().wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(100):
                    one()
            best = None
            for _ in range(3):
                s.record()
                g.replay()
                t.record()
                torch.cuda.synchronize()
                ms = s.elapsed_time(t) / 100
                best = ms if best is None else min(best, ms)
            del g
            return best

        res["done_fraction_last_step"] = round(float(((e.term | e.trunc) != 0).float().mean()), 5)
        best = graph_ms()
        res["feature_window_kernel_graph_ms"] = round(best, 5)
        res["feature_window_GBps"] = round(65536 * 200 / (best * 1e-3) / 1e9, 1)
        # the same with no lane reset by the step (no window fills): the transform alone
        flags = e.step_flags.clone()
        e.term.zero_()
        e.trunc.zero_()
        best0 = graph_ms()
        e.step_flags.copy_(flags)
        res["feature_window_kernel_graph_ms_no_resets"] = round(best0, 5)
        res["feature_window_GBps_no_resets"] = round(65536 * 200 / (best0 * 1e-3) / 1e9, 1)
        assert torch.equal(e.obs_features(), features(e.obs))
        out["K%d" % k] = res
        e.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
