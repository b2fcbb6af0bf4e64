#!/usr/bin/env python3
"""Throughput benchmark of the MI355X F-16 environment (BASELINE.json configs[2]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs 65536] [--stack 4]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one process per GPU)

A "step" is one VecEnv step (4 FDM frames + obs/reward/termination/auto-reset) of every env
on the GPU, driven through the device-tensor VecEnv boundary (F16Envs.step) with random
actions from the device Philox stream, pre-generated into HBM before the timed region.
The observation layout is the windowed one (F16Envs(obs_layout="window"): the (N, K, 15)
obs is a strided view of per-env frame histories, one new 64-B frame slot written per step);
the contiguous ping-pong layout is timed beside it (`layouts`).
Envs shard across ranks (weak scaling, no collective in the stepping loop); the job-level
value is all ranks' env-steps divided by the max-over-ranks wall time.

Prints ONE JSON line on rank 0 (driver contract), including
  roofline     -- algorithmic HBM bytes per launch of the step kernel (the bytes its layout
                  must move; SURVEY 8(d)'s B(K) beside it as contract_*) / its average launch
                  duration (HIP events on the launch stream), vs the 8 TB/s HBM peak;
                  `traffic` = PMC-measured HBM bytes per launch from profiles/ if present;
  cpu_baseline -- the CPU oracle (oracle/f16ref.c, fp64 C restatement, OpenMP) timed on this
                  host on a bounded sample of the same workload (rank 0, at every N, after the
                  closing barrier); rccl_world -- the size of the group RCCL reports.
"""
from __future__ import annotations

import argparse
import ctypes
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# kernel arguments in device memory (this ROCm's default, pinned here): with them in host memory
# every step launch pays ~3 us more for its first scalar loads (tools/size_sweep.py A/B)
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

METRIC = "env-steps/sec at 65 536 envs, 1/2/4/8 MI355X; HBM GB/s fraction"
HBM_PEAK_GBPS = 8000.0  # /opt/skills/guides/MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--workload", choices=("cfg3", "cfg5"), default="cfg3",
                    help="cfg3: the headline (reference task); cfg5: random ICs + wind gusts")
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (cfg3 65536, cfg5 131072)")
    ap.add_argument("--stack", type=int, default=4)
    ap.add_argument("--obs-layout", choices=("window", "contiguous"), default="window",
                    help="observation layout of the headline (the other is timed beside it at N=1)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="N > 1 process group: nccl (RCCL over xGMI, the measurement); gloo only "
                         "rehearses the multi-rank code path on a box with fewer GPUs than ranks")
    ap.add_argument("--action-pool", type=int, default=0,
                    help="distinct pre-generated action batches (0 = one per timed step)")
    ap.add_argument("--rollout-envs", type=int, default=32768, help="cfg4 rollout envs per GPU (0 = skip)")
    ap.add_argument("--rollout-steps", type=int, default=2048, help="cfg4 PPO n_steps")
    ap.add_argument("--gather-chunk", type=int, default=256, help="steps per RCCL gather chunk")
    ap.add_argument("--policy-steps", type=int, default=256,
                    help="rollout leg: steps of the policy-in-the-loop rollout (0 = skip)")
    ap.add_argument("--burn-in", type=int, default=None,
                    help="untimed steps after the phase spread (default: max_steps = 1200) so the timed window "
                         "sees the steady-state episode mix (crashes, goals, truncations, auto-resets)")
    # test hooks (tests/test_bench_launch.py, tests/test_gpu_bench_legs.py)
    ap.add_argument("--fail-leg", default=None,
                    help="raise inside this side leg (forced failure: the line gets legs_failed, exit 1)")
    ap.add_argument("--launch-selftest", action="store_true",
                    help="ranks only join the process group (gloo) and rank 0 prints the launch fields: "
                         "checks the --gpus N launcher without a GPU")
    ap.add_argument("--selftest-fail-rank", type=int, default=-1, help="with --launch-selftest: this rank exits 3")
    return ap.parse_args()


def launch_ranks(args, argv):
    """`bench.py --gpus N` (N > 1) started without a torch.distributed launcher: start the N
    ranks as children of `python -m torch.distributed.run` (one process per GPU, rendezvous on
    127.0.0.1) and relay rank 0's JSON line. This process makes no GPU call (torch is not even
    imported here) and never exec's: it waits for the launcher, forwards the ranks' other
    output to stderr as it arrives, and exits non-zero when any rank failed or no line came."""
    import subprocess
    # --standalone: the launcher's own c10d store binds a free port itself and keeps it (a port
    # probed here and handed over could be taken by another process in between);
    # --local-addr keeps the rendezvous on 127.0.0.1 (the container hostname may not resolve)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
           "--nnodes=1", "--nproc-per-node", str(args.gpus), os.path.abspath(__file__), *argv]
    print("[bench] launching %d ranks: %s" % (args.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1)
    line = None
    for ln in proc.stdout:
        if ln.startswith('{"metric"'):
            line = ln.strip()
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    rc = proc.wait()
    if line is not None:
        print(line, flush=True)
    if rc != 0:
        print("[bench] a rank failed (launcher exit %d)" % rc, file=sys.stderr, flush=True)
        return rc if rc > 0 else 1
    if line is None:
        print("[bench] rank 0 printed no result line", file=sys.stderr, flush=True)
        return 1
    return 0


def launch_selftest(args, world, rank):
    """--launch-selftest: the rank side of the launcher check -- join the group over gloo, agree
    on the world size, rank 0 prints the line's launch fields (no GPU, no kernels)."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.ones(1)
    dist.all_reduce(t)
    if rank == args.selftest_fail_rank:
        sys.exit(3)
    dist.barrier()
    envs = args.envs or 65536
    if rank == 0:
        line = {"metric": METRIC, "value": None, "n_gpus": world, "selftest": True,
                "ranks_joined": int(t.item()),
                "config": {"envs_per_gpu": envs, "global_envs": envs * world}}
        # the closing fields every line carries at every N, made by the same code as the real run
        line.update(closing_fields(args, world, min(envs, 4096), args.stack))
        print(json.dumps(line), flush=True)
    dist.destroy_process_group()


def closing_fields(args, world, n, stack, cfg5=False, leg=None):
    """The fields every result line carries at every N, made on rank 0 after
    the closing barrier, when no rank is timing anything: the process group as the collective
    library reports it (`rccl_world`: dist.get_world_size() of the nccl = RCCL group; None under
    gloo or without a group) and the CPU baseline."""
    import torch.distributed as dist
    pg = {"backend": None, "world_size": 1}
    if dist.is_available() and dist.is_initialized():
        pg = {"backend": str(dist.get_backend()), "world_size": dist.get_world_size()}
    out = {"process_group": pg, "rccl_world": pg["world_size"] if pg["backend"] == "nccl" else None}
    if not args.no_cpu_baseline:
        run = leg or (lambda name, fn, *a: fn(*a))
        out["cpu_baseline"] = run("cpu_baseline", cpu_baseline, n, stack, args.cpu_seconds, cfg5)
    return out


def cpu_baseline(envs, stack, seconds, cfg5=False):
    """Time the fp64 CPU oracle on the same workload (random actions, auto-reset)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    try:
        from oracle_ref import OracleEnvs, build_oracle, lib
        build_oracle()
    except Exception as e:  # noqa: BLE001
        return {"value": None, "unit": "env-steps/s", "cores": 0, "kind": "port",
                "sample": "oracle unavailable: %s" % e}
    import numpy as np
    threads = int(lib().f16ref_threads())
    # CPUs this process may run on (on the GPU box: the whole machine; the lease's share is OMP_NUM_THREADS)
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    n = min(envs, 65536)
    e = OracleEnvs(n, stack_k=stack, seed=1, cfg5=cfg5)
    e.reset()
    tw = time.perf_counter()  # untimed warm-up (thread pool, first touch of the env arrays)
    while time.perf_counter() - tw < 0.5:
        e.step(e.sample_actions(2, 0))
    steps = 0
    t0 = time.perf_counter()
    while True:
        a = e.sample_actions(1, steps)
        e.step(a)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds or steps >= 2000:
            break
    e.close()
    # SURVEY 8(d) also asks for the all-cores rate at N = 4096 (cfg2's env count), and the rate
    # against the thread count: 4 096 envs at 1, 2, 4, 8 ... threads up to the inherited count
    def rate4096(nthreads, secs):
        lib().f16ref_set_threads(nthreads)
        e4 = OracleEnvs(4096, stack_k=stack, seed=1, cfg5=cfg5)
        e4.reset()
        for w in range(3):
            e4.step(e4.sample_actions(2, w))
        s4 = 0
        t4 = time.perf_counter()
        while time.perf_counter() - t4 < secs:
            e4.step(e4.sample_actions(1, s4))
            s4 += 1
        el4 = time.perf_counter() - t4
        e4.close()
        return round(4096 * s4 / el4, 1), s4, el4
    scaling = {}
    for nt in sorted({1, 2, 4, 8, threads}):
        if nt <= threads:
            scaling[str(nt)] = rate4096(nt, min(1.5, seconds))[0]
    lib().f16ref_set_threads(0)
    n4 = None
    if n > 4096:
        v4, s4, el4 = rate4096(threads, min(3.0, seconds))
        lib().f16ref_set_threads(0)
        n4 = {"value": v4, "unit": "env-steps/s", "cores": threads,
              "sample": "4096 envs x %d random-action steps, %.1f s" % (s4, el4)}
    per_core = scaling[str(threads)] / threads
    # BASELINE cfg1 semantics beside it: ONE env, 1000 random-action steps, reference stack K=10
    e1 = OracleEnvs(1, stack_k=10, seed=1)
    e1.reset()
    rng = np.random.default_rng(0)
    acts = rng.uniform([-1, -1, -1, 0], [1, 1, 1, 1], (1000, 1, 4)).astype(np.float32)
    t1 = time.perf_counter()
    for t in range(1000):
        e1.step(acts[t])
    el1 = time.perf_counter() - t1
    e1.close()
    cfg1 = {"value": round(1000 / el1, 1), "unit": "env-steps/s", "cores": 1,
            "sample": "BASELINE cfg1: 1 env x 1000 random-action steps (numpy default_rng(0), K=10), "
                      "oracle/f16ref.c through its ctypes step (one env, no parallelism)"}
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
    except OSError:
        pass
    return {"value": round(n * steps / el, 1), "unit": "env-steps/s", "cores": threads, "kind": "port", "cfg1": cfg1,
            "n4096": n4,
            "thread_scaling_4096_envs": scaling,
            "all_affinity_cpus_extrapolated": {
                "value": round(per_core * affinity, 1), "cores": affinity, "measured": False,
                "basis": "per-thread rate at %d threads (4096 envs) x %d CPUs of the affinity set, linear as "
                         "thread_scaling_4096_envs is up to the share" % (threads, affinity),
                "why_not_measured": "the GPU pool grants each 1-GPU lease a %s-CPU share and sets "
                                    "OMP_NUM_THREADS to it (to be left as set); the affinity set is the whole "
                                    "machine's CPUs, shared with other leases" % os.environ.get("OMP_NUM_THREADS")},
            "host": {"cpu_model": model, "os_cpu_count": os.cpu_count(), "sched_affinity_cpus": affinity,
                     "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
                     "cores_note": "cores = OpenMP threads used = OMP_NUM_THREADS (the lease's CPU share); "
                                   "os_cpu_count / sched_affinity_cpus are the whole machine"},
            "sample": "oracle/f16ref.c (fp64 C restatement of the JSBSim F-16 FDM, not JSBSim), "
                      "%d envs x %d random-action steps (stack=%d, auto-reset%s), %d OpenMP threads, %.1f s"
                      % (n, steps, stack, ", cfg5 random IC + gusts" if cfg5 else "", threads, el)}


def spread_phases(envs, args, dev):
    """Steady-state episode mix before timing (dummy_vec_env.py:68-71 auto-reset load): the
    lanes' step counters are spread uniformly over [0, max_steps) (a long-running VecEnv's
    episode ages), then `burn_in` untimed random-action steps (default max_steps) let crashes,
    goal captures and truncations reach their steady rates, so any timed window -- the
    driver's 20 steps included -- carries the auto-reset work of the steady state."""
    import numpy as np
    import torch
    from f16_jsb_amd.abi import F16C_STEP
    max_steps = int(envs.cfg.max_steps)
    s = envs.get_state()
    rng = np.random.default_rng(args.seed + 77)
    phase = rng.integers(0, max_steps, size=envs.n)
    s[:, F16C_STEP] = torch.as_tensor(phase, dtype=torch.float64, device=dev)
    envs.set_state(s)
    burn = max_steps if args.burn_in is None else int(args.burn_in)
    a = torch.empty((envs.n, 4), dtype=torch.float32, device=dev)
    for t in range(burn):
        envs.sample_actions(args.seed + 3000, t, out=a)
        envs.step(a)
    torch.cuda.synchronize()
    return {"phase_spread": "step counters uniform over [0, %d)" % max_steps, "burn_in_steps": burn}


class MlpActorCritic:
    """The policy of the rollout leg's policy-in-the-loop rate: SB3's default PPO MlpPolicy shape
    (stable_baselines3 ActorCriticPolicy: flattened observation -> separate pi / vf MLPs
    [64, 64] with tanh, a 4-wide action mean with a state-independent log std, a value head;
    actions sampled from the diagonal Gaussian, their log-probability summed over the action
    dims), random-init weights. __call__(obs) -> (actions, values, log_probs) as
    on_policy_algorithm.py:202's policy(obs_tensor); value(obs) the vf branch alone."""

    def __init__(self, obs_dim, dev, seed=0):
        import torch
        g = torch.Generator(device="cpu").manual_seed(seed)

        def lin(i, o, gain):
            w = torch.randn(o, i, generator=g) * (gain / i ** 0.5)
            return w.to(dev), torch.zeros(o, device=dev)

        self.pi = [lin(obs_dim, 64, 2 ** 0.5), lin(64, 64, 2 ** 0.5)]
        self.vf = [lin(obs_dim, 64, 2 ** 0.5), lin(64, 64, 2 ** 0.5)]
        self.act_w = lin(64, 4, 0.01)
        self.val_w = lin(64, 1, 1.0)
        self.log_std = torch.zeros(4, device=dev)

    @staticmethod
    def _mlp(x, layers):
        import torch
        for w, b in layers:
            x = torch.tanh(torch.nn.functional.linear(x, w, b))
        return x

    def value(self, obs):
        import torch
        x = obs.reshape(obs.shape[0], -1)
        return torch.nn.functional.linear(self._mlp(x, self.vf), *self.val_w).reshape(-1)

    def __call__(self, obs):
        import math
        import torch
        x = obs.reshape(obs.shape[0], -1)
        mean = torch.nn.functional.linear(self._mlp(x, self.pi), *self.act_w)
        std = self.log_std.exp()
        eps = torch.randn_like(mean)
        act = mean + std * eps
        logp = (-0.5 * eps * eps - self.log_std - 0.5 * math.log(2 * math.pi)).sum(-1)
        return act, self.value(obs), logp


class GraphedPolicy:
    """A policy's forward and value forward each captured once as a HIP graph (torch.cuda.graph:
    hipStreamBeginCapture underneath) on a static (N, K, 15) input: per call one copy of the
    observation (the window view, strided) into the static input and one graph replay, instead
    of ~20 eagerly launched small kernels. The outputs are the graph's static tensors, valid
    until the next call (collect_rollout consumes them within the step, in stream order)."""

    def __init__(self, net, n, k, dev):
        import torch
        self.net, self.n = net, n
        self.x = torch.zeros((n, k, 15), dtype=torch.float32, device=dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(3):
                net(self.x), net.value(self.x)
        torch.cuda.current_stream(dev).wait_stream(side)
        self.g, self.gv = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g):
            self.out = net(self.x)
        with torch.cuda.graph(self.gv):
            self.vout = net.value(self.x)

    def __call__(self, obs):
        self.x.copy_(obs)
        self.g.replay()
        return self.out

    def value(self, obs):
        if obs.shape[0] != self.n:  # another batch (the deferred bootstrap's stash): eager
            return self.net.value(obs)
        self.x.copy_(obs)
        self.gv.replay()
        return self.vout


def rollout_bench(args, dev, rank, world):
    """BASELINE cfg4 beside the headline: a PPO-shaped rollout (n_steps x envs per GPU) into
    the device rollout buffer, HIP GAE, then the RCCL gather of every shard to rank 0.
    Rollout, GAE and gather are timed separately (max over ranks); not part of `value`.
    The envs step in the windowed layout (the headline's); the rollout is timed three ways:
    the random policy as ONE persistent launch (f16env_window_rollout_random), the random policy
    as one fused rollout-step launch per step (f16env_window_step_rollout, actions drawn
    in-kernel; beside it the plain windowed step at the same env count, and the contiguous
    layout's fused steps), and a policy network in the loop (MlpActorCritic: SB3's default
    PPO policy shape, its actions clipped in-kernel, the timeout bootstrap on device)."""
    import torch
    import torch.distributed as dist
    from f16_jsb_amd.env import F16Envs
    from f16_jsb_amd.rollout import DeviceRolloutBuffer, collect_rollout, gather_to_rank0

    n, T = args.rollout_envs, args.rollout_steps
    envs = F16Envs(n, stack_k=args.stack, device=dev, seed=args.seed + 7, env_id_base=rank * n, obs_layout="window")
    envs.reset()
    buf = DeviceRolloutBuffer(T, n, args.stack, dev)
    collect_rollout(envs, DeviceRolloutBuffer(8, n, args.stack, dev), args.seed + 3000)  # warm
    collect_rollout(envs, DeviceRolloutBuffer(8, n, args.stack, dev), args.seed + 3000, persistent=False)
    sync = torch.cuda.synchronize

    def barrier():
        if world > 1:
            dist.barrier()
        sync()

    # the same rollout as one fused launch per step (f16env_window_step_rollout), for comparison
    barrier()
    tf0 = time.perf_counter()
    collect_rollout(envs, buf, args.seed + 5000, persistent=False)
    sync()
    fused_s = time.perf_counter() - tf0
    # the plain windowed step at the same env count (what the fused rollout step adds to)
    acts = [envs.sample_actions(args.seed + 5500, t) for t in range(8)]
    sync()
    tp0 = time.perf_counter()
    for t in range(512):
        envs.step(acts[t % 8])
    sync()
    plain_ms = (time.perf_counter() - tp0) / 512 * 1e3
    # the two kernels alone (dispatch events of each launch): the rollout-slot build vs the plain
    # windowed step, 256 launches each
    small = DeviceRolloutBuffer(256, n, args.stack, dev)
    roll_kern_ms, _, _ = envs.profile_kernel(lambda: collect_rollout(envs, small, args.seed + 5600, persistent=False), 256)
    step_kern_ms, _, _ = envs.profile_kernel(lambda: [envs.step(acts[t % 8]) for t in range(256)], 256)
    del small
    barrier()
    t0 = time.perf_counter()
    last_v, last_d = collect_rollout(envs, buf, args.seed + 4000)  # one persistent launch
    sync()
    t1 = time.perf_counter()
    buf.compute_returns_and_advantage(last_v, last_d)
    sync()
    t2 = time.perf_counter()
    # GAE kernel alone: HIP events on the launch stream, 5 launches
    stream = torch.cuda.current_stream(dev)
    ge0, ge1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ge0.record(stream)
    for _ in range(5):
        buf.compute_returns_and_advantage(last_v, last_d)
    ge1.record(stream)
    sync()
    gae_kernel_ms = ge0.elapsed_time(ge1) / 5
    gae_bytes = T * n * 20 + n * 5  # rewards, values, starts read; advantages, returns written; last values, dones
    # the contiguous layout's fused rollout steps (round 3's per-step path)
    cont = {}
    if world == 1:
        ec = F16Envs(n, stack_k=args.stack, device=dev, seed=args.seed + 7, obs_layout="contiguous")
        ec.reset()
        collect_rollout(ec, DeviceRolloutBuffer(8, n, args.stack, dev), args.seed + 3000, persistent=False)
        sync()
        tc0 = time.perf_counter()
        collect_rollout(ec, buf, args.seed + 5000, persistent=False)
        sync()
        cont = {"rollout_fused_contiguous_s": round(time.perf_counter() - tc0, 4)}
        ec.close()
    # policy in the loop (on_policy_algorithm.py:194-262 with a policy network), eager and with
    # the policy's forwards captured as HIP graphs
    pol = {}
    if args.policy_steps > 0:
        net = MlpActorCritic(args.stack * 15, dev, seed=args.seed)
        pbuf = DeviceRolloutBuffer(args.policy_steps, n, args.stack, dev)

        def policy_leg(pf, vf, bootstrap="deferred"):
            collect_rollout(envs, DeviceRolloutBuffer(8, n, args.stack, dev), policy_fn=pf, value_fn=vf,
                            bootstrap=bootstrap)
            barrier()
            tq0 = time.perf_counter()
            lv, ld = collect_rollout(envs, pbuf, policy_fn=pf, value_fn=vf, bootstrap=bootstrap)
            pbuf.compute_returns_and_advantage(lv, ld)
            sync()
            pol_s = time.perf_counter() - tq0
            o = envs.obs  # the policy's share: its forward (and the value forward) alone, same batch
            for _ in range(3):
                pf(o), vf(o)
            sync()
            tq1 = time.perf_counter()
            for _ in range(50):
                pf(o)
            sync()
            tq2 = time.perf_counter()
            for _ in range(50):
                vf(o)
            sync()
            tq3 = time.perf_counter()
            return {"rollout_plus_gae_s": round(pol_s, 4),
                    "env_steps_per_s": round(n * world * args.policy_steps / pol_s, 1),
                    "ms_per_step": round(pol_s / args.policy_steps * 1e3, 5),
                    "policy_forward_ms": round((tq2 - tq1) / 50 * 1e3, 5),
                    "value_forward_ms": round((tq3 - tq2) / 50 * 1e3, 5)}

        with torch.no_grad():
            eager = policy_leg(net, net.value)
            gp = GraphedPolicy(net, n, args.stack, dev)
            graphed = policy_leg(gp, gp.value)
            graphed_per_step = policy_leg(gp, gp.value, bootstrap="per_step")
        pol = {"policy_in_the_loop": {
            "policy": "MlpActorCritic (SB3 default PPO MlpPolicy shape: pi/vf [64, 64] tanh, Gaussian, random init) "
                      "on the window view; actions clipped in-kernel, timeout bootstrap on device, deferred: "
                      "truncated lanes' terminal observations stashed per step, V once after the loop "
                      "(f16env_window_step_rollout + f16env_bootstrap_stash / _apply), then GAE",
            "steps": args.policy_steps, **graphed,
            "policy_execution": "forward and value forward each captured as a HIP graph (torch.cuda.graph), "
                                "one replay per call (the deferred bootstrap's value call over the stash: eager)",
            "bootstrap_per_step": {**graphed_per_step,
                                   "note": "V over the whole batch of terminal observations every step "
                                           "(f16env_bootstrap_timeouts), as round 4's first version"},
            "eager": eager}}
        del pbuf
    gathered = 0
    t_gather = 0.0
    if world > 1:
        small = DeviceRolloutBuffer(2, 64, args.stack, dev)
        gather_to_rank0(small)  # communicator warm-up
        barrier()
        t3 = time.perf_counter()
        out = gather_to_rank0(buf, chunk_steps=args.gather_chunk)
        barrier()
        t_gather = time.perf_counter() - t3
        if rank == 0:
            gathered = sum(v.numel() * v.element_size() for v in out.values())
        del out
    tt = torch.tensor([t1 - t0, t2 - t1, t_gather, fused_s, gae_kernel_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    shard_bytes = sum(v.numel() * v.element_size() for v in buf.state_dict().values())
    step_kernel = envs.step_kernel_name  # (before close: the name is the handle's)
    envs.close()
    del buf
    torch.cuda.empty_cache()
    fused_ms = float(tt[3]) / T * 1e3
    r = {
        "workload": "BASELINE cfg4: %d envs/GPU x %d GPUs, PPO n_steps=%d, stack=%d, windowed observations, random "
                    "policy (device Philox; values/log-probs zero) -- the policy-in-the-loop rate beside it"
                    % (n, world, T, args.stack),
        "rollout_s": round(float(tt[0]), 4),
        "rollout_env_steps_per_s": round(n * world * T / float(tt[0]), 1),
        "rollout_kernel": "f16_rollout_kernel (the whole rollout in one launch, state on-chip, windowed output)",
        "rollout_fused_steps_s": round(float(tt[3]), 4),
        "rollout_fused_steps_env_steps_per_s": round(n * world * T / float(tt[3]), 1),
        "rollout_fused_ms_per_step": round(fused_ms, 5),
        "window_step_ms_same_envs": round(plain_ms, 5),
        "fused_over_plain_step": round(fused_ms / plain_ms, 4),
        "rollout_step_kernel_ms": round(roll_kern_ms, 5),
        "window_step_kernel_ms_same_envs": round(step_kern_ms, 5),
        "rollout_step_kernel": step_kernel.replace("false>", "true>") + " (the rollout-slot build)",
        **cont,
        "gae_ms": round(float(tt[1]) * 1e3, 3),
        "gae_kernel_ms": round(float(tt[4]), 4),
        "gae_achieved_GBps": round(gae_bytes / (float(tt[4]) * 1e-3) / 1e9, 1),
        "gae_frac_of_hbm_peak": round(gae_bytes / (float(tt[4]) * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
        "gae_bytes": gae_bytes,
        **pol,
        "shard_bytes_per_rank": shard_bytes,
        "gather_s": round(float(tt[2]), 4) if world > 1 else None,
        "gather_bytes_at_rank0": gathered if world > 1 else None,
        "gather_GBps_at_rank0": round(gathered / float(tt[2]) / 1e9, 2) if world > 1 and tt[2] > 0 else None,
        "gather": "%s dist.gather, %d-step chunks, frame-deduplicated obs (newest frame + initial stack)"
                  % ("RCCL" if args.dist_backend == "nccl" else "gloo (rehearsal)", args.gather_chunk)
                  if world > 1 else "n/a (1 GPU)",
    }
    return r


def graph_ms(fn, iters=200):
    """ms per call of `fn` (one kernel launch through the C ABI) with the host out of the loop:
    `iters` calls captured once as a HIP graph (torch.cuda.graph: hipStreamBeginCapture on the
    current stream, which the ctypes launches use), the graph replayed and timed with events.
    What remains per call is the kernel and its dependent-launch boundary. None if capture fails."""
    import torch
    try:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                fn()
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                fn()
        g.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = None
        for _ in range(3):
            s.record()
            g.replay()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / iters
            best = ms if best is None else min(best, ms)
        del g
        return best
    except Exception:  # noqa: BLE001
        return None


def features_bench(envs, stream, iters=200):
    """SURVEY 8f rank 3 beside the headline: the policy feature transform (features.py:37-67,
    15 -> 17 floats per frame) over the env's (N, K, 15) device obs; HBM-bound, 128 B/frame."""
    import torch
    from f16_jsb_amd.features import features
    obs = envs.obs
    out = torch.empty(obs.shape[:-1] + (17,), dtype=torch.float32, device=obs.device)
    for _ in range(10):
        features(obs, out)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    for _ in range(iters):
        features(obs, out)
    e.record(stream)
    torch.cuda.synchronize()
    host_ms = s.elapsed_time(e) / iters
    # the kernel itself: the host's per-call Python + ctypes time (~5-10 us) is longer than the
    # launch, so a host-driven loop measures the wrapper; graph replay takes the host out
    gms = graph_ms(lambda: features(obs, out), iters)
    ms = gms if gms is not None else host_ms
    frames = obs.numel() // 15
    gbps = frames * (15 + 17) * 4 / (ms * 1e-3) / 1e9
    # the same features emitted alongside obs by the step call (F16Envs.step(..., features=)):
    # marginal cost per step vs a plain step, same actions
    # (the window layout has no fused form: the step, then f16env_features_strided on the view)
    n = obs.shape[0]
    act = envs.sample_actions(99, 0)

    def stepf(use):
        if envs.window:
            o = envs.step(act).obs
            if use == 1:
                features(o, out)
            elif use == 2:  # the feature window: one frame per env transformed per step
                envs.obs_features()
        else:
            envs.step(act, features=out if use else None)

    modes = (0, 1, 2) if envs.window else (0, 1)
    for use in modes:
        for _ in range(5):
            stepf(use)
    t = {m: [] for m in modes}
    for _ in range(2):
        for use in modes:
            s.record(stream)
            for _ in range(iters // 2):
                stepf(use)
            e.record(stream)
            torch.cuda.synchronize()
            t[use].append(s.elapsed_time(e) / (iters // 2))
    plain, fused = min(t[0]), min(t[1])
    fw = {}
    if envs.window:
        # the feature-window kernel alone: graph replay of the incremental call after a step
        # (the step and the call are captured together; the step's own replay is subtracted)
        def one_step():
            envs.step(act)

        def step_and_window():
            envs.step(act)
            envs.obs_features()

        g_step = graph_ms(one_step, iters // 4)
        g_both = graph_ms(step_and_window, iters // 4)
        fw = {"step_with_feature_window_ms": round(min(t[2]), 5),
              "feature_window_kernel": "f16_feature_window_kernel",
              "feature_window_bytes_per_env": 64 + 2 * 68,
              "feature_window_calls": dict(envs.feature_window_calls)}
        if g_step is not None and g_both is not None:
            fw["feature_window_ms_graph"] = round(g_both - g_step, 5)
        fw.update(fused_step_legs(envs, act, s, e, iters))
    return {"kernel": "f16_features_strided_kernel" if envs.window else "f16_features_kernel", "frames": frames, "ms": round(ms, 5),
            "timing": "HIP-graph replay of %d launches (kernel + launch boundary)" % iters if gms is not None
            else "host-driven launches", "host_driven_ms": round(host_ms, 5),
            "frames_per_s": round(frames / (ms * 1e-3), 1), "achieved_GBps": round(gbps, 1),
            "frac_of_hbm_peak": round(gbps / HBM_PEAK_GBPS, 4), "bytes_per_frame": 128,
            "step_ms": round(plain, 5), "step_with_features_ms": round(fused, 5), **fw}


def fused_step_legs(envs, act, s, e, iters):
    """Beside the features leg (windowed layout, same env count and K): (1) a fused_features
    handle, whose plain step keeps the feature window in its epilogue (f16env_window_step_ex,
    F16_STEP_FEATURE_WINDOW), step + features per step against the plain
    step; (2) the plain step with its actions drawn in the kernel (step(None, seed, step):
    no sampling launch, no action read; item 5) against sample_actions + step; (3) a fused_poses
    handle (the render/telemetry pose export in the epilogue) against step + f16env_poses. Host-driven
    loops timed by HIP events on the launch stream (the region) and the kernels' own dispatch
    events (profile_kernel)."""
    import torch
    from f16_jsb_amd.env import F16Envs
    out = {}
    fx = F16Envs(envs.n, stack_k=envs.k, seed=1, obs_layout="window", fused_features=True)
    fx.reset()
    for _ in range(8):  # the first step catches the feature window up, the rest fuse
        fx.step(act)
    n2 = iters // 2

    def region(fn):
        best = None
        for _ in range(2):
            torch.cuda.synchronize()
            s.record()
            for t in range(n2):
                fn(t)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / n2
            best = ms if best is None else min(best, ms)
        return best

    fused_ms = region(lambda t: fx.step(act))
    fk, _, _ = fx.profile_kernel(lambda: [fx.step(act) for _ in range(n2)], n2)
    out["fused_features_step_ms"] = round(fused_ms, 5)
    out["fused_features_kernel_ms"] = round(fk, 5)
    out["fused_features_kernel"] = lib_name(fx, 2)
    out["fused_features_calls"] = dict(fx.feature_window_calls)
    fx.close()
    # in-kernel actions on the plain handle (no features): the winx build with act == NULL
    samp = torch.empty_like(act)
    sample_then_step = region(lambda t: (envs.sample_actions(5, t, out=samp), envs.step(samp)))
    in_kernel = region(lambda t: envs.step(None, seed=5, step=t))
    ik, _, _ = envs.profile_kernel(lambda: [envs.step(None, seed=5, step=t) for t in range(n2)], n2)
    out["sample_then_step_ms"] = round(sample_then_step, 5)
    out["in_kernel_actions_step_ms"] = round(in_kernel, 5)
    out["in_kernel_actions_kernel_ms"] = round(ik, 5)
    out["in_kernel_actions_kernel"] = lib_name(envs, 0)
    # (3) the pose export in the step's epilogue (fused_poses, F16_STEP_POSES, ABI 5) against the
    # plain step followed by the separate pose kernel (telemetry.poses of the newest frame)
    from f16_jsb_amd.abi import F16_STEP_POSES
    from f16_jsb_amd.telemetry import poses as _poses
    fp = F16Envs(envs.n, stack_k=envs.k, seed=1, obs_layout="window", fused_poses=True)
    fp.reset()
    pbuf = torch.empty((envs.n, 10), dtype=torch.float32, device=act.device)
    for _ in range(4):
        fp.step(act)
    fused_p = region(lambda t: fp.step(act))
    fpk, _, _ = fp.profile_kernel(lambda: [fp.step(act) for _ in range(n2)], n2)
    step_then_poses = region(lambda t: (envs.step(act), _poses(envs.obs, pbuf)))
    out["fused_poses_step_ms"] = round(fused_p, 5)
    out["fused_poses_kernel_ms"] = round(fpk, 5)
    out["fused_poses_kernel"] = lib_name(fp, F16_STEP_POSES)
    out["step_then_poses_ms"] = round(step_then_poses, 5)
    fp.close()
    return out


def lib_name(envs, flags):
    """The winx kernel instance f16env_window_step_ex launches for `flags` on this handle."""
    from f16_jsb_amd._lib import lib
    return lib().f16env_window_step_ex_kernel_name(envs._h, flags).decode()


def telemetry_bench(envs, stream, iters=200):
    """SURVEY 8f rank 4 beside the headline: render/telemetry poses (jsbsim_gym.py:381-415) of
    every env's newest frame, strided read of the (N, K, 15) obs; HBM-bound, 100 B/env."""
    import torch
    from f16_jsb_amd.telemetry import poses
    obs = envs.obs
    out = torch.empty((obs.shape[0], 10), dtype=torch.float32, device=obs.device)
    for _ in range(10):
        poses(obs, out)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    for _ in range(iters):
        poses(obs, out)
    e.record(stream)
    torch.cuda.synchronize()
    host_ms = s.elapsed_time(e) / iters
    gms = graph_ms(lambda: poses(obs, out), iters)  # the kernel without the wrapper's host time
    ms = gms if gms is not None else host_ms
    n = obs.shape[0]
    gbps = n * 100 / (ms * 1e-3) / 1e9
    return {"kernel": "f16_poses_kernel", "envs": n, "ms": round(ms, 5), "envs_per_s": round(n / (ms * 1e-3), 1),
            "timing": "HIP-graph replay of %d launches (kernel + launch boundary)" % iters if gms is not None
            else "host-driven launches", "host_driven_ms": round(host_ms, 5),
            "achieved_GBps": round(gbps, 1), "frac_of_hbm_peak": round(gbps / HBM_PEAK_GBPS, 4), "bytes_per_env": 100}


def sampler_bench(envs, stream, batches=64, iters=20):
    """The action sampler beside the headline (jsbsim_gym.py:575's action_space.sample() per env,
    the device Philox stream): `batches` steps' actions for every env in ONE launch
    (f16env_sample_actions_steps), 16 B per env-step written; and the one-batch launch
    (f16env_sample_actions) under graph replay for comparison (launch-latency-bound: 1 MB per
    launch at 65 536 envs). Kernel time from HIP events on the launch stream."""
    import torch
    n = envs.n
    out = envs.sample_actions(7, 0, steps=batches)
    for _ in range(3):
        envs.sample_actions(7, 0, out=out, steps=batches)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    for i in range(iters):
        envs.sample_actions(7, i * batches, out=out, steps=batches)
    e.record(stream)
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    nbytes = batches * n * 16
    one = torch.empty((n, 4), dtype=torch.float32, device=envs.device)
    g1 = graph_ms(lambda: envs.sample_actions(7, 0, out=one), 200)
    gbps = nbytes / (ms * 1e-3) / 1e9
    del out
    return {"kernel": "f16_sample_actions_steps_kernel", "envs": n, "batches_per_launch": batches,
            "ms_per_launch": round(ms, 5), "bytes_per_launch": nbytes, "achieved_GBps": round(gbps, 1),
            "frac_of_hbm_peak": round(gbps / HBM_PEAK_GBPS, 4),
            "env_steps_per_s": round(batches * n / (ms * 1e-3), 1),
            "one_batch_launch_ms_graph": None if g1 is None else round(g1, 5),
            "one_batch_frac_of_hbm_peak": None if g1 is None else round(n * 16 / (g1 * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
            "timing": "HIP events around %d back-to-back launches (multi-step); graph replay of 200 launches "
                      "(one batch)" % iters}


def persistent_bench(dev, n, stack, steps, seed):
    """The headline workload (n envs, stack K, random actions, auto-reset) run as ONE
    persistent launch (f16env_rollout_random: actions drawn in-kernel from the same Philox
    stream, state on-chip, per step only the rollout slot written) -- what a step costs without
    the per-step launch, prologue and state traffic. Not the headline: the headline steps
    through the VecEnv boundary with the actions handed in each step."""
    import torch
    from f16_jsb_amd.env import F16Envs
    e = F16Envs(n, stack_k=stack, device=dev, seed=seed)
    e.reset()
    f32 = torch.float32
    fr = torch.empty((steps, n, 15), dtype=f32, device=dev)
    ac = torch.empty((steps, n, 4), dtype=f32, device=dev)
    rw = torch.empty((steps, n), dtype=f32, device=dev)
    ns = torch.empty((steps - 1, n), dtype=f32, device=dev)
    ls = torch.empty(n, dtype=f32, device=dev)
    e.rollout_random(seed, 0, 20, fr[:20], ac[:20], rw[:20], ns[:19], ls)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.rollout_random(seed, 20, steps, fr, ac, rw, ns, ls)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    e.close()
    del fr, ac, rw, ns
    torch.cuda.empty_cache()
    return {"kernel": "f16_rollout_kernel", "envs": n, "stack_k": stack, "steps": steps,
            "ms_per_step": round(el / steps * 1e3, 5), "env_steps_per_s": round(n * steps / el, 1),
            "note": "one launch for all steps, actions drawn in-kernel (random policy); not the headline"}


def cfg2_bench(dev, n=4096, steps=1200):
    """BASELINE cfg2: 4 096 envs on a 64 x 64 altitude x airspeed grid, each trimmed for level
    flight on the device (f16env_trim), then flown with its constant trim action for 1 200
    steps (the parity check of this config is tests/test_gpu_parity.py::
    test_cfg2_trimmed_level_flight_4096). Times the trim and the steps."""
    import numpy as np
    import torch
    from f16_jsb_amd.abi import F16_IC_N
    from f16_jsb_amd.env import F16Envs
    e = F16Envs(n, stack_k=4, device=dev, seed=3, max_steps=10**6)
    ic = np.zeros((n, F16_IC_N))
    ic[:] = np.array(list(e.cfg.ic))
    side = int(round(n ** 0.5))
    hh, uu = np.meshgrid(np.linspace(3000, 30000, side), np.linspace(600, 1200, n // side), indexing="ij")
    ic[:, 2], ic[:, 3] = hh.ravel()[:n], uu.ravel()[:n]
    ic_d = torch.as_tensor(ic, device=dev)
    e.trim(ic_d)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t_ic, res = e.trim(ic_d)
    torch.cuda.synchronize()
    trim_s = time.perf_counter() - t0
    ok = float((res.max(dim=1).values < 1e-2).float().mean())
    ok3 = float((res.max(dim=1).values < 1e-3).float().mean())
    goals = torch.zeros((n, 3), dtype=torch.float32, device=dev)
    goals[:, 2] = 50000.0
    e.reset(goals=goals, ic=t_ic)
    act = torch.zeros((n, 4), dtype=torch.float32, device=dev)
    act[:, 1], act[:, 3] = t_ic[:, 13].float(), t_ic[:, 15].float()
    for _ in range(10):
        e.step(act)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        e.step(act)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    e.close()
    return {"workload": "BASELINE cfg2: %d envs, device trim (alpha, elevator, throttle Newton) on a %dx%d "
                        "altitude x airspeed grid, constant trim action" % (n, side, n // side),
            "trim_ms": round(trim_s * 1e3, 3), "trimmed_fraction": round(ok, 4),
            "trimmed_fraction_1e-3": round(ok3, 4), "trimmed_basis": "max |udot|, |wdot| (ft/s^2), |qdot| (rad/s^2) "
            "below 1e-2 (resp. 1e-3); the slow, high corners of the grid cannot fly level", "steps": steps,
            "ms_per_step": round(el / steps * 1e3, 5), "env_steps_per_s": round(n * steps / el, 1)}


def sb3_compat_bench(dev, n, steps=20):
    """SURVEY 8d 'also reported': the SB3 drop-in mode -- F16VecEnv with numpy returns and the
    per-env infos list (dummy_vec_env.py:56-73 semantics), at the reference's stack K=10 --
    timed at the VecEnv boundary including the device->host copies and the Python infos."""
    import numpy as np
    import torch
    from f16_jsb_amd.env import F16VecEnv
    venv = F16VecEnv(num_envs=n, stack_k=10, device=dev, seed=5, return_numpy=True)
    venv.reset()
    rng = np.random.default_rng(0)
    # numpy actions, as SB3's collect_rollouts hands them over (on_policy_algorithm.py:210-218)
    acts = [rng.uniform([-1, -1, -1, 0], [1, 1, 1, 1], (n, 4)).astype(np.float32) for _ in range(4)]
    for t in range(3):
        venv.step(acts[t % 4])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(steps):
        obs, rew, dones, infos = venv.step(acts[t % 4])
    el = time.perf_counter() - t0
    venv.close()
    return {"envs": n, "stack_k": 10, "steps": steps, "ms_per_step": round(el / steps * 1e3, 3),
            "env_steps_per_s": round(n * steps / el, 1),
            "note": "numpy actions in; numpy obs/rew/dones + N infos out per step (SB3 VecEnv contract, "
                    "PCIe-inclusive: pinned staging, one obs + one packed flag copy, shared info for running lanes)"}


def cfg1_hip_bench(dev, steps=1000):
    """BASELINE cfg1 on the HIP path: ONE env, K = 10, 1 000 random-action steps (numpy
    default_rng(0) actions, uploaded once), the per-step latency of a single-env step launch
    through F16Envs.step -- the GPU is the wrong tool for one env; reported beside the CPU
    oracle's cfg1 figure (cpu_baseline.cfg1)."""
    import numpy as np
    import torch
    from f16_jsb_amd.env import F16Envs
    e = F16Envs(1, stack_k=10, device=dev, seed=0)
    e.reset()
    acts = torch.as_tensor(np.random.default_rng(0).uniform([-1, -1, -1, 0], [1, 1, 1, 1], (steps, 1, 4))
                           .astype(np.float32), device=dev)
    for t in range(20):
        e.step(acts[t])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(steps):
        e.step(acts[t])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    name = e.step_kernel_name
    e.close()
    return {"envs": 1, "stack_k": 10, "steps": steps, "kernel": name, "ms_per_step": round(el / steps * 1e3, 5),
            "env_steps_per_s": round(steps / el, 1)}


def layout_leg(dev, args, layout, steps=300):
    """The headline workload in the other observation layout, beside the headline (N=1): same
    phase spread + burn-in, `steps` timed steps (region HIP events) and the kernel's own
    per-launch duration (dispatch events)."""
    import torch
    from f16_jsb_amd.env import F16Envs
    e = F16Envs(args.envs, stack_k=args.stack, device=dev, seed=args.seed, obs_layout=layout)
    e.reset()
    spread_phases(e, args, dev)
    acts = [e.sample_actions(args.seed + 1000, t) for t in range(16)]
    stream = torch.cuda.current_stream(dev)
    s, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record(stream)
    for t in range(steps):
        e.step(acts[t % 16])
    en.record(stream)
    torch.cuda.synchronize()
    region = s.elapsed_time(en) / steps
    kern_ms, _, _ = e.profile_kernel(lambda: [e.step(acts[t % 16]) for t in range(steps)], steps)
    b, lb = e.stack_bytes_per_env_step(), e.algorithmic_bytes_per_env_step()
    out = {"layout": layout, "kernel": e.step_kernel_name, "region_ms_per_step": round(region, 5),
           "kernel_ms": round(kern_ms, 5), "env_steps_per_s_region": round(args.envs / (region * 1e-3), 1),
           "algorithmic_bytes_per_env_step": lb, "contract_bytes_per_env_step": b,
           "frac_of_hbm_peak": round(lb * args.envs / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5),
           "contract_frac": round(b * args.envs / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5)}
    e.close()
    return out


def load_traffic(envs, stack, state_bytes, layout, name="pmc_traffic.json"):
    """Per-launch HBM bytes of the step kernel from the committed PMC summary, if it was
    measured on this workload, state size and observation layout (cfg5: pmc_traffic_cfg5.json)."""
    p = os.path.join(ROOT, "profiles", name)
    try:
        with open(p) as f:
            d = json.load(f)
        if (d.get("envs") == envs and d.get("stack_k") == stack and d.get("state_bytes") == state_bytes
                and d.get("layout", "contiguous") == layout):
            return d.get("hbm_bytes_per_launch")
    except Exception:  # noqa: BLE001
        pass
    return None


def load_valu(envs, stack, kernel):
    """VALU side of the step kernel (SURVEY 8(d) asks for it beside the HBM fraction): the
    committed SQ-counter summary (tools/pmc_valu.py), if it was measured on this workload.
    The VALU issue peak for one wave per SIMD is one wave64 instruction per 4 cycles."""
    p = os.path.join(ROOT, "profiles", "pmc_valu.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if d.get("envs") == envs and d.get("stack_k") == stack and d.get("kernel") == kernel.split("<")[0]:
            return {"valu_insts_per_wave_step": d["valu_insts_per_wave_step"], "valu_busy_frac": d["valu_busy_frac"],
                    "wait_any_frac": d["wait_any_frac"], "wave_cycles": d["wave_cycles"],
                    "source": "profiles/pmc_valu.json (rocprofv3 --pmc SQ_* passes)"}
    except Exception:  # noqa: BLE001
        pass
    return None


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:  # no launcher around us: start the ranks (launch_ranks makes no GPU call)
            return launch_ranks(args, sys.argv[1:])
        if args.gpus < 1:
            print("[bench] --gpus must be >= 1", file=sys.stderr)
            return 2
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        # under an external launcher the job's size is the launcher's; a mismatch would time and
        # label the wrong configuration
        print("[bench] WORLD_SIZE=%d but --gpus %d" % (world, args.gpus), file=sys.stderr)
        return 2
    if args.launch_selftest:
        launch_selftest(args, world, rank)
        return 0
    import torch
    import torch.distributed as dist

    if args.dist_backend == "gloo":
        # rehearsal only: ranks share the box's GPUs round-robin (device_count does not
        # initialise the GPU); the nccl measurement keeps one GPU per rank
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from f16_jsb_amd.build import build
    from f16_jsb_amd.env import F16VecEnv

    if rank == 0 or world == 1:
        build()
    if world > 1:
        dist.barrier()

    cfg5 = args.workload == "cfg5"
    if args.envs is None:
        args.envs = 131072 if cfg5 else 65536
    n = args.envs
    venv = F16VecEnv(num_envs=n, stack_k=args.stack, device=dev, seed=args.seed, return_numpy=False,
                     env_id_base=rank * n, cfg5=cfg5, obs_layout=args.obs_layout)
    envs = venv.envs
    kernel_name, waves_per_simd = envs.step_kernel_name, envs.waves_per_simd
    venv.reset()
    burn = spread_phases(envs, args, dev)
    pool = args.action_pool if args.action_pool > 0 else args.steps
    # the run's actions pre-generated in HBM by ONE launch each (f16env_sample_actions_steps: the
    # same draws as one f16env_sample_actions launch per step)
    acts = envs.sample_actions(args.seed + 1000, 0, steps=pool)
    warm = torch.empty((max(args.warmup, 1), n, 4), dtype=torch.float32, device=dev)
    if args.warmup > 0:
        envs.sample_actions(args.seed + 2000, 0, out=warm[:args.warmup], steps=args.warmup)
    from f16_jsb_amd.abi import F16C_EP_COUNT
    stream = torch.cuda.current_stream(dev)
    start_ev, end_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # The host operations between the warm-up and the timed region run once here first: the
    # first launch after a new kind of runtime call (a first reduce kernel, a first event
    # record, a fresh allocation) costs the host ~100 us (tools/driver_gap.py,
    # profiles/r03_driver_gap.json), which lands in a 20-step region as ~5 us per step
    envs.get_state()[:, F16C_EP_COUNT].sum()
    start_ev.record(stream)
    end_ev.record(stream)
    torch.cuda.synchronize()
    for t in range(args.warmup):
        envs.step(warm[t])
    torch.cuda.synchronize()

    ep0 = envs.get_state()[:, F16C_EP_COUNT].sum()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # the per-step action views made before the clock starts (indexing acts[t] in the loop costs
    # the host ~2 us per step -- on the critical path of the first launch of a short region)
    act_views = acts.unbind(0)
    gc.disable()  # no collector pause inside the timed steps (a gc.collect() here idles the GPU ~50 ms)
    t0 = time.perf_counter()
    start_ev.record(stream)
    for t in range(args.steps):
        envs.step(act_views[t % pool])
    end_ev.record(stream)
    torch.cuda.synchronize()
    # each rank's own K steps, barrier to barrier; the job's time is the max over ranks (all_reduce
    # below). The closing barrier stays outside the clock: its collective latency (tens of us on
    # RCCL) is not stepping, and a 20-step region would carry it as ~1-2 us per step at N > 1 only
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    gc.enable()
    gpu_ms_per_step = start_ev.elapsed_time(end_ev) / args.steps
    # auto-resets inside the timed region, from the lanes' episode counters (read after it:
    # nothing is added to the timed loop)
    resets_timed = int((envs.get_state()[:, F16C_EP_COUNT].sum() - ep0).item())
    # per-launch duration of the step kernel: start/stop events recorded by each launch's own
    # dispatch packet (hipExtLaunchKernel, f16env_profile_*) on the launch stream, over a
    # second pass of the same steps -- the kernel's execution, as rocprofv3's kernel trace
    # measures it, without the dependent-launch boundary the timed region above includes
    nk = max(200, min(args.steps, 500))  # >= 200 launches: a 20-step run's mean is one outlier away from noise

    def second_pass():
        for t in range(nk):
            envs.step(acts[t % pool])

    kern_ms, kern_min_ms, _ = envs.profile_kernel(second_pass, nk)
    legs_failed = []

    def leg(name, fn, *a, **kw):
        """A side leg beside the headline: its failure keeps the headline line but is reported
        (`legs_failed`) and makes the run exit non-zero."""
        try:
            if args.fail_leg == name:
                raise RuntimeError("forced failure (--fail-leg %s)" % name)
            return fn(*a, **kw)
        except Exception as ex:  # noqa: BLE001
            import traceback
            traceback.print_exc()
            legs_failed.append(name)
            return {"error": "%s: %s" % (type(ex).__name__, ex)}

    feat = leg("features", features_bench, envs, stream)
    telem = leg("telemetry", telemetry_bench, envs, stream)
    sampler = leg("sampler", sampler_bench, envs, stream)
    if world > 1:
        tt = torch.tensor([elapsed, kern_ms, gpu_ms_per_step, kern_min_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, kern_ms, gpu_ms_per_step, kern_min_ms = float(tt[0]), float(tt[1]), float(tt[2]), float(tt[3])
    venv.close()
    del acts, warm
    torch.cuda.empty_cache()
    one = world == 1 and not cfg5
    sb3 = leg("sb3_compat", sb3_compat_bench, dev, n) if (one and not args.no_cpu_baseline) else None
    cfg2 = leg("cfg2", cfg2_bench, dev) if (one and not args.no_cpu_baseline) else None
    persist = leg("persistent", persistent_bench, dev, n, args.stack, 1000, args.seed + 6000) if one else None
    other = "contiguous" if args.obs_layout == "window" else "window"
    layouts = leg("layouts", layout_leg, dev, args, other) if one else None
    rollout = None
    if not cfg5 and args.rollout_envs > 0 and args.rollout_steps > 0:
        rollout = leg("rollout", rollout_bench, args, dev, rank, world)
    cfg1 = leg("cfg1_hip", cfg1_hip_bench, dev) if one else None

    if world > 1:
        # closing barrier: every rank's GPU legs are done before rank 0 samples the CPU baseline,
        # so no timed region of any rank overlaps it
        dist.barrier()
    if rank != 0:
        dist.destroy_process_group()
        if legs_failed:
            print("[bench] rank %d: legs failed: %s" % (rank, ", ".join(legs_failed)), file=sys.stderr, flush=True)
            return 1
        return 0
    total_env_steps = n * world * args.steps
    value = total_env_steps / elapsed
    # roofline bytes: what this layout's step kernel must move per env step (window: state read
    # + written, action, reward, flags and the new frame into both histories, 16 + 2*60 + 4 + 2
    # + 2S; contiguous: SURVEY.md 8(d)'s B(K) with the stack read and rewritten). SURVEY's B(K)
    # -- the step's contract with a materialised K-frame stack -- is reported beside it
    # ("contract_*"): the windowed layout meets that contract without moving its extra bytes.
    bytes_per_env_step = envs.algorithmic_bytes_per_env_step() + (24 if cfg5 else 0)  # + gust state r/w
    contract_bytes = envs.stack_bytes_per_env_step() + (24 if cfg5 else 0)
    bytes_per_launch = bytes_per_env_step * n
    # launch duration used for the roofline: the kernel's average execution time from its own
    # dispatch events (what rocprofv3 --kernel-trace reports); the timed region's GPU time per
    # launch (back-to-back launches incl. the ~1.5 us dependent-kernel boundary) beside it
    # (cfg5: the step is two kernels -- step + deferred reset -- so the region time is used)
    roof_ms = gpu_ms_per_step if cfg5 else kern_ms
    achieved = bytes_per_launch / (roof_ms * 1e-3) / 1e9
    traffic = load_traffic(n, args.stack, envs.state_bytes_per_env, args.obs_layout,
                           "pmc_traffic_cfg5.json" if cfg5 else "pmc_traffic.json")
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": ("BASELINE cfg5: %d F-16 envs per MI355X, randomised ICs + Gauss-Markov wind gusts, "
                         "stack=%d, random actions (device Philox, pre-generated in HBM), auto-reset to a new "
                         "random IC on done" if cfg5 else
                         "BASELINE cfg3: %d F-16 envs per MI355X, waypoint-goal task, stack=%d, random actions "
                         "(device Philox, pre-generated in HBM), auto-reset on done") % (n, args.stack),
            "envs_per_gpu": n,
            "global_envs": n * world,
            "stack_k": args.stack,
            "fdm_frames_per_step": 4,
            "parallelism": "env-sharded x%d (no collective in the step loop)" % world,
            **({"process_group": args.dist_backend + (" (rehearsal: ranks share GPUs)" if args.dist_backend == "gloo" else "")}
               if world > 1 else {}),
        },
        "roofline": {
            # the path has no dense contraction, so the roof the fraction is quoted against is HBM
            # (BASELINE.json); the kernel itself is latency-bound: one wave per SIMD at 65 536 envs,
            # neither HBM (frac) nor VALU issue (valu.valu_busy_frac) saturated
            "bound": "hbm",
            "limiter": ("latency (%s per SIMD: neither HBM nor VALU issue saturated)"
                        % ("one wave" if waves_per_simd == 1 else "%d waves" % waves_per_simd)),
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 5),
            "traffic": traffic,
            "valu": None if cfg5 else load_valu(n, args.stack, kernel_name),
            # cfg5: auto-resets happen inside the step kernel from the reset cache, which
            # f16_ic_fill_kernel refills every F16ENV_ICC_PERIOD (64) steps
            "kernel": kernel_name + (" + f16_ic_fill_kernel (reset cache refill)" if cfg5 else ""),
            "waves_per_simd": waves_per_simd,
            "kernel_ms": round(roof_ms, 5),
            "kernel_ms_min": round(kern_min_ms, 5),
            "kernel_timing": ("HIP events around the timed region / launches (step kernels + the amortised reset-cache refills)" if cfg5 else
                              "start/stop HIP events recorded by each launch's dispatch packet (hipExtLaunchKernel) "
                              "on the launch stream, mean over %d launches" % nk),
            "region_ms_per_launch": round(gpu_ms_per_step, 5),
            "region_timing": "HIP events around the timed region on the launch stream / launches",
            "algorithmic_bytes_per_env_step": bytes_per_env_step,
            "bytes_basis": ("%s layout: 16 (action) + 2 x 60 (new frame into both histories) + 4 + 2 + S + (S - 16) "
                            "(the per-episode state column is written back only by lanes the step reset), S = %d"
                            % (args.obs_layout, envs.state_bytes_per_env) if envs.window else
                            "SURVEY 8(d) B(K) = 16 + 60K + 60(K-1) + 4 + 2 + 2S, S = %d" % envs.state_bytes_per_env),
            # SURVEY 8(d)'s B(K), the bytes of the same step with the K-frame stack materialised
            "contract_bytes_per_env_step": contract_bytes,
            "contract_frac": round(contract_bytes * n / (roof_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5),
            "obs_layout": args.obs_layout,
            "launch_env_steps": n,
        },
        "episode_mix": {
            "done_fraction_mean_timed": round(resets_timed / (n * args.steps), 6),
            "auto_resets_timed": resets_timed,
            "setup": burn,
            "source": "sum of the lanes' episode counters after minus before the timed region / (envs x steps)",
        },
        "features": feat,
        "telemetry": telem,
        "sampler": sampler,
    }
    if rollout is not None:
        out["rollout"] = rollout
    if sb3 is not None:
        out["sb3_compat"] = sb3
    if cfg2 is not None:
        out["cfg2"] = cfg2
    if persist is not None:
        out["persistent_random_policy"] = persist
    if cfg1 is not None:
        out["cfg1_hip"] = cfg1
    if layouts is not None:
        out["layouts"] = {args.obs_layout: {"kernel": kernel_name, "kernel_ms": round(kern_ms, 5),
                                            "region_ms_per_step": round(gpu_ms_per_step, 5)},
                          other: layouts}
    # at every N: the process group RCCL reports and the CPU baseline (rank 0, after the closing
    # barrier above)
    out.update(closing_fields(args, world, n, args.stack, cfg5, leg))
    out["legs_failed"] = legs_failed
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if legs_failed:
        print("[bench] legs failed: %s" % ", ".join(legs_failed), file=sys.stderr, flush=True)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
