"""bench.py --gpus N without an external launcher: the parent starts N rank
processes through torch.distributed.run, relays rank 0's JSON line and exits non-zero when a
rank fails. CPU only: the ranks run --launch-selftest (join a gloo group, agree on the world
size, rank 0 prints the launch fields), so no GPU call is made anywhere."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout, env=e)


def test_gpus2_spawns_two_ranks_and_relays_rank0_line():
    p = _run(["--gpus", "2", "--launch-selftest", "--cpu-seconds", "0.3"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout  # exactly the relayed line on stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_joined"] == 2
    assert d["config"]["global_envs"] == 2 * 65536
    # the N > 1 line carries the CPU baseline and the group's world size
    # (rccl_world is the nccl group's size; this rehearsal's group is gloo, so it reads None)
    assert "rccl_world" in d and d["rccl_world"] is None
    assert d["process_group"] == {"backend": "gloo", "world_size": 2}
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1, cb


def test_gpus3_envs_scale_with_world():
    p = _run(["--gpus", "3", "--envs", "1000", "--launch-selftest", "--no-cpu-baseline"])
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 3 and d["config"]["global_envs"] == 3000


def test_failing_rank_makes_the_launcher_exit_nonzero():
    p = _run(["--gpus", "2", "--launch-selftest", "--selftest-fail-rank", "1"])
    assert p.returncode != 0
    assert '"metric"' not in p.stdout


def test_external_launcher_world_size_must_match_gpus():
    p = _run(["--gpus", "1", "--launch-selftest"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 1" in p.stderr


def test_gpus1_runs_in_process():
    # --gpus 1 is the driver's N = 1 command: no launcher, the rank runs here (selftest: gloo world 1)
    p = _run(["--gpus", "1", "--launch-selftest", "--no-cpu-baseline"],
             env={"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29611", "WORLD_SIZE": "1", "RANK": "0"})
    assert p.returncode == 0, p.stderr[-3000:]
    assert "launching" not in p.stderr
    line = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')][-1]  # (gloo logs to stdout too)
    assert json.loads(line)["n_gpus"] == 1
