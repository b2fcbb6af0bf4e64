"""The rollout gather on the real collective backend (dist.gather on "nccl" had only
ever run over gloo). torch.distributed's "nccl" backend is RCCL on ROCm; with the box's one
GPU the process group has one rank, so RCCL's communicator setup and its gather path execute
on the MI355X and the result must equal the local shard bit for bit (the cross-rank layout is
covered by the gloo tests at world 2 and 3, tests/test_rollout_cpu.py). Run in a child process
so the communicator cannot outlive the test."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_gather_to_rank0_world1(gpu):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_gather_run.py")], env=env, capture_output=True,
                       text=True, timeout=240)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    res = json.loads(lines[-1])
    assert res["backend"] == "nccl" and res["bit_identical"], res
    assert set(res["fields"]) >= {"frames", "actions", "rewards", "episode_starts", "obs0"}, res
