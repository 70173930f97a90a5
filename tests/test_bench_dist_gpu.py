"""bench.py's N>1 path as the driver launches it (``torch.distributed.run``, one process per
rank), rehearsed on one GPU: two ranks share cuda:0 over gloo (``MS_BENCH_BACKEND=gloo``).

What must hold: rank 0 prints ONE JSON line whose env lines are sharded (``envs_total`` =
2 x envs per GPU, max-over-ranks timing behind barriers) and whose PPO line ran the
Trainer's flat-gradient all-reduce over the global env list. Sizes are small; the figures
are not performance claims.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_one_gpu_gloo():
    env = dict(os.environ, MS_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--envs", "1024", "--steps", "20", "--warmup", "3",
           "--extras", "9x9x10:2048", "--ppo-updates", "1", "--ppo-steps-per-env", "8"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "weak"
    assert out["config"]["envs_per_gpu"] == 1024 and out["config"]["envs_total"] == 2048
    assert out["value"] > 0 and out["roofline"]["frac"] > 0
    assert "cpu_baseline" not in out  # N=1 only
    (pt,) = out["north_star_points"]
    assert pt["board"] == "9x9x10" and pt["envs_total"] == 4096 and pt["value"] > 0
    assert pt["multistep"]["value"] > 0
    ppo = out["ppo"]
    assert ppo["envs_total"] == 2048 and ppo["steps_per_env"] == 8 and ppo["updates_per_s"] > 0
    assert ppo["loss"] == ppo["loss"]  # finite, not NaN
