"""RCCL (torch.distributed's "nccl" backend on ROCm) on gfx950, before the driver's 8-GPU run.

A child process (one rank, world 1, 127.0.0.1 rendezvous) initialises the nccl backend exactly as
bench.py / ms_amd.dist.init_from_env do (``device_id`` given), then runs the data-parallel
``ppo_update`` (group=WORLD, flat-gradient bucket) of the shipped 96x5 model on one fp16 minibatch:
the flat-bucket all-reduce and the (pos, count) all-reduce of the belief loss both go through RCCL.
With one rank an all-reduce mean is the identity, so the gradients the optimizer steps on and the
stepped parameters must equal the group-less call BITWISE. It also times the 3.80 MB all-reduce
(one per minibatch). Reference: SURVEY.md §8(e); /root/reference/train_rl.py:337
(the reference itself is single-device)."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import PKG_DIR, ROOT

pytestmark = pytest.mark.gpu

CHILD = r'''
import copy, json, os, sys, time
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["MS_PKG_DIR"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
from ms_amd.buffers import Batch
from ms_amd.models import build_model
from ms_amd.ppo import FlatGrads, PPOConfig, ppo_update

dev = torch.device("cuda", 0)
torch.manual_seed(0)
m0 = build_model("cnn_residual", obs_shape=(10, 16, 16),
                 model_cfg=dict(stem_channels=96, blocks=5, dropout=0.0, value_hidden=256)).to(dev).train()
M = 2048
g = torch.Generator(device=dev).manual_seed(0)
rev = torch.rand(M, 16, 16, device=dev, generator=g) < 0.4
cnt = torch.randint(0, 9, (M, 16, 16), device=dev, generator=g)
obs = torch.zeros(M, 10, 16, 16, device=dev)
obs[:, 0] = rev.float()
obs.scatter_(1, (1 + cnt).unsqueeze(1), rev.float().unsqueeze(1))
mask = ~rev.view(M, -1)
acts = torch.multinomial(mask.float() + 1e-6, 1, generator=g).squeeze(1)
b = Batch(obs=obs, action_mask=mask, actions=acts, old_logp=-torch.rand(M, device=dev, generator=g) * 5,
          values=torch.randn(M, device=dev, generator=g), advantages=torch.randn(M, device=dev, generator=g),
          returns=torch.randn(M, device=dev, generator=g),
          mine_labels=(torch.rand(M, 16, 16, device=dev, generator=g) < 0.15).float(), mine_valid=~rev)
cfg = PPOConfig(aux_mine_weight=0.05, aux_mine_calib_weight=0.01)

def run(group):
    m = copy.deepcopy(m0)
    opt = torch.optim.AdamW(m.parameters(), lr=3e-4)
    fg = FlatGrads(m.parameters())
    scaler = torch.amp.GradScaler("cuda")
    st = ppo_update(m, opt, b, cfg, scaler, amp_dtype=torch.float16, group=group, flat_grads=fg, sync_stats=True)
    torch.cuda.synchronize()
    return fg.flat.clone(), torch.cat([p.detach().flatten() for p in m.parameters()]), st, fg

g0, p0, s0, _ = run(None)
g1, p1, s1, fg = run(dist.group.WORLD)
g2, p2, s2, _ = run(None)

def diff(a, b):
    d = (a - b).abs()
    return {"n": int((d > 0).sum()), "max": float(d.max()), "first": int((d > 0).nonzero()[0]) if (d > 0).any() else -1}

res = {"grads_equal": bool(torch.equal(g0, g1)), "params_equal": bool(torch.equal(p0, p1)),
       "repeat_equal": bool(torch.equal(g0, g2)), "diff_group": diff(g0, g1), "diff_repeat": diff(g0, g2),
       "loss": [float(s0["loss"]), float(s1["loss"])], "finite": bool(torch.isfinite(g1).all()),
       "flat_numel": fg.flat.numel()}
for _ in range(5):
    fg.all_reduce_mean(dist.group.WORLD)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(20):
    fg.all_reduce_mean(dist.group.WORLD)
torch.cuda.synchronize()
res["allreduce_ms"] = (time.perf_counter() - t) / 20 * 1e3
x = torch.arange(6, dtype=torch.float32, device=dev)
dist.all_reduce(x)  # the 6-float stats all-reduce shape
res["small_ok"] = bool(torch.equal(x, torch.arange(6, dtype=torch.float32, device=dev)))
dist.barrier()
dist.destroy_process_group()
print("RESULT " + json.dumps(res), flush=True)
'''


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_world1_ppo_update_equals_groupless(gpu, tmp_path):
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), MS_PKG_DIR=PKG_DIR, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert r.returncode == 0 and line, f"rc {r.returncode}\nstdout:\n{r.stdout[-3000:]}\nstderr:\n{r.stderr[-3000:]}"
    res = json.loads(line[-1][len("RESULT "):])
    print(res)
    (tmp_path / "rccl.json").write_text(json.dumps(res))
    assert res["flat_numel"] == 950947
    assert res["finite"] and res["small_ok"]
    assert res["grads_equal"] and res["params_equal"], res
    assert res["loss"][0] == res["loss"][1]
    assert 0 < res["allreduce_ms"] < 50
