"""The multi-rank Trainer path on one GPU: two processes on
cuda:0 joined by the gloo backend, each running ``Trainer.update`` on its half
of the global env list (``shard=(r, 2)``), against one process running the
whole list.

What must hold, and why it can:
* the rollouts are identical -- envs are contiguous blocks of the global seed
  list and the sampler hash is keyed by the GLOBAL env index, so rank r's
  buffer rows are the unsharded run's rows for its envs;
* the updated parameters agree within the DP tolerance of
  tests/test_dist_gloo.py -- minibatches are stratified over env stripes
  (RolloutBuffer.get_stratified_minibatches), so rank r's minibatch k is its
  part of the unsharded minibatch k, and the flat-gradient all-reduce averages
  equal-sized rank means.
This exercises Trainer's world > 1 code: env shard, broadcast_module,
FlatGrads.all_reduce_mean and the (pos, count) all-reduce of the belief loss.
"""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG_DIR, ROOT

pytestmark = pytest.mark.gpu

LR = 3e-4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(model):
    from ms_amd.train import PPOTrainConfig
    cfg = PPOTrainConfig(H=9, W=9, mine_count=10, num_envs=32, steps_per_env=8, mini_batches=2, ppo_epochs=2,
                         lr=LR, aux_mine_weight=0.05, aux_mine_calib_weight=0.01, total_updates=10)
    model_d = {"name": "cnn_residual", "dropout": 0.0, **model}
    return cfg, {}, model_d, {}


def _run(rank, world, model, amp, dev):
    from ms_amd.dist import DistInfo
    from ms_amd.train import Trainer
    cfg, env_d, model_d, extras = _cfg(model)
    info = DistInfo(rank=rank, world=world, local_rank=0, group=dist.group.WORLD if world > 1 else None)
    tr = Trainer(cfg, env_d, model_d, extras, seed=3, info=info, amp=amp, device=dev)
    init = {k: v.detach().cpu().clone() for k, v in tr.model.state_dict().items()}
    tr.update(0)
    b = tr.buffer
    roll = {k: getattr(b, k).detach().cpu().clone() for k in
            ("obs", "action_mask", "actions", "logp", "rewards", "dones", "values", "mine_labels", "mine_valid")}
    return roll, {k: v.detach().cpu().clone() for k, v in tr.model.state_dict().items()}, tr.strata, init


def _worker(rank, world, port, out_dir, model, amp):
    import sys
    sys.path[:0] = [PKG_DIR, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    torch.set_float32_matmul_precision("highest")
    roll, params, strata, _ = _run(rank, world, model, amp, dev)
    torch.save({"roll": roll, "params": params, "strata": strata}, os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


def _compare(tmp_path, model, amp, atol_noise, tol_fp, tol_delta=None):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), model, amp), nprocs=2, join=True)
    torch.set_float32_matmul_precision("highest")
    roll1, params1, strata, init = _run(0, 1, model, amp, torch.device("cuda:0"))
    r = [torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(2)]
    assert strata == 8 and r[0]["strata"] == r[1]["strata"] == 8
    T, N = 8, 32
    for k, full in roll1.items():
        full = full.view(T, N, *full.shape[1:])
        halves = [x["roll"][k].view(T, N // 2, *full.shape[2:]) for x in r]
        sharded = torch.cat(halves, dim=1)
        if k in ("logp", "values"):
            torch.testing.assert_close(sharded, full, rtol=tol_fp, atol=tol_fp, msg=k)
        else:
            assert torch.equal(sharded, full), k
    for k, v in params1.items():
        assert torch.equal(r[0]["params"][k], r[1]["params"][k]), k  # ranks stay in lockstep
        d = (r[0]["params"][k] - v).abs()
        if k == "policy_head.2.bias":
            # log-softmax is shift invariant: this gradient is 0 in exact arithmetic, so AdamW
            # turns rounding noise into +-lr steps; only the step-size bound below applies
            assert float(d.max()) <= 4 * 2 * LR + 1e-6
            continue
        # AdamW turns summation-order rounding on near-zero gradients into up to +-lr per step
        # (4 steps here); everything else must agree closely
        assert float(d.max()) <= 4 * 2 * LR + 1e-6, k
        if tol_delta is None:
            frac_off = float((d > atol_noise).float().mean())
            assert frac_off < 0.02, (k, frac_off)
        else:
            # bf16: the value head's autocast GEMMs round differently at another batch size, so
            # compare whole update steps: relative L2 of (2-rank step - 1-rank step)
            d1, d2 = v - init[k], r[0]["params"][k] - init[k]
            e = float((d2 - d1).norm() / d1.norm().clamp_min(1e-12))
            print(f"bf16 DP step error {k}: {e:.3e}")
            assert e < tol_delta, (k, e)


def test_two_rank_trainer_equals_one_rank_fp32(gpu, tmp_path):
    _compare(tmp_path, dict(stem_channels=16, blocks=2, value_hidden=32), "fp32", atol_noise=2e-5, tol_fp=1e-5)


def test_two_rank_trainer_equals_one_rank_fused_bf16(gpu, tmp_path):
    """The production path (fused MFMA trunk, bf16 autocast) through the same DP machinery."""
    _compare(tmp_path, dict(stem_channels=96, blocks=1, value_hidden=32), "bf16", atol_noise=None, tol_fp=1e-2,
             tol_delta=0.1)
