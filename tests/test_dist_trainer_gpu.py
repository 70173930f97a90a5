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
* Dropout2d masks are keyed by GLOBAL sample id (ms_amd.dropout), so the
  dropout-on runs (fused fp16 + GradScaler, the default AMP) follow the same
  rule.
* an fp16 overflow on ONE rank makes EVERY rank skip the step and halve the
  GradScaler scale: the all-reduce precedes unscale_, so the inf reaches all
  ranks (ppo.py:97-106, train_rl.py:415-420 in the reference).
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


def _inject_overflow(model):
    """The first backward's gradient of one parameter becomes +inf (on the rank that calls this)."""
    n = {"calls": 0}

    def hook(g):
        n["calls"] += 1
        return g + float("inf") if n["calls"] == 1 else g
    model.value_head[6].bias.register_hook(hook)
    return n


def _capture_first_grads(model):
    """The gradients the first minibatch's optimizer step sees -- after the flat-bucket all-reduce
    (DP) and GradScaler.unscale_, before clipping and AdamW -- keyed by parameter name."""
    import torch.nn.utils as U
    orig = U.clip_grad_norm_
    names = {id(p): n for n, p in model.named_parameters()}
    box = {}

    def clip(params, *a, **kw):
        params = list(params)
        if not box:
            box.update({names[id(p)]: p.grad.detach().float().cpu().clone() for p in params if p.grad is not None})
        return orig(params, *a, **kw)
    U.clip_grad_norm_ = clip
    return box, (lambda: setattr(U, "clip_grad_norm_", orig))


def _run(rank, world, model, amp, dev, inject=False):
    from ms_amd.dist import DistInfo
    from ms_amd.train import Trainer
    cfg, env_d, model_d, extras = _cfg(model)
    info = DistInfo(rank=rank, world=world, local_rank=0, group=dist.group.WORLD if world > 1 else None)
    tr = Trainer(cfg, env_d, model_d, extras, seed=3, info=info, amp=amp, device=dev)
    init = {k: v.detach().cpu().clone() for k, v in tr.model.state_dict().items()}
    scale0 = tr.scaler.get_scale() if tr.scaler is not None else None
    hooked = _inject_overflow(tr.model) if inject else None
    grads, restore = _capture_first_grads(tr.model)
    try:
        tr.update(0)
    finally:
        restore()
    if hooked is not None:
        assert hooked["calls"] == cfg.ppo_epochs * cfg.mini_batches
    b = tr.buffer
    roll = {k: getattr(b, k).detach().cpu().clone() for k in
            ("obs", "action_mask", "actions", "logp", "rewards", "dones", "values", "mine_labels", "mine_valid")}
    scale = (scale0, tr.scaler.get_scale()) if tr.scaler is not None else None
    return roll, {k: v.detach().cpu().clone() for k, v in tr.model.state_dict().items()}, tr.strata, init, scale, grads


def _worker(rank, world, port, out_dir, model, amp, inject_rank):
    import sys
    sys.path[:0] = [PKG_DIR, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    torch.set_float32_matmul_precision("highest")
    roll, params, strata, _, scale, grads = _run(rank, world, model, amp, dev, inject=(rank == inject_rank))
    torch.save({"roll": roll, "params": params, "strata": strata, "scale": scale, "grads": grads},
               os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


def _compare(tmp_path, model, amp, tol_fp, tol_delta, inject_rank=-1, tol_grad=None):
    """2 ranks vs 1 rank: identical rollouts, ranks in lockstep, per tensor the relative L2 of the
    first minibatch's all-reduced gradient against the one-rank gradient below ``tol_grad`` (before
    AdamW, whose sign-like first step magnifies rounding noise: a broken all-reduce scaling of
    one tensor shows here), and of (2-rank update step - 1-rank update step) below ``tol_delta``.
    With ``inject_rank`` >= 0 that rank (and the 1-rank run) overflows on the first minibatch."""
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), model, amp, inject_rank), nprocs=2, join=True)
    torch.set_float32_matmul_precision("highest")
    roll1, params1, strata, init, scale1, grads1 = _run(0, 1, model, amp, torch.device("cuda:0"),
                                                        inject=inject_rank >= 0)
    r = [torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(2)]
    if tol_grad is not None:
        assert set(grads1) == set(r[0]["grads"]) == set(r[1]["grads"]) and len(grads1) > 0
        gworst = 0.0
        for k, g in grads1.items():
            assert torch.equal(r[0]["grads"][k], r[1]["grads"][k]), k  # one all-reduced bucket
            if k == "policy_head.2.bias":  # 0 in exact arithmetic (log-softmax shift invariance)
                continue
            e = float((r[0]["grads"][k] - g).norm() / g.norm().clamp_min(1e-30))
            gworst = max(gworst, e)
            # the value MLP runs on PyTorch's 16-bit autocast GEMMs, whose kernels (and so the
            # rounding of their 16-bit outputs) depend on the row count: 5x the bound there
            bound = tol_grad * (5 if (k.startswith("value_head") and amp != "fp32") else 1)
            assert e < bound, (k, e, bound)
        print(f"{amp} DP worst per-tensor relative gradient error {gworst:.3e} (bound {tol_grad})")
    assert strata == 8 and r[0]["strata"] == r[1]["strata"] == 8
    if scale1 is not None:
        # every rank keeps the same GradScaler state as the one-rank run; an overflow on one
        # rank halved the scale everywhere (growth_interval 2000: no growth within one update)
        assert r[0]["scale"] == r[1]["scale"] == scale1, (r[0]["scale"], r[1]["scale"], scale1)
        if inject_rank >= 0:
            assert scale1[1] <= scale1[0] * 0.5
    T, N = 8, 32
    for k, full in roll1.items():
        full = full.view(T, N, *full.shape[1:])
        halves = [x["roll"][k].view(T, N // 2, *full.shape[2:]) for x in r]
        sharded = torch.cat(halves, dim=1)
        if k in ("logp", "values"):
            torch.testing.assert_close(sharded, full, rtol=tol_fp, atol=tol_fp, msg=k)
        else:
            assert torch.equal(sharded, full), k
    worst = 0.0
    n_steps = 4 - (1 if inject_rank >= 0 else 0)  # optimizer steps taken (2 epochs x 2 minibatches)
    for k, v in params1.items():
        assert torch.equal(r[0]["params"][k], r[1]["params"][k]), k  # ranks stay in lockstep
        d = (r[0]["params"][k] - v).abs()
        # AdamW turns summation-order rounding on near-zero gradients into up to +-lr per step
        assert float(d.max()) <= n_steps * 2 * LR + 1e-6, k
        if k == "policy_head.2.bias":
            # log-softmax is shift invariant: this gradient is 0 in exact arithmetic, so AdamW
            # turns rounding noise into +-lr steps; only the step-size bound above applies
            continue
        d1, d2 = v - init[k], r[0]["params"][k] - init[k]
        e = float((d2 - d1).norm() / d1.norm().clamp_min(1e-12))
        worst = max(worst, e)
        assert e < tol_delta, (k, e)
    print(f"{amp} DP worst per-tensor relative step error {worst:.3e} (bound {tol_delta})")


def test_two_rank_trainer_equals_one_rank_fp32(gpu, tmp_path):
    """fp32 PyTorch chain: only summation order differs, so the update steps agree closely."""
    _compare(tmp_path, dict(stem_channels=16, blocks=2, value_hidden=32), "fp32", tol_fp=1e-5, tol_delta=2e-2,
             tol_grad=1e-5)


def test_two_rank_trainer_equals_one_rank_fp32_dropout(gpu, tmp_path):
    """Dropout on: the keyed masks make rank r's samples draw the one-GPU run's masks."""
    _compare(tmp_path, dict(stem_channels=16, blocks=2, value_hidden=32, dropout=0.05), "fp32", tol_fp=1e-5,
             tol_delta=2e-2, tol_grad=1e-5)


def test_two_rank_trainer_equals_one_rank_fused_bf16(gpu, tmp_path):
    """The production path (fused MFMA trunk, bf16 autocast) through the same DP machinery.
    The value head's autocast GEMMs round differently at another batch size, hence the looser
    bound."""
    _compare(tmp_path, dict(stem_channels=96, blocks=1, value_hidden=32), "bf16", tol_fp=1e-2, tol_delta=0.1,
             tol_grad=2e-3)


def test_two_rank_trainer_equals_one_rank_fused_fp16_scaler_dropout(gpu, tmp_path):
    """The default AMP: fused fp16 trunk + GradScaler, dropout 0.05 (keyed masks)."""
    _compare(tmp_path, dict(stem_channels=96, blocks=1, value_hidden=32, dropout=0.05), "fp16", tol_fp=1e-2,
             tol_delta=0.1, tol_grad=2e-3)


def test_fp16_overflow_on_one_rank_skips_on_every_rank(gpu, tmp_path):
    """An inf gradient on rank 1 only: both ranks skip that step and halve the scale together,
    and the run equals a one-rank run that overflowed at the same minibatch."""
    _compare(tmp_path, dict(stem_channels=96, blocks=1, value_hidden=32, dropout=0.05), "fp16", tol_fp=1e-2,
             tol_delta=0.1, inject_rank=1)
