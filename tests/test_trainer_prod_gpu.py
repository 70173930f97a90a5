"""The Trainer's production update at production size: the shipped model
(configs/16x16x40_medium.yaml: 96 channels x 5 blocks, dropout 0.05, belief heads on), a real
rollout of 4096 envs x 8 steps through the HIP env, GAE, and one 4096-sample stratified
minibatch; ppo_update (reference ppo.py:23-119) on

  * the fused fp16 path with a GradScaler (the Trainer's default AMP, train_rl.py:415-420),
  * PyTorch's own fp16 autocast chain (model.fused = False), and
  * an fp32 PyTorch chain (MIOpen GEMM convolutions, MIOPEN_DEBUG_CONV_WINOGRAD=0),

all three from the same weights with the same keyed Dropout2d masks (ms_amd.dropout). The fused
gradients must sit within max(5e-2, 2 x PyTorch-fp16-autocast error) of the fp32 gradients per
tensor -- the bound of tests/test_parity_gpu.py's fixture-sized Trainer test -- and the loss terms
within 2e-2 relative.
"""
from __future__ import annotations

import os

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _record_grads(model, opt):
    grads = {}
    step0 = opt.step

    def step(*a, **k):
        for n, p in model.named_parameters():
            if p.grad is not None:
                grads[n] = p.grad.detach().clone()
        return step0(*a, **k)
    opt.step = step
    return grads


def test_trainer_fp16_update_shipped_model_4096_envs(gpu):
    from ms_amd.dropout import MINIBATCH, keyed_dropout, mix_seed
    from ms_amd.models import build_model
    from ms_amd.ppo import FlatGrads, ppo_update
    from ms_amd.rollout import collect_rollout
    from ms_amd.train import Trainer, load_config
    cfg, env_d, model_d, extras = load_config(os.path.join(ROOT, "configs", "16x16x40_medium.yaml"))
    cfg.num_envs, cfg.steps_per_env = 4096, 8
    tr = Trainer(cfg, env_d, model_d, extras, seed=0, amp="fp16", device=gpu)
    pc = tr.ppo_cfg
    assert pc.aux_mine_weight > 0 and pc.aux_mine_calib_weight > 0
    tr.model.train()
    buf, aux = collect_rollout(tr.vec, tr.model, cfg.steps_per_env, gpu, pc.aux_mine_weight,
                               pc.aux_mine_calib_weight, amp_dtype=torch.float16, sample_seed=17)
    buf.compute_gae(aux["last_values"], gamma=cfg.gamma, lam=cfg.gae_lambda)
    batch = next(iter(buf.get_stratified_minibatches(cfg.mini_batches, tr.stripes_local, tr.stripe_begin, seed=5)))
    assert batch.obs.shape[0] == 4096 and float(batch.mine_valid.float().sum()) > 0
    init = {k: v.detach().clone() for k, v in tr.model.state_dict().items()}
    del tr
    mcfg = {k: v for k, v in model_d.items() if k != "name"}
    runs = {}
    for mode in ("fused-fp16", "torch-fp16", "fp32"):
        m = build_model("cnn_residual", obs_shape=(10, 16, 16), model_cfg=dict(mcfg)).to(gpu)
        m.load_state_dict(init)
        m.train()
        m.fused = mode == "fused-fp16"
        amp = None if mode == "fp32" else torch.float16
        if amp is not None:
            with torch.autocast("cuda", dtype=amp):
                assert m.use_fused(batch.obs) == m.fused
        opt = torch.optim.AdamW(m.parameters(), lr=cfg.lr)
        grads = _record_grads(m, opt)
        scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 10) if amp is not None else None
        with keyed_dropout(m, batch.rows, mix_seed(0, MINIBATCH), 123):
            stats = ppo_update(m, opt, batch, pc, scaler, amp_dtype=amp, flat_grads=FlatGrads(m.parameters()))
        assert grads, f"{mode}: the optimizer did not step (overflow skip)"
        runs[mode] = (stats, grads)
        del m, opt
        torch.cuda.empty_cache()
    ref_stats, ref_grads = runs["fp32"]
    for k in ("loss", "policy_loss", "value_loss", "entropy", "aux_bce", "aux_calib"):
        e = abs(runs["fused-fp16"][0][k] - ref_stats[k]) / max(abs(ref_stats[k]), 1e-3)
        print(f"stat {k}: fused {runs['fused-fp16'][0][k]:.6f} fp32 {ref_stats[k]:.6f} rel {e:.2e} "
              f"torch-fp16 {runs['torch-fp16'][0][k]:.6f}")
        assert e < 2e-2, k
    worst = 0.0
    for k, g in ref_grads.items():
        if k == "policy_head.2.bias":  # exact gradient 0 (log-softmax shift invariance)
            continue
        e_f, e_t = _rel(runs["fused-fp16"][1][k], g), _rel(runs["torch-fp16"][1][k], g)
        worst = max(worst, e_f / max(5e-2, 2 * e_t))
        assert e_f <= max(5e-2, 2 * e_t), (k, e_f, e_t)
    print(f"worst gradient error / bound = {worst:.3f}")


def test_keyed_dropout_masks(gpu):
    """ms_dropout_masks: values keep / (1 - p) in {0, 1/(1-p)}, keep rate ~ 1 - p, a function of
    (seed, counter, global sample id, block, channel) only: any subset of rows (a rank's shard, a
    minibatch's rows in any order) draws exactly the masks those rows draw in the full set."""
    from ms_amd.dropout import dropout_masks
    p = 0.05
    rows = torch.arange(7, 7 + 20000, dtype=torch.int64, device=gpu)
    m = dropout_masks(rows, 5, 96, p, seed=11, counter=3)
    assert m.shape == (5, 20000, 96)
    scale = torch.tensor(1.0 / (1.0 - p), dtype=torch.float32)
    assert bool(((m == 0) | (m == scale.item())).all())
    keep = float((m > 0).float().mean())
    assert abs(keep - (1 - p)) < 3e-3, keep
    perm = torch.randperm(20000, device=gpu)[:4096]
    sub = dropout_masks(rows[perm], 5, 96, p, seed=11, counter=3)
    assert torch.equal(sub, m[:, perm])
    other = dropout_masks(rows, 5, 96, p, seed=11, counter=4)
    assert float((other != m).float().mean()) > 0.05  # a new counter is a new draw
    # block / channel masks are not correlated with each other
    k = (m > 0).float()
    c = torch.corrcoef(torch.stack([k[0].flatten(), k[1].flatten()]))[0, 1]
    assert abs(float(c)) < 0.02


def test_keyed_dropout_fused_equals_chain(gpu):
    """With a key set, the fused trunk (fp16) and the PyTorch chain apply the same Dropout2d
    masks: their train-mode outputs agree at the fused path's eval-mode accuracy, and both differ
    from the eval-mode output."""
    from ms_amd.dropout import keyed_dropout
    from ms_amd.models import build_model
    torch.manual_seed(0)
    m = build_model("cnn_residual", obs_shape=(10, 16, 16),
                    model_cfg=dict(stem_channels=96, blocks=2, dropout=0.3, value_hidden=32)).to(gpu)
    obs = (torch.rand(64, 10, 16, 16, device=gpu) < 0.1).float()
    rows = torch.arange(1000, 1064, device=gpu)
    outs = {}
    for fused in (True, False):
        m.fused = fused
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16), keyed_dropout(m, rows, 5, 9):
            m.train()
            outs[fused] = m(obs)[0].float()
            m.eval()
            outs[("eval", fused)] = m(obs)[0].float()
    e_train = _rel(outs[True], outs[False])
    e_eval = _rel(outs[("eval", True)], outs[("eval", False)])
    print(f"fused vs chain: train {e_train:.2e} eval {e_eval:.2e}")
    assert e_train < max(2e-2, 3 * e_eval)
    assert _rel(outs[True], outs[("eval", True)]) > 10 * e_train
