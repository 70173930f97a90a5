"""GPU checks of the rollout side: GAE kernel (bit-exact vs the reference
golden and the oracle), masked sampler, on-device collect_rollout replayed
through the oracle, and one PPO update of the trainer."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import ROOT, golden
import oracle as O

pytestmark = pytest.mark.gpu


def test_gae_kernel_golden_bitexact(gpu):
    from ms_amd.buffers import RolloutBuffer
    z = golden("gae.npz")
    T, N = int(z["T"]), int(z["N"])
    b = RolloutBuffer(N, T, (10, 4, 4), 16, gpu)
    b.rewards.copy_(torch.from_numpy(z["rewards"]))
    b.values.copy_(torch.from_numpy(z["values"]))
    b.dones.copy_(torch.from_numpy(z["dones"]))
    b.compute_gae(torch.from_numpy(z["last_values"]).to(gpu), gamma=float(z["gamma"]), lam=float(z["lam"]))
    assert np.array_equal(b.advantages.cpu().numpy(), z["advantages"])
    assert np.array_equal(b.returns.cpu().numpy(), z["returns"])


def test_gae_kernel_vs_oracle_full_size(gpu):
    from ms_amd.buffers import RolloutBuffer
    T, N = 64, 4096
    g = torch.Generator().manual_seed(1)
    r, v = torch.randn(T * N, generator=g), torch.randn(T * N, generator=g)
    d, lv = torch.rand(T * N, generator=g) < 0.3, torch.randn(N, generator=g)
    b = RolloutBuffer(N, T, (10, 1, 1), 1, gpu)
    b.rewards.copy_(r)
    b.values.copy_(v)
    b.dones.copy_(d)
    b.compute_gae(lv.to(gpu))
    adv, ret = O.gae(r.view(T, N).numpy(), v.view(T, N).numpy(), d.view(T, N).numpy(), lv.numpy())
    assert np.array_equal(b.advantages.cpu().numpy(), adv.reshape(-1))
    assert np.array_equal(b.returns.cpu().numpy(), ret.reshape(-1))


def test_sampler_logp_and_mask(gpu):
    from ms_amd.rollout import sample_masked
    g = torch.Generator(device=gpu).manual_seed(0)
    N, A = 4096, 256
    logits = torch.randn(N, A, device=gpu, generator=g) * 3
    mask = torch.rand(N, A, device=gpu, generator=g) < 0.3
    mask[0] = False  # all-invalid row -> treated as all valid (train_rl.py:166-168)
    a, lp = sample_masked(logits, mask, seed=5, counter=0)
    m2 = mask.clone()
    m2[0] = True
    assert bool(m2.gather(1, a[:, None]).all())
    ref = torch.log_softmax(logits.masked_fill(~m2, -float("inf")), -1).gather(1, a[:, None]).squeeze(1)
    torch.testing.assert_close(lp, ref, rtol=1e-5, atol=1e-5)


def test_sampler_distribution(gpu):
    from ms_amd.rollout import sample_masked
    A = 16
    logits = torch.linspace(-2, 2, A, device=gpu).repeat(20000, 1)
    mask = torch.ones_like(logits, dtype=torch.bool)
    mask[:, 3] = False
    counts = torch.zeros(A, device=gpu)
    for c in range(10):
        a, _ = sample_masked(logits, mask, seed=9, counter=c)
        counts += torch.bincount(a, minlength=A).float()
    p = torch.softmax(logits[0].masked_fill(~mask[0], -float("inf")), -1)
    n = counts.sum()
    assert counts[3] == 0
    exp = p * n
    chi2 = float((((counts - exp) ** 2) / exp.clamp_min(1e-9))[mask[0]].sum())
    assert chi2 < 45.0, chi2  # 14 dof; p ~ 5e-5


def test_collect_rollout_replays_through_oracle(gpu):
    from ms_amd import EnvConfig, VecMinesweeper
    from ms_amd.models import build_model
    from ms_amd.rollout import collect_rollout
    H, W, K, N, T = 9, 9, 10, 256, 24
    vec = VecMinesweeper(N, EnvConfig(H=H, W=W, mine_count=K), seed=3)
    torch.manual_seed(0)
    model = build_model("cnn_residual", obs_shape=(10, H, W),
                        model_cfg=dict(stem_channels=16, blocks=1, dropout=0.0, value_hidden=16)).to(gpu).eval()
    buf, aux = collect_rollout(vec, model, T, gpu, aux_mine_weight=0.05, amp_dtype=None)
    o = O.OracleVec(H, W, K, N, seed=3)
    obs0, _ = o.reset()
    assert np.array_equal(buf.obs[:N].cpu().numpy(), obs0)
    acts = buf.actions.view(T, N).cpu().numpy()
    for t in range(T):
        lab, val = o.labels()
        assert np.array_equal(buf.mine_labels[t * N:(t + 1) * N].cpu().numpy(), lab), t
        assert np.array_equal(buf.mine_valid[t * N:(t + 1) * N].cpu().numpy(), val), t
        ref = o.step(acts[t])
        assert np.array_equal(buf.rewards[t * N:(t + 1) * N].cpu().numpy(), ref["reward"]), t
        assert np.array_equal(buf.dones[t * N:(t + 1) * N].cpu().numpy(), ref["done"]), t
        nxt = buf.obs[(t + 1) * N:(t + 2) * N] if t + 1 < T else aux["last_obs"]
        assert np.array_equal(nxt.cpu().numpy(), ref["obs"]), t
    # stored logp / values are the model's on the stored obs (fp32, eval mode)
    with torch.no_grad():
        lg, v = model(buf.obs)
    lp = torch.log_softmax(lg.masked_fill(~buf.action_mask, -1e9), -1).gather(1, buf.actions[:, None]).squeeze(1)
    torch.testing.assert_close(buf.logp, lp, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(buf.values, v, rtol=1e-4, atol=1e-4)
    assert bool(buf.action_mask.gather(1, buf.actions[:, None]).all())


@pytest.mark.parametrize("amp", ["fp16", "bf16"])
def test_trainer_update_runs(gpu, amp):
    """Trainer updates under the default fp16 autocast + GradScaler (the reference's) and
    under bf16: finite stats, parameters move. A GradScaler step skipped for overflow (its
    scale then halves) is the reference's behaviour too, so 4 updates leave room for it."""
    from ms_amd.train import Trainer, load_config
    import os
    cfg, env_d, model_d, extras = load_config(os.path.join(ROOT, "configs", "16x16x40_medium.yaml"))
    cfg.num_envs, cfg.steps_per_env, cfg.total_updates = 256, 8, 4
    model_d = dict(model_d, stem_channels=32, blocks=2, value_hidden=32)
    tr = Trainer(cfg, env_d, model_d, extras, seed=0, device=gpu, amp=amp)
    assert (tr.scaler is not None) == (amp == "fp16")
    before = [p.detach().clone() for p in tr.model.parameters()]
    for u in range(4):
        st = tr.update(u)
        assert all(np.isfinite(v) for v in st.values()), st
        assert {"loss", "policy_loss", "value_loss", "entropy", "aux_bce", "aux_calib"} <= set(st)
    assert any(not torch.equal(a, b) for a, b in zip(before, tr.model.parameters()))
