"""ppo_update parity (CPU, fp32, dropout 0, no scaler) against one update of
the reference's ppo_update captured in tests/golden/ppo.npz."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import golden


def _batch(z):
    from ms_amd.buffers import Batch
    t = lambda k: torch.from_numpy(z[k])  # noqa: E731
    return Batch(obs=t("obs"), action_mask=t("mask"), actions=t("actions"), old_logp=t("old_logp"),
                 values=t("values"), advantages=t("advantages"), returns=t("returns"),
                 mine_labels=t("mine_labels"), mine_valid=t("mine_valid"))


def test_ppo_update_matches_reference_golden():
    from ms_amd.models import build_model
    from ms_amd.ppo import PPOConfig, ppo_update
    torch.set_float32_matmul_precision("highest")
    z = golden("ppo.npz")
    m = build_model("cnn_residual", obs_shape=(10, 8, 8),
                    model_cfg=dict(stem_channels=16, blocks=2, dropout=0.0, value_hidden=32))
    m.load_state_dict({k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w::")})
    opt = torch.optim.AdamW(m.parameters(), lr=3e-4)
    cfg = PPOConfig(ent_coef=0.003, aux_mine_weight=0.05, aux_mine_calib_weight=0.01)
    stats = ppo_update(m, opt, _batch(z), cfg, scaler=None, amp_dtype=None)
    ref = dict(zip(z["stat_names"].tolist(), z["stat_values"].tolist()))
    assert set(stats) == set(ref)
    for k in ref:
        assert stats[k] == pytest.approx(ref[k], rel=1e-5, abs=1e-6), k
    for k, v in m.state_dict().items():
        np.testing.assert_allclose(v.numpy(), z["post::" + k], rtol=1e-5, atol=1e-6, err_msg=k)


def test_ppo_losses_no_aux_when_weights_zero():
    from ms_amd.models import build_model
    from ms_amd.ppo import PPOConfig, ppo_losses
    z = golden("ppo.npz")
    m = build_model("cnn_residual", obs_shape=(10, 8, 8),
                    model_cfg=dict(stem_channels=16, blocks=2, dropout=0.0, value_hidden=32))
    out = ppo_losses(m, _batch(z), PPOConfig(), amp_dtype=None)
    assert set(out) == {"loss", "policy_loss", "value_loss", "entropy"}


def test_empty_valid_set_gives_zero_aux():
    from ms_amd.models import build_model
    from ms_amd.ppo import PPOConfig, ppo_losses
    z = golden("ppo.npz")
    b = _batch(z)
    b.mine_valid = torch.zeros_like(b.mine_valid)
    m = build_model("cnn_residual", obs_shape=(10, 8, 8),
                    model_cfg=dict(stem_channels=16, blocks=2, dropout=0.0, value_hidden=32))
    out = ppo_losses(m, b, PPOConfig(aux_mine_weight=0.05, aux_mine_calib_weight=0.01), amp_dtype=None)
    assert float(out["aux_bce"]) == 0.0 and float(out["aux_calib"]) == 0.0


def test_flat_grads_leave_unused_mine_head_alone():
    """Both belief weights 0: the mine head gets no gradient, so (as after the reference's
    zero_grad(set_to_none=True), ppo.py:96) AdamW must not touch it -- no weight decay, no
    stale-moment step -- across several updates; FlatGrads must give the same parameters as
    the per-tensor path."""
    from ms_amd.models import build_model
    from ms_amd.ppo import FlatGrads, PPOConfig, ppo_update
    torch.set_float32_matmul_precision("highest")
    z = golden("ppo.npz")
    runs = []
    for use_flat in (False, True):
        m = build_model("cnn_residual", obs_shape=(10, 8, 8),
                        model_cfg=dict(stem_channels=16, blocks=2, dropout=0.0, value_hidden=32))
        m.load_state_dict({k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w::")})
        opt = torch.optim.AdamW(m.parameters(), lr=3e-4)
        fg = FlatGrads(m.parameters()) if use_flat else None
        # one update with the belief losses on (mine-head moments become non-zero), then two off
        for w in (0.05, 0.0, 0.0):
            cfg = PPOConfig(ent_coef=0.003, aux_mine_weight=w, aux_mine_calib_weight=0.0)
            if w == 0.0:
                before = {k: v.clone() for k, v in m.state_dict().items() if k.startswith("mine_head")}
            ppo_update(m, opt, _batch(z), cfg, scaler=None, amp_dtype=None, flat_grads=fg)
        for k, v in before.items():
            assert torch.equal(m.state_dict()[k], v), k
        runs.append({k: v.clone() for k, v in m.state_dict().items()})
    for k in runs[0]:
        torch.testing.assert_close(runs[1][k], runs[0][k], rtol=1e-6, atol=1e-7, msg=k)
