"""Data-parallel PPO update over torch.distributed (gloo, world_size 2, CPU):
two ranks holding halves of a minibatch must produce the same parameters as
one process updating on the whole minibatch (flat-gradient all-reduce, global
pos_weight / valid-count for the belief loss)."""
from __future__ import annotations

import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, PKG_DIR, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make(z):
    from ms_amd.models import build_model
    m = build_model("cnn_residual", obs_shape=(10, 8, 8),
                    model_cfg=dict(stem_channels=16, blocks=2, dropout=0.0, value_hidden=32))
    m.load_state_dict({k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w::")})
    return m


def _batch(z, sl):
    from ms_amd.buffers import Batch
    t = lambda k: torch.from_numpy(z[k][sl].copy())  # noqa: E731
    return Batch(obs=t("obs"), action_mask=t("mask"), actions=t("actions"), old_logp=t("old_logp"),
                 values=t("values"), advantages=t("advantages"), returns=t("returns"),
                 mine_labels=t("mine_labels"), mine_valid=t("mine_valid"))


def _worker(rank, world, port, out_dir):
    import sys
    sys.path[:0] = [PKG_DIR, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from ms_amd.ppo import FlatGrads, PPOConfig, ppo_update
    z = np.load(os.path.join(GOLDEN, "ppo.npz"))
    m = _make(z)
    fg = FlatGrads(m.parameters())
    opt = torch.optim.AdamW(m.parameters(), lr=3e-4)
    n = z["obs"].shape[0] // world
    cfg = PPOConfig(ent_coef=0.003, aux_mine_weight=0.05, aux_mine_calib_weight=0.01)
    for _ in range(2):
        ppo_update(m, opt, _batch(z, slice(rank * n, (rank + 1) * n)), cfg, amp_dtype=None,
                   group=dist.group.WORLD, flat_grads=fg)
    torch.save({k: v.clone() for k, v in m.state_dict().items()}, os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_two_rank_update_equals_single_process(tmp_path):
    from ms_amd.ppo import PPOConfig, ppo_update
    z = np.load(os.path.join(GOLDEN, "ppo.npz"))
    m = _make(z)
    opt = torch.optim.AdamW(m.parameters(), lr=3e-4)
    cfg = PPOConfig(ent_coef=0.003, aux_mine_weight=0.05, aux_mine_calib_weight=0.01)
    for _ in range(2):
        ppo_update(m, opt, _batch(z, slice(None)), cfg, amp_dtype=None)
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    for k, v in m.state_dict().items():
        assert torch.equal(r0[k], r1[k]), k  # ranks stay in lockstep
        if k == "policy_head.2.bias":
            # log-softmax is shift invariant: this gradient is 0 in exact arithmetic, so
            # AdamW turns rounding noise into +-lr steps; only bound it by the step size
            assert float((r0[k] - v).abs().max()) <= 2 * 3e-4 * 2
            continue
        # the all-reduce sums in another order than one process; AdamW's per-element
        # normalisation magnifies that rounding on near-zero gradients (<= 0.07 * lr)
        np.testing.assert_allclose(r0[k].numpy(), v.numpy(), rtol=2e-5, atol=2e-5, err_msg=k)
