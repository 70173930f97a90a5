"""End-to-end trainer CLI (ms_amd.train, the train_rl.py entry point): updates, quick
eval + best checkpoint, final eval, and the reference's run-directory layout
(train_rl.py:623-630, 667-783): ckpt_{latest,best,final}.pt, train_metrics.csv,
summary.json."""
from __future__ import annotations

import csv
import json
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = """
env: {H: 9, W: 9, mine_count: 10}
model: {name: cnn_residual, stem_channels: 96, blocks: 1, dropout: 0.05, value_hidden: 32}
ppo: {num_envs: 64, steps_per_env: 8, mini_batches: 2, ppo_epochs: 1, total_updates: 3, lr: 0.0003,
      aux_mine_weight: 0.05, aux_mine_calib_weight: 0.01}
training: {early_stop_patience: 100}
"""


def test_train_cli_run_directory(gpu, tmp_path):
    from ms_amd.train import main
    cfg = tmp_path / "c.yaml"
    cfg.write_text(CFG)
    out = tmp_path / "run"
    main(["--config", str(cfg), "--out", str(out), "--save_every", "1", "--quick_eval_interval", "1",
          "--eval_quick_episodes", "16", "--quick_eval_pairs", "1", "--eval_episodes", "16", "--eval_num_envs", "8"])
    for f in ("ckpt_latest.pt", "ckpt_best.pt", "ckpt_final.pt", "train_metrics.csv", "summary.json"):
        assert (out / f).exists(), f
    rows = list(csv.DictReader(open(out / "train_metrics.csv")))
    assert len(rows) == 3 and all(r["quick_win_rate"] != "" for r in rows)
    s = json.load(open(out / "summary.json"))
    assert s["best_update"] >= 1 and s["metrics_raw"]["episodes"] == 16.0
    assert 0.0 <= s["metrics_raw"]["win_rate"] <= 1.0
    st = torch.load(out / "ckpt_best.pt", weights_only=True)
    assert set(st) == {"model", "cfg", "model_meta", "metric"}
    assert st["model_meta"]["name"] == "cnn_residual"
