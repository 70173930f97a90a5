"""Update-loop schedules against the reference: the entropy
coefficient and belief-loss weight per update, as the reference's train_rl.py
wrote them to train_metrics.csv for five YAML configurations
(tests/golden/sched.npz, made by tests/golden/gen_sched_golden.py;
train_rl.py:456-541). Also the early-stop patience rule (train_rl.py:462-470)."""
from __future__ import annotations

import os
import tempfile

import pytest

from conftest import golden


def _cases():
    z = golden("sched.npz")
    return [(str(z["names"][i]), str(z["yaml"][i]), z[f"ent_{i}"], z[f"aux_{i}"]) for i in range(len(z["names"]))]


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c[0])
def test_schedules_match_reference(case):
    from ms_amd.train import aux_schedule_params, aux_weight_at, ent_coef_at, load_config
    name, text, ent_ref, aux_ref = case
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "cfg.yaml")
        with open(path, "w") as f:
            f.write(text)
        cfg, _, _, extras = load_config(path)
    params = aux_schedule_params(cfg, extras.get("training", {}))
    assert cfg.total_updates == len(ent_ref) == len(aux_ref)
    for u in range(cfg.total_updates):
        assert ent_coef_at(cfg, u) == ent_ref[u], (name, u)
        assert aux_weight_at(u, cfg.total_updates, *params) == aux_ref[u], (name, u)


@pytest.mark.parametrize("v,want", [(None, None), (0, None), (-3, None), ("x", None), (400, 400), ("25", 25)])
def test_early_stop_patience(v, want):
    from ms_amd.train import early_stop_patience
    assert early_stop_patience({} if v is None else {"early_stop_patience": v}) == want
