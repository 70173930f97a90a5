"""Generate tests/golden/sched.npz: the entropy-coefficient and belief-loss-weight
schedules of the REFERENCE update loop (train_rl.py:515-541), read back from the
``ent_coef`` / ``aux_weight`` columns of the train_metrics.csv that the
reference's own train_rl.py writes (train_rl.py:604-613, 699-709).

Run in the build container only (the reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_sched_golden.py

Each case runs ``python /root/reference/train_rl.py`` on a tiny CPU problem
(4x4 board, 2 envs x 2 steps, a 16-channel one-block model) so only the
schedules matter. The fixture stores the YAML text of each case and the
per-update values; nothing of the reference's source is copied.
"""
from __future__ import annotations

import csv
import os
import subprocess
import sys
import tempfile

import numpy as np
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

BASE = {
    "env": {"H": 4, "W": 4, "mine_count": 2, "guarantee_safe_neighborhood": True},
    "model": {"name": "cnn_residual", "stem_channels": 16, "blocks": 1, "dropout": 0.0, "value_hidden": 8},
    "ppo": {"num_envs": 2, "steps_per_env": 2, "mini_batches": 1, "ppo_epochs": 1, "lr": 0.0003},
}

# (name, total_updates, ppo overrides, training section)
CASES = [
    ("shipped_like", 30, {"ent_coef": 0.003, "ent_coef_min": 0.001, "ent_decay_updates": 12,
                          "aux_mine_weight": 0.05, "aux_mine_calib_weight": 0.01}, {}),
    ("aux_warmup_decay", 30, {"ent_coef": 0.01, "ent_coef_min": 0.002, "ent_decay_updates": 50,
                              "aux_mine_weight": 0.1},
     {"aux_mine_warmup_weight": 0.2, "aux_mine_final_weight": 0.01, "aux_mine_warmup_updates": 5,
      "aux_mine_decay_power": 2.0}),
    ("aux_sqrt_no_warmup", 25, {"ent_coef": 0.004, "aux_mine_weight": 0.0},
     {"aux_mine_final_weight": 0.3, "aux_mine_decay_power": 0.5}),
    ("aux_off", 12, {"ent_coef": 0.002, "ent_coef_min": 0.0, "ent_decay_updates": 1, "aux_mine_weight": 0.0}, {}),
    ("aux_rise_bad_power", 20, {"aux_mine_weight": 0.02},
     {"aux_mine_warmup_weight": 0.0, "aux_mine_final_weight": 0.08, "aux_mine_warmup_updates": 3,
      "aux_mine_decay_power": "not-a-number"}),
]


def main():
    names, yamls, ent, aux = [], [], [], []
    for name, total, ppo, training in CASES:
        cfg = {k: dict(v) for k, v in BASE.items()}
        cfg["ppo"].update(ppo, total_updates=total)
        if training:
            cfg["training"] = dict(training)
        text = yaml.safe_dump(cfg, sort_keys=True)
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "cfg.yaml")
            with open(path, "w") as f:
                f.write(text)
            out = os.path.join(td, "run")
            env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", PYTHONPATH=REF, CUDA_VISIBLE_DEVICES="")
            subprocess.run([sys.executable, os.path.join(REF, "train_rl.py"), "--config", path, "--out", out,
                            "--quick_eval_interval", "0", "--skip_final_eval", "--save_every", "100000"],
                           check=True, env=env, cwd=td, stdout=subprocess.DEVNULL)
            with open(os.path.join(out, "train_metrics.csv")) as f:
                rows = list(csv.DictReader(f))
        assert len(rows) == total, (name, len(rows))
        names.append(name)
        yamls.append(text)
        ent.append(np.array([float(r["ent_coef"]) for r in rows]))
        aux.append(np.array([float(r["aux_weight"]) for r in rows]))
        print(name, "ent", ent[-1][:3], "aux", aux[-1][:3])
    arrays = {"names": np.array(names), "yaml": np.array(yamls)}
    for i in range(len(names)):
        arrays[f"ent_{i}"] = ent[i]
        arrays[f"aux_{i}"] = aux[i]
    np.savez(os.path.join(HERE, "sched.npz"), **arrays)


if __name__ == "__main__":
    main()
