"""G7: evaluation fixtures from the REFERENCE (eval.py:54-90, 265-511).

    PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_eval_golden.py

Writes tests/golden/eval_metrics.npz (AUROC / ECE inputs and the reference's outputs)
and eval_vec_*.npz (the reference evaluate_vec run with tests/eval_model.DetModel on
CPU: its metric dict). Data only; the tests never import the reference."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import eval as ref_eval  # noqa: E402  (the reference's eval.py, via PYTHONPATH)
from minesweeper.env import EnvConfig  # noqa: E402

from eval_model import DetModel, RuleModel  # noqa: E402

rng = np.random.default_rng(7)
d = {}
for i, n in enumerate((50, 1000, 20000)):
    labels = (rng.random(n) < 0.2).astype(np.float32)
    scores = (rng.random(n) * 0.6 + 0.4 * labels).astype(np.float32)
    d[f"labels{i}"], d[f"scores{i}"] = labels, scores
    d[f"auroc{i}"] = np.float64(ref_eval._compute_auroc(labels, scores))
    d[f"ece{i}"] = np.float64(ref_eval._compute_ece(scores, labels))
np.savez(os.path.join(HERE, "eval_metrics.npz"), **d)

for (H, W, K, eps, ne) in ((8, 8, 4, 30, 7), (9, 9, 10, 24, 8), (16, 16, 40, 12, 5)):
    torch.manual_seed(0)
    m = DetModel()
    res = ref_eval.evaluate_vec(m, EnvConfig(H=H, W=W, mine_count=K), episodes=eps, seed=0, num_envs=ne)
    keys = sorted(res)
    np.savez(os.path.join(HERE, f"eval_vec_{H}x{W}x{K}.npz"), keys=np.array(keys),
             values=np.array([res[k] for k in keys], dtype=np.float64), episodes=eps, num_envs=ne)
    print(H, W, K, {k: res[k] for k in ("win_rate", "avg_steps", "avg_progress", "belief_auroc", "belief_ece")})

# RuleModel fixtures: enough episodes to include wins at 16x16x40 and at C5's 30x16x99, so
# win accounting and the belief AUROC check run at the benchmark shapes
for (H, W, K, eps, ne) in ((16, 16, 40, 96, 16), (30, 16, 99, 96, 16)):
    m = RuleModel()
    res = ref_eval.evaluate_vec(m, EnvConfig(H=H, W=W, mine_count=K), episodes=eps, seed=0, num_envs=ne)
    keys = sorted(res)
    np.savez(os.path.join(HERE, f"eval_vec_rule_{H}x{W}x{K}.npz"), keys=np.array(keys),
             values=np.array([res[k] for k in keys], dtype=np.float64), episodes=eps, num_envs=ne)
    print("rule", H, W, K, {k: res[k] for k in ("wins", "win_rate", "avg_steps", "belief_auroc", "belief_ece")})
