"""Same-process A/B of the Trainer's update loop (bench.py's PPO line: configs/16x16x40_medium.yaml,
4096 envs, T = 64, 3 x 8 minibatches, fp16 + GradScaler): AdamW as torch's fused kernel (the
Trainer's default) against the foreach implementation, alternated R rounds of U timed updates.
    python tools/ppo_ab.py [--rounds 3] [--updates 3]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--updates", type=int, default=3)
args = ap.parse_args()
import torch  # noqa: E402
from torch.optim import AdamW  # noqa: E402
from ms_amd.train import Trainer, load_config  # noqa: E402

dev = torch.device("cuda")
cfg, env_d, model_d, extras = load_config(os.path.join(ROOT, "configs", "16x16x40_medium.yaml"))
cfg.num_envs, cfg.steps_per_env, cfg.total_updates = 4096, 64, 4000
tr = Trainer(cfg, env_d, model_d, extras, seed=0, amp="fp16", device=dev)
opts = {"fused": tr.opt, "foreach": AdamW(tr.model.parameters(), lr=cfg.lr, foreach=True)}
u = 0
tr.update(u)
u += 1
torch.cuda.synchronize()
for r in range(args.rounds):
    for name, opt in opts.items():
        tr.opt = opt
        tr.update(u)  # warm-up of this optimizer's state
        u += 1
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.updates):
            tr.update(u)
            u += 1
        torch.cuda.synchronize()
        print(f"round {r} {name}: {(time.perf_counter() - t0) / args.updates:.4f} s per update", flush=True)
