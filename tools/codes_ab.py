"""Same-process A/B of the Trainer's rollout-buffer layout: u8 cell codes (obs_codes=True, the
default) against the f32 one-hot buffer, at bench.py's PPO configuration (16x16x40 medium,
4096 envs x 64 steps, 3 x 8 minibatches, fp16). python tools/codes_ab.py [--reps 3]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
import torch  # noqa: E402
from ms_amd.train import Trainer, load_config  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--updates", type=int, default=2)
args = ap.parse_args()
dev = torch.device("cuda:0")
trs = {}
for codes in (False, True):
    cfg, env_d, model_d, extras = load_config(os.path.join(ROOT, "configs", "16x16x40_medium.yaml"))
    cfg.num_envs, cfg.steps_per_env, cfg.total_updates = 4096, 64, 4000
    trs[codes] = Trainer(cfg, env_d, model_d, extras, seed=0, amp="fp16", device=dev, obs_codes=codes)
    trs[codes].update(0)
torch.cuda.synchronize()
for rep in range(args.reps):
    for codes in (False, True):
        tr = trs[codes]
        ph = []
        t0 = time.perf_counter()
        for u in range(args.updates):
            ph.append(tr.update(1 + rep * args.updates + u, profile=True))
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / args.updates
        ro = sum(p["rollout_s"] for p in ph) / len(ph)
        pp = sum(p["ppo_s"] for p in ph) / len(ph)
        print(f"{'codes' if codes else 'f32  '} {el:.4f} s/update (rollout {ro:.4f}, ppo {pp:.4f}) "
              f"buffer obs {tr.buffer.obs.numel() * tr.buffer.obs.element_size() / 1e9:.3f} GB", flush=True)
