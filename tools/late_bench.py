"""Cost of late-start resets on the tape + step loop: the shared generator (k_late, one serial
wave over the step's done envs in env order, as the reference's single generator requires) and
the keyed mode (k_late_keyed, one wave per resetting env, all at once; include/msenv.h).

    python tools/late_bench.py [--envs 4096] [--steps 200]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))

import torch  # noqa: E402

from ms_amd import EnvConfig, VecMinesweeper  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=4096)
ap.add_argument("--steps", type=int, default=200)
a = ap.parse_args()
dev = torch.device("cuda:0")
cfg = EnvConfig(H=16, W=16, mine_count=40)
cases = [("no late start", None)]
for rng in ("shared", "keyed"):
    for p in (0.5, 1.0):
        cases.append((f"{rng} late start p={p}, 20-120 hidden", dict(prob=p, min_hidden=20, max_hidden=120, rng=rng)))
for name, late in cases:
    v = VecMinesweeper(a.envs, cfg, seed=0, late_start_cfg=late, late_start_seed=1, device=dev)
    v.reset()
    dones = 0
    for t in range(20):
        v.step(v.tape_actions(t, 0))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(a.steps):
        _, _, d, _ = v.step(v.tape_actions(20 + t, 0))
        dones += d
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / a.steps
    print(f"{name:40s}: {el * 1e6:7.1f} us/step (eager tape + step), "
          f"{a.envs / el / 1e6:7.1f} M env-steps/s, {float(dones.sum()) / a.steps:6.1f} resets/step", flush=True)
