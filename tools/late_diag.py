"""Where the reference-exact (shared-generator) late start spends its cycles: k_late's in-kernel
accounting (libmsenv_diag.so, MS_DIAG), summed over one launch per step, per reset.
    python tools/late_diag.py [--envs 4096] [--prob 0.5] [--steps 10]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MSENV_LIB"] = os.path.join(ROOT, "minesweeper-ppo_amd", "libmsenv_diag.so")
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=4096)
ap.add_argument("--prob", type=float, default=0.5)
ap.add_argument("--steps", type=int, default=10)
args = ap.parse_args()
from ms_amd import EnvConfig, VecMinesweeper, _lib as L  # noqa: E402

late = dict(prob=args.prob, min_hidden=20, max_hidden=120, rng="shared")
v = VecMinesweeper(args.envs, EnvConfig(H=16, W=16, mine_count=40), seed=0, late_start_cfg=late, late_start_seed=1)
v.reset()
for t in range(20):
    v.step(v.tape_actions(t, 0))
stamps = torch.zeros((args.envs, 16), dtype=torch.int64, device="cuda")
L.check(v._lib.ms_set_diag(v._h, stamps.data_ptr()))
tot = np.zeros(16)
for t in range(20, 20 + args.steps):
    a = v.tape_actions(t, 0)
    stamps.zero_()
    torch.cuda.synchronize()
    v.step(a)
    torch.cuda.synchronize()
    tot += stamps[0].cpu().numpy().astype(np.float64)
n = max(tot[1], 1)
print(f"16x16x40, {args.envs} envs, p = {args.prob}, {args.steps} steps: {tot[1] / args.steps:.0f} resets/step, "
      f"{tot[2] / args.steps:.0f} late starts/step, {tot[10] / max(tot[2], 1):.2f} attempts per late start")
print(f"k_late cycles per step {tot[0] / args.steps:.0f}, per reset {tot[0] / n:.0f}")
names = {3: "no late start (draw, stores, emit)", 4: "first clicks (placement)", 5: "extra-click loops",
         9: "late envs' stores + emit"}
for k, name in names.items():
    print(f"  {name:40s} {tot[k] / n:8.0f} cycles per reset ({tot[k] / max(tot[0], 1) * 100:5.1f} %)")
print(f"  extra clicks per late start {tot[6] / max(tot[2], 1):.1f}, flood fills {tot[7] / max(tot[2], 1):.1f}, "
      f"flood iterations per fill {tot[8] / max(tot[7], 1):.1f}, loop cycles per click {tot[5] / max(tot[6], 1):.0f}")
print(f"  flood clicks: {tot[15] / max(tot[7], 1):.0f} cycles draw + select, {tot[14] / max(tot[7], 1):.0f} cycles fill + list")
