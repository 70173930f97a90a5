"""Diagnostic: per-phase in-kernel cycle stamps of k_step (libmsenv_diag.so).

Phases (stamps 0..5): 0->1 loads, 1->2 placement, 2->3 flood fill,
3->4 reduce+aux+state store, 4->5 obs/mask emit. Stamps 6/7 = s_memrealtime
(100 MHz, chip-wide) at wave start/end, for the launch spread.
Run: python tools/diag_step.py [--envs N] [--board 16x16x40] [--tape 0]
"""
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
ap.add_argument("--board", default="16x16x40")
ap.add_argument("--tape", type=int, default=0)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--debug-flags", type=int, default=0, help="MS_DBG_* (4: k_step instead of k_step_packed)")
args = ap.parse_args()
H, W, K = (int(x) for x in args.board.split("x"))
# k_step_packed runs (ms_step picks it for 9x9 / 8x8 with 1 <= K <= 16 unless flag 4 is set)
packed = not (args.debug_flags & 4) and H <= 16 and H * W <= 128 and 1 <= K <= 16 and W in (8, 9)
from ms_amd import EnvConfig, VecMinesweeper, _lib as L  # noqa: E402

v = VecMinesweeper(args.envs, EnvConfig(H=H, W=W, mine_count=K), seed=0)
stamps = torch.zeros((args.envs, 16), dtype=torch.int64, device="cuda")
if args.debug_flags:
    v.set_debug_flags(args.debug_flags)
v.reset()
for t in range(30):
    v.step(v.tape_actions(t, args.tape))
L.check(v._lib.ms_set_diag(v._h, stamps.data_ptr()))
rows = []
for t in range(30, 30 + args.steps):
    a = v.tape_actions(t, args.tape)
    stamps.zero_()
    torch.cuda.synchronize()
    v.step(a)
    torch.cuda.synchronize()
    rows.append(stamps.cpu().numpy().copy())
S = np.concatenate(rows)
ph = np.diff(S[:, :6], axis=1).astype(np.float64)
names = ["loads", "placement", "flood", "reduce+store", "obs"]
print(f"board {args.board} envs {args.envs} tape {args.tape} flags {args.debug_flags}: cycles per phase (s_memtime ticks)")
for i, n in enumerate(names):
    col = ph[:, i]
    print(f"  {n:14s} mean {col.mean():9.0f}  p50 {np.median(col):9.0f}  p99 {np.percentile(col, 99):9.0f}  max {col.max():9.0f}")
tot = S[:, 5] - S[:, 0]
print(f"  {'total':14s} mean {tot.mean():9.0f}  p50 {np.median(tot):9.0f}  p99 {np.percentile(tot, 99):9.0f}  max {tot.max():9.0f}")
# placement sub-phases (slots 8..13; 14 = fixpoint rounds) of the boards that placed this step
pl = (S[:, 13] > S[:, 8]) if not packed else np.zeros(len(S), bool)
ppl = (S[:, 13] > S[:, 15]) & (S[:, 15] > 0) if packed else np.zeros(len(S), bool)
if ppl.any():
    P_ = S[ppl].astype(np.float64)
    print(f"  packed placement sub-phases over {ppl.sum()} placements (of {len(S)} board steps):")
    for n, (a0, a1) in (("jump+lemire", (15, 10)), ("t+dup", (10, 11)), ("chain", (11, 12)), ("rows+state", (12, 13))):
        d = P_[:, a1] - P_[:, a0]
        print(f"    {n:16s} mean {d.mean():8.0f}  p50 {np.median(d):8.0f}  p99 {np.percentile(d, 99):8.0f}")
if pl.any():
    P_ = S[pl]
    sub = np.diff(P_[:, 8:14], axis=1).astype(np.float64)
    sn = ["jump-ahead", "lemire", "candidates+clear", "fixpoint", "rows+state"]
    print(f"  placement sub-phases over {pl.sum()} placements (of {len(S)} board steps):")
    for i, n in enumerate(sn):
        print(f"    {n:16s} mean {sub[:, i].mean():8.0f}  p50 {np.median(sub[:, i]):8.0f}  p99 {np.percentile(sub[:, i], 99):8.0f}")
    print(f"    fixpoint rounds mean {P_[:, 14].mean():.2f} max {P_[:, 14].max()}")
    pt = (P_[:, 2] - P_[:, 1]).astype(np.float64)
    print(f"    whole placement phase of placing boards: mean {pt.mean():.0f} p50 {np.median(pt):.0f} p99 {np.percentile(pt, 99):.0f}")
# k_step_packed: obs sub-phases (slot 8 = image written, 9 = obs copied out, 5 = end)
pk = (S[:, 9] > S[:, 8]) & (S[:, 8] > 0) if packed else np.zeros(len(S), bool)
if pk.any():
    P_ = S[pk].astype(np.float64)
    for n, (a0, a1) in (("codes+image", (4, 8)), ("copy-out", (8, 9)), ("mask+state", (9, 5))):
        d = P_[:, a1] - P_[:, a0]
        print(f"  obs sub-phase {n:12s} mean {d.mean():8.0f}  p50 {np.median(d):8.0f}  p99 {np.percentile(d, 99):8.0f}")
# realtime (100 MHz): spread of wave starts/ends within one launch
for k in range(args.steps):
    blk = rows[k]
    st, en = blk[:, 6], blk[:, 7]
    if k < 3:
        print(f"  step {k}: wave start spread {(st.max()-st.min())/100:.2f} us, end spread "
              f"{(en.max()-st.min())/100:.2f} us (first start -> last end), mean wave "
              f"{(en-st).mean()/100:.2f} us")
