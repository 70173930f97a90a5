"""Cost of late-start resets on the tape + step loop: the shared generator (k_late, one serial
wave over the step's done envs in env order, as the reference's single generator requires) and
the keyed mode (k_late_keyed, one wave per resetting env, all at once; include/msenv.h).

Every case is timed the way bench.py times the env step: after a warm-up of every case, S steps
(ms_tape_actions + ms_step, outputs preallocated) are captured in one HIP graph and replayed R
times between two events; the resets per step are counted in an eager pass afterwards.

    python tools/late_bench.py [--envs 4096] [--steps 50] [--replays 4]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))

import torch  # noqa: E402

from ms_amd import EnvConfig, VecMinesweeper  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=4096)
ap.add_argument("--steps", type=int, default=50)
ap.add_argument("--replays", type=int, default=4)
a = ap.parse_args()
dev = torch.device("cuda:0")
cfg = EnvConfig(H=16, W=16, mine_count=40)
cases = [("no late start", None)]
for rng in ("shared", "keyed"):
    for p in (0.5, 1.0):
        cases.append((f"{rng} late start p={p}, 20-120 hidden", dict(prob=p, min_hidden=20, max_hidden=120, rng=rng)))


def make(late):
    v = VecMinesweeper(a.envs, cfg, seed=0, late_start_cfg=late, late_start_seed=1, device=dev)
    v.reset()
    n, A = a.envs, 256
    out = {"obs": torch.empty((n, 10, 16, 16), device=dev), "action_mask": torch.empty((n, A), dtype=torch.bool, device=dev),
           "rewards": torch.empty(n, device=dev), "dones": torch.empty(n, dtype=torch.bool, device=dev)}
    act = torch.empty(n, dtype=torch.int64, device=dev)
    return v, out, act


def run(v, out, act, t0, steps):
    for t in range(steps):
        v.tape_actions(t0 + t, 0, out=act)
        v.step(act, out=out)


for _ in range(2):  # warm-up: every kernel of every case loaded and run
    for _, late in cases:
        v, out, act = make(late)
        run(v, out, act, 0, 5)
torch.cuda.synchronize()
for name, late in cases:
    v, out, act = make(late)
    run(v, out, act, 0, 20)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        run(v, out, act, 20, 2)  # side-stream warm-up before capture
        with torch.cuda.graph(g, stream=s):
            run(v, out, act, 22, a.steps)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.replays):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    el = e0.elapsed_time(e1) / 1e3 / (a.replays * a.steps)
    resets = 0
    for t in range(20):
        v.tape_actions(1000 + t, 0, out=act)
        v.step(act, out=out)
        resets += int(out["dones"].sum())
    print(f"{name:40s}: {el * 1e6:8.1f} us/step (graph: tape + step), {a.envs / el / 1e6:8.2f} M env-steps/s, "
          f"{resets / 20:6.1f} resets/step, {el * 1e6 / max(resets / 20, 1e-9):6.2f} us per reset", flush=True)
