"""Recompute every env-step roofline fraction of a bench.py JSON line from the rocprofv3
kernel trace of the SAME run (tools/profile_round.sh step 1), so the committed fractions
can be checked against profiles/.

    python tools/trace_check.py --trace DIR --line bench_line_n1.json --out trace_check.json

k_step: mean dispatch duration of the config's grid (one 64-lane wave per env: grid
threads = 64 * envs; k_step_packed, four boards per wave, is keyed the same way) -> algorithmic bytes / duration. k_run: the config's dispatches
minus the first (the untimed warm-up launch), summed and divided by the timed steps (the
multistep record's timed_steps: bench.py times max(--steps, --min-timed-steps) of them).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("--trace", required=True)
ap.add_argument("--line", required=True)
ap.add_argument("--out", required=True)
a = ap.parse_args()

files = glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True)
if not files:
    raise SystemExit(f"no kernel_trace.csv under {a.trace}")
rows = []
for f in files:
    for r in csv.DictReader(open(f)):
        rows.append(r)


def grid_threads(r):
    for k in ("Grid_Size_X", "Grid_Size", "grid_size_x"):
        if k in r and r[k]:
            return int(r[k])
    raise SystemExit(f"no grid size column in {list(r)}")


disp = defaultdict(list)  # (kernel tag, board, grid threads) -> [(start, dur_ns)]
for r in rows:
    name = r["Kernel_Name"]
    # k_step_packed / k_run_packed (four small boards per wave) are k_step / k_run of 9x9 / 8x8
    for tag, pat in (("k_step", "k_step<"), ("k_step", "k_step_packed<"), ("k_run", "k_run<"),
                     ("k_run", "k_run_packed<")):
        if pat in name:
            board = name.split(pat, 1)[1].split(">", 1)[0].split(",")[:2]
            g = grid_threads(r)
            if pat in ("k_step_packed<", "k_run_packed<"):
                g *= 4  # 16 boards per 256-thread workgroup -> the same key as 64 lanes per board
            key = (tag, f"{int(board[0])}x{int(board[1])}", g)
            disp[key].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))

line = json.loads(open(a.line).read())
pts = [line] + list(line.get("north_star_points", []))
out = []
for p in pts:
    board = p.get("board") or p["config"]["board"]
    n = p.get("envs_per_gpu") or p["config"]["envs_per_gpu"]
    hw = "x".join(board.split("x")[:2])
    grid = 64 * n
    rl = p["roofline"]
    per_launch = rl["algo_bytes_per_launch"]
    # the headline / point runs first in bench.py; later dispatches of the same grid belong to
    # other phases (the PPO rollout), so keep only the config's own
    # (warm-up + K graph steps + K dispatch-timed eager steps)
    ks = sorted(disp.get(("k_step", hw, grid), []))[:line["warmup"] + 2 * line["steps"]]  # warm-up, timed graph, span graph
    rec = {"board": board, "envs_per_gpu": n}
    if ks:
        dur = sum(d for _, d in ks) / len(ks) / 1e6  # ms
        rec["k_step"] = {"dispatches": len(ks), "trace_mean_ms": dur, "line_kernel_ms": rl["kernel_ms"],
                         "trace_frac": per_launch / (dur * 1e-3) / 1e9 / rl["peak"], "line_frac": rl["frac"]}
        rec["k_step"]["ratio_line_over_trace"] = rec["k_step"]["line_frac"] / rec["k_step"]["trace_frac"]
    ms = p.get("multistep")
    kr = sorted(disp.get(("k_run", hw, grid), []))
    if ms and len(kr) > 1:
        timed = kr[1:]
        steps = ms.get("timed_steps", line["steps"])
        per_step_ms = sum(d for _, d in timed) / steps / 1e6
        mrl = ms["roofline"]
        tf = per_launch / (per_step_ms * 1e-3) / 1e9 / mrl["peak"]
        rec["k_run"] = {"dispatches_timed": len(timed), "trace_ms_per_step": per_step_ms,
                        "line_kernel_ms_per_step": mrl["kernel_ms_per_step"], "trace_frac": tf,
                        "line_frac": mrl["frac"], "ratio_line_over_trace": mrl["frac"] / tf}
    out.append(rec)
json.dump({"trace": a.trace, "line": a.line, "points": out}, open(a.out, "w"), indent=1)
for r in out:
    print(r["board"], r["envs_per_gpu"], {k: round(v["ratio_line_over_trace"], 3) for k, v in r.items()
                                          if isinstance(v, dict)})
