"""Per-dispatch timeline of the headline env step (k_tape -> k_step pairs) from a
rocprofv3 kernel trace: kernel durations and the idle gaps between them.

    python tools/step_gaps.py --trace DIR [--grid-envs 4096]
"""
import argparse
import csv
import glob
import os
import statistics as st

ap = argparse.ArgumentParser()
ap.add_argument("--trace", required=True)
ap.add_argument("--grid-envs", type=int, default=4096)
a = ap.parse_args()
rows = []
for f in glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ev = []
for r in rows:
    name, gx = r["Kernel_Name"], int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
    if "k_tape<16, 16>" in name and gx >= a.grid_envs and gx < 2 * a.grid_envs:
        ev.append(("tape", int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    elif "k_step<16, 16" in name and gx == 64 * a.grid_envs:
        ev.append(("step", int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
tape_d, step_d, gap_ts, gap_st, period = [], [], [], [], []
for i in range(1, len(ev) - 1):
    k, s, e = ev[i]
    if k == "tape" and ev[i + 1][0] == "step":
        tape_d.append(e - s)
        step_d.append(ev[i + 1][2] - ev[i + 1][1])
        gap_ts.append(ev[i + 1][1] - e)
        if ev[i - 1][0] == "step":
            gap_st.append(s - ev[i - 1][2])
            period.append(ev[i + 1][2] - ev[i - 1][2])
med = lambda v: st.median(v) / 1e3 if v else float("nan")  # noqa: E731
print(f"pairs {len(tape_d)}: k_tape {med(tape_d):.2f} us, gap tape->step {med(gap_ts):.2f} us, "
      f"k_step {med(step_d):.2f} us, gap step->tape {med(gap_st):.2f} us, period {med(period):.2f} us (medians)")
