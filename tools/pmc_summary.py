"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (counter_collection.csv)
into the per-launch HBM traffic json bench.py reads (profiles/<round>/pmc_*.json).

    python tools/pmc_summary.py --fetch DIR --write DIR --kernel k_step --out FILE.json \
        [--config "16x16x40, 4096 envs, tape 0"] [--algo-bytes N]

FETCH_SIZE / WRITE_SIZE are in KB per dispatch (summed over the TCC instances by
rocprofv3). MI355X_MICROARCH.md: FETCH_SIZE reports half of a wide 16-B/lane
streaming read on gfx950; k_step's reads are small scattered state loads, so its
FETCH_SIZE is taken as reported (noted in the json)."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(lambda: defaultdict(float))  # kernel -> dispatch -> value
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            per[r["Kernel_Name"]][r.get("Dispatch_Id", r.get("Correlation_Id"))] += float(r["Counter_Value"])
    return per


ap = argparse.ArgumentParser()
ap.add_argument("--fetch", required=True)
ap.add_argument("--write", required=True)
ap.add_argument("--kernel", default="k_step")
ap.add_argument("--out", required=True)
ap.add_argument("--config", default="16x16x40, 4096 envs, tape 0")
ap.add_argument("--algo-bytes", type=int, default=4096 * 10729)
ap.add_argument("--command", default="")
ap.add_argument("--steps-per-launch", type=int, default=1, help="env steps one launch performs (k_run: S)")
ap.add_argument("--bench-log", default=None,
                help="log of the profiled bench.py run: its JSON line gives k_run's steps per launch")
ap.add_argument("--fetch-wide", action="store_true",
                help="double FETCH_SIZE (gfx950 reports half of 16-B/lane streaming reads)")
a = ap.parse_args()
if a.bench_log:
    line = [x for x in open(a.bench_log).read().splitlines() if x.startswith("{")][-1]
    ms = json.loads(line).get("multistep")
    if a.kernel == "k_run" and ms:
        a.steps_per_launch = int(ms["roofline"]["steps_per_launch"])
        a.algo_bytes = a.algo_bytes * a.steps_per_launch
fe, wr = load(a.fetch, "FETCH_SIZE"), load(a.write, "WRITE_SIZE")
allk = {}
for k in sorted(set(fe) | set(wr)):
    fv, wv = list(fe.get(k, {}).values()), list(wr.get(k, {}).values())
    allk[k] = {"FETCH_SIZE_KB_mean": sum(fv) / max(1, len(fv)), "WRITE_SIZE_KB_mean": sum(wv) / max(1, len(wv)),
               "dispatches": max(len(fv), len(wv))}
name = next(k for k in allk if a.kernel in k)
fb = allk[name]["FETCH_SIZE_KB_mean"] * 1024 * (2 if a.fetch_wide else 1)
wb = allk[name]["WRITE_SIZE_KB_mean"] * 1024
out = {"command": a.command, "kernel": name, "config": a.config, "fetch_bytes_per_launch": fb,
       "write_bytes_per_launch": wb, "traffic_bytes_per_launch": fb + wb,
       "algorithmic_bytes_per_launch": a.algo_bytes, "steps_per_launch": a.steps_per_launch,
       "traffic_bytes_per_step": (fb + wb) / a.steps_per_launch,
       "note": ("FETCH_SIZE doubled (16-B/lane streaming reads, MI355X_MICROARCH.md HBM note)" if a.fetch_wide else
                "FETCH_SIZE taken as reported (small scattered state loads, not 16-B/lane streams)")
               + "; WRITE_SIZE exact for 16-B/lane stores",
       "all_kernels": allk}
json.dump(out, open(a.out, "w"), indent=1)
print(json.dumps({k: out[k] for k in ("kernel", "traffic_bytes_per_launch", "algorithmic_bytes_per_launch")}))
